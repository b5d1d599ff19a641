# round 5, session ab: k_stage's steps in flight per lane (experiment builds libfu_su2 /
# libfu_su8, -DFU_STAGE_U=2 / 8, against 4) under the non-temporal stores: ER-1M kernel 8
# (rounds 1-19) three alternations, R-MAT-24 kernel 9 one; bitwise checks of each build.
set -o pipefail
O=gpurun_out/ab
mkdir -p $O
export TMPDIR=/tmp
L=simgrid-flow-updating-implementation_amd/fu
for lib in libfu_su2 libfu_su8; do
  timeout -k 10 300 env FU_LIBRARY=$PWD/$L/$lib.so python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "er_vs_c_oracle or ca_sync_fixture_bitwise or headline_window or pregather_multi" > $O/pytest_$lib.log 2>&1 || exit $?
done
for i in 1 2 3; do
  for lib in libfu libfu_su2 libfu_su8; do
    timeout -k 10 200 env FU_LIBRARY=$PWD/$L/$lib.so python tools/sweep.py er:n=1000000,m=4000000 --variants=stage_nopack --warm=1 --timed=19 --reps=5 > $O/sweep_er_${lib}_$i.log 2>&1 || exit $?
  done
done
for lib in libfu libfu_su2 libfu_su8; do
  timeout -k 10 300 env FU_LIBRARY=$PWD/$L/$lib.so python tools/sweep.py rmat:scale=24,ef=16 --variants=deg_np_pre --warm=3 --timed=20 --reps=3 > $O/sweep_rmat_${lib}_1.log 2>&1 || exit $?
done
exit 0

# round 5, session s: non-temporal index loads (experiment builds): libfu_colnt (k_stage's
# column offsets, ER and R-MAT), libfu_sidxnt (k_round_staged's staged indices, ER),
# libfu_posnt (k_transpose's positions, R-MAT). Bitwise checks, then ER-1M kernel 8 (rounds
# 1-19) three alternations and R-MAT-24 kernel 9 two alternations against the default build.
set -o pipefail
O=gpurun_out/s
mkdir -p $O
export TMPDIR=/tmp
L=simgrid-flow-updating-implementation_amd/fu
for lib in libfu_colnt libfu_sidxnt libfu_posnt; do
  timeout -k 10 300 env FU_LIBRARY=$PWD/$L/$lib.so python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "er_vs_c_oracle or ca_sync_fixture_bitwise or headline_window or pregather_multi" > $O/pytest_$lib.log 2>&1 || exit $?
done
for i in 1 2 3; do
  for lib in libfu libfu_colnt libfu_sidxnt; do
    timeout -k 10 200 env FU_LIBRARY=$PWD/$L/$lib.so python tools/sweep.py er:n=1000000,m=4000000 --variants=stage_nopack --warm=1 --timed=19 --reps=5 > $O/sweep_er_${lib}_$i.log 2>&1 || exit $?
  done
done
for i in 1 2; do
  for lib in libfu libfu_colnt libfu_posnt; do
    timeout -k 10 300 env FU_LIBRARY=$PWD/$L/$lib.so python tools/sweep.py rmat:scale=24,ef=16 --variants=deg_np_pre --warm=3 --timed=20 --reps=3 > $O/sweep_rmat_${lib}_$i.log 2>&1 || exit $?
  done
done
exit 0

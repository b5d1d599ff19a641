# round 5, session o: the non-temporal G stores of k_stage (libfu_stnt, -DFU_STAGE_NT), the
# screen's best in session n: ER-1M kernel 8 (rounds 1-19 unpacked) five more alternations
# with the default build, R-MAT-24 kernel 9 (the same stores write G_A) two alternations, and
# the kernel-9 bitwise tests on the variant.
set -o pipefail
O=gpurun_out/o
mkdir -p $O
export TMPDIR=/tmp
L=simgrid-flow-updating-implementation_amd/fu
timeout -k 10 400 env FU_LIBRARY=$PWD/$L/libfu_stnt.so python -u -m pytest -s -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "pregather or rmat24 or dist_kernel9 or isolated_rows" > $O/pytest_stnt.log 2>&1 || exit $?
for i in 1 2 3 4 5; do
  for lib in libfu libfu_stnt; do
    timeout -k 10 200 env FU_LIBRARY=$PWD/$L/$lib.so python tools/sweep.py er:n=1000000,m=4000000 --variants=stage_nopack --warm=1 --timed=19 --reps=5 > $O/sweep_er_${lib}_$i.log 2>&1 || exit $?
  done
done
for i in 1 2; do
  for lib in libfu libfu_stnt; do
    timeout -k 10 300 env FU_LIBRARY=$PWD/$L/$lib.so python tools/sweep.py rmat:scale=24,ef=16 --variants=deg_np_pre --warm=3 --timed=20 --reps=3 > $O/sweep_rmat_${lib}_$i.log 2>&1 || exit $?
  done
done
exit 0

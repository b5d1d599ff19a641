# round 5, session f: kernel 8's light tile geometry, 512 x 64 (experiment build libfu_st512,
# -DFU_STAGE_TE=512 -DFU_STAGE_TN=64) against the 1024 x 128 default on ER-1M: bitwise check
# of the variant, then tools/sweep.py (kernel 8, rounds after 1 warm round, unpacked) in
# separate processes, alternating three times.
set -o pipefail
O=gpurun_out/f
mkdir -p $O
export TMPDIR=/tmp
L=simgrid-flow-updating-implementation_amd/fu
timeout -k 10 300 env FU_LIBRARY=$PWD/$L/libfu_st512.so python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "er_vs_c_oracle and stage or ca_sync_fixture_bitwise and stage" > $O/pytest_st512.log 2>&1 || exit $?
for i in 1 2 3; do
  for lib in libfu libfu_st512; do
    timeout -k 10 200 env FU_LIBRARY=$PWD/$L/$lib.so python tools/sweep.py er:n=1000000,m=4000000 --variants=stage_nopack --warm=1 --timed=19 --reps=5 > $O/sweep_${lib}_$i.log 2>&1 || exit $?
  done
done

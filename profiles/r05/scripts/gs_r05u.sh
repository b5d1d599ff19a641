# round 5, session u: kernel 9's transposes with plain G_A loads and non-temporal G_B stores
# (libfu_trld0, -DFU_TR_NTLOAD=0) against the default (both non-temporal): R-MAT-24, three
# alternations; bitwise kernel-9 tests on the variant.
set -o pipefail
O=gpurun_out/u
mkdir -p $O
export TMPDIR=/tmp
L=simgrid-flow-updating-implementation_amd/fu
timeout -k 10 300 env FU_LIBRARY=$PWD/$L/libfu_trld0.so python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "pregather_multi or ca_sync_fixture_bitwise and pregather" > $O/pytest_trld0.log 2>&1 || exit $?
for i in 1 2 3; do
  for lib in libfu libfu_trld0; do
    timeout -k 10 300 env FU_LIBRARY=$PWD/$L/$lib.so python tools/sweep.py rmat:scale=24,ef=16 --variants=deg_np_pre --warm=3 --timed=20 --reps=3 > $O/sweep_rmat_${lib}_$i.log 2>&1 || exit $?
  done
done
exit 0

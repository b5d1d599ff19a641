# round 5, session af: kernel 8's stage for 1-byte codes as k_stage<64 KB> with two blocks per
# CU (experiment build libfu_nar2, -DFU_STAGE_NARROW=2: the 1-byte layout's Q doubled, 63
# VGPRs) against the default: bitwise tests through every packing width, then BASELINE
# config 2 as written (bench.py defaults, 1000 rounds) three alternations.
set -o pipefail
O=gpurun_out/af
mkdir -p $O
export TMPDIR=/tmp
L=simgrid-flow-updating-implementation_amd/fu
timeout -k 10 400 env FU_LIBRARY=$PWD/$L/libfu_nar2.so python -u -m pytest -s -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "config2_as_written or headline_window or pack or stage" > $O/pytest_nar2.log 2>&1 || exit $?
for i in 1 2 3; do
  for lib in libfu libfu_nar2; do
    timeout -k 10 300 env FU_LIBRARY=$PWD/$L/$lib.so python bench.py --no-unit --no-conv --cpu-seconds 0 > $O/bench_default_${lib}_$i.log 2>&1 || exit $?
  done
done
exit 0

# round 5, session r: k_stage's store hint by element width, BASELINE config 2 as written
# (bench.py defaults: ER-1M, 1000 rounds, phases per 100 rounds through the 32/16/8-bit
# widths): libfu (non-temporal for doubles only, write-back for packed codes), libfu_st0
# (write-back always), libfu_st2 (non-temporal always), alternating processes three times.
set -o pipefail
O=gpurun_out/r
mkdir -p $O
export TMPDIR=/tmp
L=simgrid-flow-updating-implementation_amd/fu
timeout -k 10 300 python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "config2_as_written or headline_window or packed" > $O/pytest.log 2>&1 || exit $?
for i in 1 2 3; do
  for lib in libfu libfu_st0 libfu_st2; do
    timeout -k 10 300 env FU_LIBRARY=$PWD/$L/$lib.so python bench.py --no-unit --no-conv --cpu-seconds 0 > $O/bench_default_${lib}_$i.log 2>&1 || exit $?
  done
done
exit 0

# round 6, session k: split-plane flows (16-bit low pieces written alone once converged):
# the whole GPU suite on the new library, then the driver's command alternating the new
# library and the session-j library (fu/libfu_base.so, built from commit f27b78a).
set -o pipefail
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 600 python -u -m pytest -s -x -v --timeout 400 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || exit $?
B=simgrid-flow-updating-implementation_amd/fu/libfu_base.so
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-unit --cpu-seconds 0 > $O/bench_new_$i.log 2>&1 || exit $?
  FU_LIBRARY=$PWD/$B timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-unit --cpu-seconds 0 > $O/bench_base_$i.log 2>&1 || exit $?
done
exit 0

# round 6, session m: fu_reset drops an autotune pass left pending for a packing width (calls
# too short for a pass); the autotune / packing / window tests, then the driver's command twice.
set -o pipefail
O=gpurun_out/r06m
mkdir -p $O
timeout -k 10 600 python -u -m pytest -s -x -v --timeout 400 --timeout-method thread tests -m gpu -k "autotune or reset or packed or headline or marked or config2 or width" > $O/pytest.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd_$i.log 2>&1 || exit $?
done
exit 0

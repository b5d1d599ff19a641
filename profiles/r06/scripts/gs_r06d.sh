# round 6, session d: mark 0 of the one-call window taken from k_round0's own start event
# (hipExtLaunchKernel): the headline-window bitwise test, the window A/B, the driver's command.
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 300 python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests -m gpu -k "headline_window or config2_as_written or abi" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab_window.py --reps 10 > $O/ab_window.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd_1.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-unit > $O/bench_driver_cmd_2.log 2>&1 || exit $?
exit 0

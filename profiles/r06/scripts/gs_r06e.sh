# round 6, session e: round 0's marks from k_round0's own start / stop events, the window's
# host path warmed in bench.prepare: the marked-window and headline GPU tests, the window A/B,
# the driver's command three times.
set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 300 python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests -m gpu -k "marked_window or headline_window" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab_window.py --reps 10 > $O/ab_window.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd_1.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-unit > $O/bench_driver_cmd_2.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-unit > $O/bench_driver_cmd_3.log 2>&1 || exit $?
exit 0

# round 6, session b: the window marks created with the handle (no event creation inside the
# timed window): the driver's command twice, the headline window test, and a kernel trace of the
# driver's command.
set -o pipefail
O=gpurun_out/r06b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests -m gpu -k "headline_window or abi or marked" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd_1.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-unit > $O/bench_driver_cmd_2.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-unit --cpu-seconds 0 > $O/prof.log 2>&1 || exit $?
exit 0

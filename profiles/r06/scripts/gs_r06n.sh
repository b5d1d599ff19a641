# round 6, session n: the final tree after the reset fix: the whole GPU suite, smoke, the driver's command.
set -o pipefail
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 600 python -u -m pytest -s -x -v --timeout 400 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || exit $?
exit 0

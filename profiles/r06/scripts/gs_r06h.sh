# round 6, session h: the final tree (7-byte codes removed again): the whole GPU suite, smoke,
# the driver's command, and a kernel trace of the driver's command (window record).
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -s -x -v --timeout 400 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-unit --cpu-seconds 0 > $O/prof.log 2>&1 || exit $?
exit 0

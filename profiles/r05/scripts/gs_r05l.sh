# round 5, session l: the tree with every C ABI entry point exception-guarded and the new
# window tests: the GPU suite (capture off), smoke, the driver's command, a kernel trace of it.
set -o pipefail
O=gpurun_out/l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -s -x -v --durations=15 --timeout 400 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-unit > $O/prof_driver.log 2>&1 || exit $?
python3 tools/window_stats.py $O/prof_driver/run_kernel_trace.csv --n 1000000 --E 7999972 --kernel stage --steps 20 --which 1 --out $O/er1m_s20_window_stats.json > /dev/null
exit 0

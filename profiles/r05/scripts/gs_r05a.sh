# round 5, session a: the iso_rows fix, the host plans in fu_plan.cpp, the removed kernel-9
# options. The GPU suite with pytest's capture off (-s), so a HIP runtime message (a memory
# access fault) lands in the log; smoke; the driver's command (now with config2_1000,
# rmat24_unit, pairwise_unit); kernel traces of its window and of the R-MAT window, reduced
# by tools/window_stats.py.
set -o pipefail
O=gpurun_out/a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-unit > $O/prof_driver.log 2>&1 || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_rmat -o run -- python3 bench.py --workload rmat --steps 20 --warmup 5 --no-conv --cpu-seconds 0 > $O/prof_rmat.log 2>&1 || exit $?
python3 tools/window_stats.py $O/prof_driver/run_kernel_trace.csv --n 1000000 --E 7999972 --kernel stage --steps 20 --which 1 --out $O/er1m_s20_window_stats.json > /dev/null
python3 tools/window_stats.py $O/prof_rmat/run_kernel_trace.csv --n 16777216 --E 520761504 --kernel pregather --steps 20 --which 1 --out $O/rmat24_s20_window_stats.json > /dev/null
exit 0

# round 5, session a: the iso_rows fix and the removed kernel-9 options. The GPU suite with
# pytest's capture off (-s), so a HIP runtime message (a memory-access fault) lands in the log,
# smoke, the driver's command, its kernel trace (window stats), the R-MAT line.
set -o pipefail
O=gpurun_out/a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $O/prof_driver.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --workload rmat --steps 20 --warmup 5 --no-conv --cpu-seconds 0 > $O/bench_rmat.log 2>&1 || exit $?

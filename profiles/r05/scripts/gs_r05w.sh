# round 5, session w: the final tree (nt stage stores for doubles, plain transpose loads,
# fu_mem_info, build_rev's 2^31 guard): the GPU suite, smoke, the driver's command, the R-MAT
# window's kernel trace and PMC bytes (the tracked R-MAT records).
set -o pipefail
O=gpurun_out/w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -s -x -v --durations=15 --timeout 400 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_rmat -o run -- python3 bench.py --workload rmat --steps 20 --warmup 5 --no-conv --cpu-seconds 0 > $O/prof_rmat.log 2>&1 || exit $?
python3 tools/window_stats.py $O/prof_rmat/run_kernel_trace.csv --n 16777216 --E 520761504 --kernel pregather --steps 20 --which 1 --out $O/rmat24_s20_window_stats.json --dump $O/rmat24_s20_window_trace.csv > /dev/null
rm -rf gpurun_out/pmc
PMC_GROUPS="FETCH_SIZE WRITE_SIZE" TARGET_ARGS="--spec rmat:scale=24,ef=16 --layout degree --kernel pregather --warm 2 --rounds 20 --pack 0" bash tools/pmc.sh || exit $?
python3 tools/pmc_window.py gpurun_out/pmc 20 > $O/pmc_rmat24_pregather.json || exit $?
mv gpurun_out/pmc $O/pmc_rmat
exit 0

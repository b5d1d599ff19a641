# round 5, session e: the final tree: the driver's command twice (separate processes), its
# kernel trace and the R-MAT window's, reduced by tools/window_stats.py, the default
# bench.py (1000 rounds) and the RGG-64M strong line.
set -o pipefail
O=gpurun_out/e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $O/bench_driver_cmd_2.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-unit > $O/prof_driver.log 2>&1 || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_rmat -o run -- python3 bench.py --workload rmat --steps 20 --warmup 5 --no-conv --cpu-seconds 0 > $O/prof_rmat.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --no-unit --cpu-seconds 0 > $O/bench_default.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload rgg-dist --strong --steps 20 --warmup 5 --no-conv > $O/bench_rgg64m_strong.log 2>&1 || exit $?
python3 tools/window_stats.py $O/prof_driver/run_kernel_trace.csv --n 1000000 --E 7999972 --kernel stage --steps 20 --which 1 --out $O/er1m_s20_window_stats.json --dump $O/er1m_s20_window_trace.csv > /dev/null
python3 tools/window_stats.py $O/prof_rmat/run_kernel_trace.csv --n 16777216 --E 520761504 --kernel pregather --steps 20 --which 1 --out $O/rmat24_s20_window_stats.json --dump $O/rmat24_s20_window_trace.csv > /dev/null
exit 0

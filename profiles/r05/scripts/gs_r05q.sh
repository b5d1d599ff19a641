# round 5, session q: the final tree (non-temporal stage stores): the driver's command twice,
# the kernel traces of the ER and R-MAT windows (the tracked window records), the default
# bench.py (1000 rounds), and the PMC bytes of both windows (FETCH_SIZE / WRITE_SIZE passes,
# tools/pmc.sh; the records bench.py quotes as roofline.traffic).
set -o pipefail
O=gpurun_out/q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $O/bench_driver_cmd_2.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-unit > $O/prof_driver.log 2>&1 || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_rmat -o run -- python3 bench.py --workload rmat --steps 20 --warmup 5 --no-conv --cpu-seconds 0 > $O/prof_rmat.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --no-unit --cpu-seconds 0 > $O/bench_default.log 2>&1 || exit $?
python3 tools/window_stats.py $O/prof_driver/run_kernel_trace.csv --n 1000000 --E 7999972 --kernel stage --steps 20 --which 1 --out $O/er1m_s20_window_stats.json --dump $O/er1m_s20_window_trace.csv > /dev/null
python3 tools/window_stats.py $O/prof_rmat/run_kernel_trace.csv --n 16777216 --E 520761504 --kernel pregather --steps 20 --which 1 --out $O/rmat24_s20_window_stats.json --dump $O/rmat24_s20_window_trace.csv > /dev/null
rm -rf gpurun_out/pmc
PMC_GROUPS="FETCH_SIZE WRITE_SIZE" TARGET_ARGS="--spec er:n=1000000,m=4000000 --kernel stage --warm 2 --rounds 20 --pack 0" bash tools/pmc.sh || exit $?
python3 tools/pmc_window.py gpurun_out/pmc 20 > $O/pmc_er1m_stage.json || exit $?
mv gpurun_out/pmc $O/pmc_er
PMC_GROUPS="FETCH_SIZE WRITE_SIZE" TARGET_ARGS="--spec rmat:scale=24,ef=16 --layout degree --kernel pregather --warm 2 --rounds 20 --pack 0" bash tools/pmc.sh || exit $?
python3 tools/pmc_window.py gpurun_out/pmc 20 > $O/pmc_rmat24_pregather.json || exit $?
mv gpurun_out/pmc $O/pmc_rmat
exit 0

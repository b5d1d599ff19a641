# round 4, GPU session g: ER-1M with kernel 9 (G transposed into edge order: the tiles read it
# without indices) against kernel 8 on the same box: bench lines and PMC bytes per round
set -o pipefail
mkdir -p gpurun_out/er9
export TMPDIR=/tmp
# write -> read-back round trips against the Infinity Cache
timeout -k 10 120 tools/bin/ubench_mall > gpurun_out/er9/ubench_mall.log 2>&1 || exit $?
# the driver's command, and its kernel trace
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/er9/bench_driver_cmd.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/er9/prof_driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/er9/prof_driver.log 2>&1 || exit $?
for k in stage pregather stage pregather; do
  timeout -k 10 300 python bench.py --kernel $k --steps 20 --warmup 5 --cpu-seconds 0 --no-conv --no-unit >> gpurun_out/er9/bench_$k.log 2>&1 || exit $?
done
for k in stage pregather; do
  rm -rf gpurun_out/pmc
  PMC_GROUPS="FETCH_SIZE WRITE_SIZE" TARGET_ARGS="--kernel $k --warm 5 --rounds 20 --pack 0" bash tools/pmc.sh || exit $?
  python3 tools/pmc_window.py gpurun_out/pmc 20 > gpurun_out/er9/pmc_$k.json || exit $?
  mv gpurun_out/pmc gpurun_out/er9/pmc_$k
done
# R-MAT-24 with the round-4 defaults (lag on): PMC bytes per round by kernel
rm -rf gpurun_out/pmc
PMC_GROUPS="FETCH_SIZE WRITE_SIZE" TARGET_ARGS="--spec rmat:scale=24,ef=16 --layout degree --kernel pregather --warm 2 --rounds 20 --pack 0" bash tools/pmc.sh || exit $?
python3 tools/pmc_window.py gpurun_out/pmc 20 > gpurun_out/er9/pmc_rmat_lag.json || exit $?
mv gpurun_out/pmc gpurun_out/er9/pmc_rmat_lag

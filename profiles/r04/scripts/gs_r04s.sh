# round 4, GPU session s: the ER-1M driver window with kernel auto (after the autotune pass)
# against kernel 8 pinned, alternating on one box
set -o pipefail
mkdir -p gpurun_out/s
for i in 1 2 3; do
  for k in auto stage; do
    timeout -k 10 200 python bench.py --kernel $k --steps 20 --warmup 5 --cpu-seconds 0 --no-conv --no-unit >> gpurun_out/s/bench_$k.log 2>&1 || exit $?
  done
done

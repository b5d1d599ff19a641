# round 5, session ag: does the GPU need a longer warm period before the 20-round window?
# The driver's command (--warmup 5) against --warmup 400 (about 25 ms of rounds right before
# the window), alternating processes four times; rounds 1-19 device time from the line.
set -o pipefail
O=gpurun_out/ag
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3 4; do
  for w in 5 400; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup $w --no-unit --no-conv --cpu-seconds 0 > $O/bench_w${w}_$i.log 2>&1 || exit $?
  done
done
exit 0

# round 5, session ai: the settle's length: 25 ms (default) against 200 ms, the driver's
# command, alternating processes four times.
set -o pipefail
O=gpurun_out/ai
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-unit --no-conv --cpu-seconds 0 > $O/bench_settle25_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-unit --no-conv --cpu-seconds 0 --settle-ms 200 > $O/bench_settle200_$i.log 2>&1 || exit $?
done
exit 0

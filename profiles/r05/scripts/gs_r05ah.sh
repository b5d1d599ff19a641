# round 5, session ah: bench.prepare's settle (>= 25 ms of untimed rounds right before the
# window) against none (--settle-ms 0): the driver's command, alternating processes four
# times; then the driver's command as the driver runs it (companions included).
set -o pipefail
O=gpurun_out/ah
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-unit --no-conv --cpu-seconds 0 > $O/bench_settle25_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-unit --no-conv --cpu-seconds 0 --settle-ms 0 > $O/bench_settle0_$i.log 2>&1 || exit $?
done
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || exit $?
exit 0

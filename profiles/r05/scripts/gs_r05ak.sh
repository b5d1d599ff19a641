# round 5, session ak: the final tree's headline over eight processes on one box (the
# driver's command without the companions, which run after the window and do not touch it).
set -o pipefail
O=gpurun_out/ak
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-unit --no-conv --cpu-seconds 0 > $O/bench_$i.log 2>&1 || exit $?
done
exit 0

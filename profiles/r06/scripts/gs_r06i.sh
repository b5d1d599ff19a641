# round 6, session i: the final tree: the driver's command in six processes (the headline's
# spread), and the RGG 2^28 two-partition test (FU_BIG_GRAPH=1, 2.42e9 directed edges).
set -o pipefail
O=gpurun_out/r06i
mkdir -p $O
for i in 1 2 3 4 5 6; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-unit > $O/bench_$i.log 2>&1 || exit $?
done
FU_BIG_GRAPH=1 timeout -k 10 900 python -u -m pytest -s -x -v --timeout 850 --timeout-method thread tests -m gpu -k "2pow28" > $O/pytest_big.log 2>&1 || exit $?
exit 0

# round 5, session v: a graph beyond one handle's 2^31 directed edges on one GPU: RGG 2^28
# at degree 9 (2.4e9 directed edges) as two in-process partitions: bench.py --workload rgg-parts, then
# the bitwise test against the C oracle (FU_BIG_GRAPH=1).
set -o pipefail
O=gpurun_out/v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --workload rgg-parts --steps 20 --warmup 5 > $O/bench_rgg2p28_deg9_parts2.log 2>&1 || exit $?
FU_BIG_GRAPH=1 timeout -k 10 900 python -u -m pytest -s -x -v --timeout 1000 --timeout-method thread tests/test_gpu_parity.py -m gpu -k rgg_2pow28 > $O/pytest_big.log 2>&1 || exit $?
exit 0

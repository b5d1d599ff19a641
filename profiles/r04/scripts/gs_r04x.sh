# round 4, GPU session x: the README's other rows on the final tree: pairwise RR-64K
# (config 3) and RGG-64M on one GPU through the partitioned path (config 5's graph)
set -o pipefail
mkdir -p gpurun_out/x
timeout -k 10 300 python bench.py --workload pairwise --steps 400 --warmup 50 > gpurun_out/x/bench_pairwise.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --workload rgg-dist --strong --steps 20 --warmup 5 > gpurun_out/x/bench_rgg64m_strong.log 2>&1 || exit $?

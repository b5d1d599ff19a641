# round 4, GPU session u: a rank with no halo skips the comm-stream hop: the dist tests, then
# the one-rank RGG 2^23 line (before: ~11 us between rounds)
set -o pipefail
mkdir -p gpurun_out/u
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "dist or rccl" > gpurun_out/u/pytest.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload rgg-dist --steps 20 --warmup 5 > gpurun_out/u/bench_rggdist.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/u/prof_rggdist -o run -- python3 tools/prof_target.py --dist-rgg 8388608 --warm 5 --rounds 20 > gpurun_out/u/prof_rggdist.log 2>&1 || exit $?

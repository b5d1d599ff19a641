# round 4, GPU session v: the final tree: the GPU suite, smoke, the driver's command, the
# default bench (1000 rounds), the R-MAT line
set -o pipefail
mkdir -p gpurun_out/v
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/v/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/v/bench_driver_cmd.log 2>&1 || exit $?
timeout -k 10 500 python bench.py > gpurun_out/v/bench_default.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --workload rmat --steps 20 --warmup 5 > gpurun_out/v/bench_rmat.log 2>&1 || exit $?

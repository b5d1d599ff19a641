# round 4, final GPU session: tr_nt on by default: the GPU suite, smoke, the driver's command,
# the R-MAT line, and a kernel trace of the driver's command
set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/final/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --workload rmat --steps 20 --warmup 5 > gpurun_out/final/bench_rmat.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/bench_driver_cmd.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof_driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/final/prof_driver.log 2>&1 || exit $?

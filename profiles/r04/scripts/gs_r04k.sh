# round 4, GPU session k: kernel 9's isolated-row tiles as k_isolated (iso_rows): the GPU
# suite, the R-MAT-24 A/B, then the driver's command, the R-MAT line and a kernel trace
set -o pipefail
mkdir -p gpurun_out/k
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/k/pytest.log 2>&1 || exit $?
rm -rf gpurun_out/ab
AB_SPEC="rmat:scale=24,ef=16" AB_ARGS="--warm=3 --timed=20 --reps=3" AB_VARIANTS="deg_np_pre pre_iso0" AB_ROUNDS=3 bash tools/ab_proc.sh || exit $?
mv gpurun_out/ab gpurun_out/k/ab
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/k/bench_driver_cmd.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --workload rmat --steps 20 --warmup 5 > gpurun_out/k/bench_rmat.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k/prof_rmat -o run -- python3 tools/prof_target.py --spec rmat:scale=24,ef=16 --layout degree --kernel pregather --warm 2 --rounds 20 --pack 0 > gpurun_out/k/prof_rmat.log 2>&1 || exit $?

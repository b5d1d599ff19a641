# round 4, GPU session r: multi_short on by default: the GPU suite and smoke, the light/heavy
# threshold with it (hub_threshold 64 / 96), the R-MAT line and the driver's command
set -o pipefail
mkdir -p gpurun_out/r
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/r/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r/smoke.log 2>&1 || exit $?
rm -rf gpurun_out/ab
AB_SPEC="rmat:scale=24,ef=16" AB_ARGS="--warm=3 --timed=20 --reps=3" AB_VARIANTS="deg_np_pre pre_short_ht64 pre_short_ht96" AB_ROUNDS=2 bash tools/ab_proc.sh || exit $?
mv gpurun_out/ab gpurun_out/r/ab
timeout -k 10 500 python bench.py --workload rmat --steps 20 --warmup 5 > gpurun_out/r/bench_rmat.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r/bench_driver_cmd.log 2>&1 || exit $?

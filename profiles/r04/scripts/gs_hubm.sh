set -o pipefail
# (record of a measured session: hub_multi / hub_blocks were removed after it lost, so its
# variants naming them no longer exist in tools/sweep.py or the engine)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "multi_row_chains or dist or copy_bandwidth or lag" > gpurun_out/t_hubm.log 2>&1 || exit $?
AB_SPEC="rmat:scale=24,ef=16" AB_ARGS="--warm=3 --timed=20 --reps=3" AB_VARIANTS="deg_np_pre pre_hubmall pre_lag pre_lag_hubmall pre_hubm64k" AB_ROUNDS=2 bash tools/ab_proc.sh || exit $?
timeout -k 10 300 python bench.py --workload rgg-dist --steps 20 --warmup 5 --conv-rounds 200 > gpurun_out/b_rggdist.log 2>&1 && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-unit > gpurun_out/b_er.log 2>&1

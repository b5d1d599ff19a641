# round 4, GPU session d: hub chain waves at issue priority (hub_prio), with lag and hub_blocks
# (record of a measured session: hub_multi / hub_blocks were removed after it lost, so its
# variants naming them no longer exist in tools/sweep.py or the engine)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "multi_row_chains or lag" > gpurun_out/pytest_c.log 2>&1 || exit $?
rm -rf gpurun_out/ab
AB_SPEC="rmat:scale=24,ef=16" AB_ARGS="--warm=3 --timed=20 --reps=3" AB_VARIANTS="deg_np_pre pre_prio pre_prio_lag pre_hb256_prio pre_hb256_prio_lag" AB_ROUNDS=2 bash tools/ab_proc.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prmat_hb -o run -- python3 tools/prof_target.py --spec rmat:scale=24,ef=16 --layout degree --kernel pregather --warm 2 --rounds 20 --pack 0 --opt hub_prio=1 --opt lag=1 > gpurun_out/prmat_hb.log 2>&1

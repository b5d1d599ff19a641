# round 5, session b: R-MAT-24 kernel 9 with the hub path on CU-masked streams (hub_cus 16 /
# (the hub_cus option and its sweep variants were removed after this session: profiles/r05/b)
# 32 / 64 reserved CUs, lowest mask bits or spread, with the hot-estimate table tr_hot) against
# the defaults, process-separated (tools/ab_proc.sh: each variant alone in its own process),
# one alternation for the screen; then a bitwise check of the masked path.
set -o pipefail
export TMPDIR=/tmp
AB_SPEC="rmat:scale=24,ef=16" AB_ARGS="--warm=3 --timed=20 --reps=3" AB_ROUNDS=1 \
  AB_VARIANTS="deg_np_pre pre_hot_cu32 pre_hot_cu32s pre_hot_cu16s pre_hot_cu64s pre_cu32s pre_hot deg_np_pre pre_hot_cu16 pre_hot_cu64" \
  bash tools/ab_proc.sh || exit $?
mkdir -p gpurun_out/b
timeout -k 10 300 python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "hub_cus" > gpurun_out/b/pytest_hubcus.log 2>&1 || exit $?

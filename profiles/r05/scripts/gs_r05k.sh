# round 5, session k: the measured windows themselves bitwise: the headline through
# bench.prepare + bench.timed_rounds (and config2_1000's path), the pairwise unit's ticks
# 101-500 through fu_replay_run_timed.
set -o pipefail
O=gpurun_out/k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -s -x -v --durations=0 --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "headline_window_bitwise or pairwise_unit_window_bitwise" > $O/pytest.log 2>&1 || exit $?
exit 0

# round 5, session y: LV08's weighted link sharing and TCP window (fu_trace_build_links_ex,
# the drop-in Engine's default): the trace, platform and drop-in Engine GPU tests.
set -o pipefail
O=gpurun_out/y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests -m gpu -k "slow_platform or watcher_lines or replay or trace or cli" > $O/pytest.log 2>&1 || exit $?
exit 0

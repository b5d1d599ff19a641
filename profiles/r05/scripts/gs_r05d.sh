# round 5, session d: the tree after the option removals, the autotune plan refactor and kernel
# 9 on partitioned handles: the whole GPU suite (capture off) and smoke.
set -o pipefail
O=gpurun_out/d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -s -x -v --timeout 250 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?

# round 5, session z: stability of the final tree: the GPU suite twice in separate processes
# (capture off, so a fault message would reach the log), then the gated 2^28 test.
set -o pipefail
O=gpurun_out/z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -s -x -v --timeout 400 --timeout-method thread tests -m gpu > $O/pytest_1.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -s -x -v --timeout 400 --timeout-method thread tests -m gpu > $O/pytest_2.log 2>&1 || exit $?
FU_BIG_GRAPH=1 timeout -k 10 900 python -u -m pytest -s -x -v --timeout 1000 --timeout-method thread tests/test_gpu_parity.py -m gpu -k rgg_2pow28 > $O/pytest_big.log 2>&1 || exit $?
exit 0

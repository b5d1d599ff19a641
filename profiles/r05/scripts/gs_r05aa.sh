# round 5, session aa: RGG-64M (config 5's graph) bitwise against the C oracle: 10 rounds on
# the single-GPU engine, rounds 0-19 through the partitioned path at one rank.
set -o pipefail
O=gpurun_out/aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -s -x -v --durations=5 --timeout 900 --timeout-method thread tests/test_gpu_parity.py -m gpu -k rgg64m > $O/pytest.log 2>&1 || exit $?
exit 0

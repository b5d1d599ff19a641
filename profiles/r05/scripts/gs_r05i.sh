# round 5, session i: BASELINE config 2 as written, the whole 1000-round job bitwise against
# the C oracle (test_config2_as_written_1000_rounds_bitwise).
set -o pipefail
O=gpurun_out/i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -s -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "config2_as_written" > $O/pytest.log 2>&1 || exit $?
exit 0

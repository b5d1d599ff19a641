set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hub_scan.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
echo rc=$?
tail -5 gpurun_out/pytest.log

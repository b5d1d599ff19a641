# round 5, session ad: fu_mem_info on the GPU.
set -o pipefail
O=gpurun_out/ad
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k mem_info > $O/pytest.log 2>&1 || exit $?
exit 0

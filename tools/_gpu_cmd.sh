set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_hub_scan.py tests/test_relabel.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rmat or heavy or star or hub or fixture or degree" > gpurun_out/pytest.log 2>&1 && \
timeout -k 10 600 python -u tools/sweep.py rmat:scale=24,ef=16 --variants=recon_deg --warm=3 --timed=10 --reps=3 > gpurun_out/sweep_rmat24.log 2>&1 && \
timeout -k 10 300 python -u tools/sweep.py rmat:scale=20,ef=16 --variants=recon,recon_deg,recon_512 --warm=10 --timed=50 --reps=3 > gpurun_out/sweep_rmat.log 2>&1
echo rc=$?
tail -3 gpurun_out/pytest.log
python3 tools/show_sweep.py gpurun_out/sweep_rmat24.log
python3 tools/show_sweep.py gpurun_out/sweep_rmat.log

set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/sweep.py rgg:n=1000000,deg=8 --variants=recon,recon_512,recon_1024 --warm=400 > gpurun_out/sweep_rgg.log 2>&1 && \
timeout -k 10 400 python -u tools/sweep.py rmat:scale=20,ef=16 --variants=recon,recon_nofork,recon_512,recon_deg --warm=10 > gpurun_out/sweep_rmat.log 2>&1
echo rc=$?
tail -3 gpurun_out/pytest.log
python3 tools/show_sweep.py gpurun_out/sweep_rgg.log
python3 tools/show_sweep.py gpurun_out/sweep_rmat.log

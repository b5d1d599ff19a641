set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "rmat or heavy or star or hub or fixture or degree or bins" > gpurun_out/pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/sweep.py rmat:scale=20,ef=16 --variants=recon,recon_512,recon_1024 --warm=10 --timed=50 --reps=3 > gpurun_out/sweep_rmat.log 2>&1
echo rc=$?
tail -3 gpurun_out/pytest.log
python3 tools/show_sweep.py gpurun_out/sweep_rmat.log

set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/sweep.py rmat:scale=20,ef=16 --variants=recon,recon_deg,diag5_no_hub_chain,diag5_deg --warm=10 > gpurun_out/sweep_rmat.log 2>&1 && \
timeout -k 10 400 python -u bench.py --workload rmat --n 24 --layout degree --steps 10 --warmup 45 --no-conv --cpu-seconds 0 > gpurun_out/bench_rmat24_deg.log 2>&1 && \
timeout -k 10 400 python -u bench.py --workload rmat --n 24 --layout given --kernel recon --steps 10 --warmup 5 --no-conv --cpu-seconds 0 > gpurun_out/bench_rmat24.log 2>&1
echo rc=$?
python3 tools/show_sweep.py gpurun_out/sweep_rmat.log
tail -c 1200 gpurun_out/bench_rmat24_deg.log
tail -c 1200 gpurun_out/bench_rmat24.log

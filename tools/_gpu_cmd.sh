set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 200 --warmup 64 --no-conv > gpurun_out/bench_n2.log 2>&1
echo rc=$?
grep '^{' gpurun_out/bench_n2.log | cut -c1-400
tail -3 gpurun_out/bench_n2.log | cut -c1-300

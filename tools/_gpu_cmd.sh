set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --workload rmat --n 24 --steps 30 --warmup 64 --no-conv --cpu-seconds 0 > gpurun_out/bench_rmat24.log 2>&1
echo rc=$?
python3 -c "
import json,sys
l=[x for x in open('gpurun_out/bench_rmat24.log') if x.startswith('{')][-1]; d=json.loads(l)
print('%.4g' % d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('avg_launch_us'), d['config'].get('kernel_selected'), d['config'].get('tile_selected'), d['config']['autotune_us_per_round'])
"

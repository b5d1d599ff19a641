set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dist or autotune or rcc" > gpurun_out/pytest.log 2>&1 && \
timeout -k 10 400 python -u bench.py --workload rgg-dist --n 8388608 --steps 300 > gpurun_out/bench_rggdist.log 2>&1
echo rc=$?
tail -3 gpurun_out/pytest.log
for f in bench_rggdist; do python3 -c "
import json,sys
l=[x for x in open('gpurun_out/$f.log') if x.startswith('{')][-1]; d=json.loads(l)
print('$f', '%.4g' % d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('avg_launch_us'), d['config'].get('kernel_selected'), d['config'].get('tile_selected'), d['config'].get('E_directed'))
"; done

set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "autotune or dist or packed" > gpurun_out/pytest.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1
echo rc=$?
tail -3 gpurun_out/pytest.log
python3 -c "
import json,sys
l=[x for x in open('gpurun_out/bench.log') if x.startswith('{')][-1]; d=json.loads(l)
print('%.4g' % d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('avg_launch_us'), d['config'].get('kernel_selected'), d['config']['autotune_us_per_round'], d['config']['autotune_winner_by_width'])
"

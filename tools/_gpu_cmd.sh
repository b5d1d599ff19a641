set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
echo rc=$?
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench.log') if l.startswith('{')][-1]); print(d['value'], d['roofline']['frac'], d['cpu_baseline'])"

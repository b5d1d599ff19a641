set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/sweep.py --variants=stage,pipe_stage,pipe_stage_b4,pipe_stage_b3,pipe_stage_b2 --warm=400 > gpurun_out/sweep_b.log 2>&1
echo rc=$?
python3 tools/show_sweep.py gpurun_out/sweep_b.log

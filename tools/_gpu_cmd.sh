set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "stage or fixture or packed or autotune" > gpurun_out/pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/sweep.py --variants=stage,stage_u32 --warm=400 > gpurun_out/sweep_b.log 2>&1 && \
timeout -k 10 300 python -u tools/sweep.py --variants=stage,stage_u32 --warm=400 >> gpurun_out/sweep_b.log 2>&1 && \
timeout -k 10 300 python -u tools/sweep.py --variants=stage,stage_u32 --warm=20 --timed=20 --reps=3 > gpurun_out/sweep_c.log 2>&1
echo rc=$?
tail -3 gpurun_out/pytest.log
python3 tools/show_sweep.py gpurun_out/sweep_b.log
python3 tools/show_sweep.py gpurun_out/sweep_c.log

set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/sweep.py --variants=stage_nopack,recon_1024_nopack,recon_512_nopack,pipe_stage_nopack --warm=20 --timed=20 --reps=3 > gpurun_out/sweep_c.log 2>&1
echo rc=$?
python3 tools/show_sweep.py gpurun_out/sweep_c.log

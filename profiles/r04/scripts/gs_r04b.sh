# round 4, GPU session b: full GPU suite, R-MAT-24 A/B (lag, tr_hot), kernel trace of the
# winner candidate, PMC passes of the rgg-dist window
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/pytest_full.log 2>&1 || exit $?
AB_SPEC="rmat:scale=24,ef=16" AB_ARGS="--warm=3 --timed=20 --reps=3" AB_VARIANTS="deg_np_pre pre_lag pre_hot pre_hot_lag" AB_ROUNDS=2 bash tools/ab_proc.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prmat -o run -- python3 tools/prof_target.py --spec rmat:scale=24,ef=16 --layout degree --kernel pregather --warm 2 --rounds 20 --pack 0 --opt lag=1 --opt tr_hot=10240 > gpurun_out/prmat.log 2>&1 || exit $?
PMC_GROUPS="FETCH_SIZE WRITE_SIZE" TARGET_ARGS="--dist-rgg 8388608 --warm 5 --rounds 20" bash tools/pmc.sh || exit $?
python3 tools/pmc_window.py gpurun_out/pmc 20 > gpurun_out/pmc_rggdist_window.json

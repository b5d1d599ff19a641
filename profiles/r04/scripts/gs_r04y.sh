# round 4, GPU session y: non-temporal G_A loads / G_B stores in the transposes (tr_nt)
set -o pipefail
mkdir -p gpurun_out/y
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "multi_row_chains" > gpurun_out/y/pytest.log 2>&1 || exit $?
rm -rf gpurun_out/ab
AB_SPEC="rmat:scale=24,ef=16" AB_ARGS="--warm=3 --timed=20 --reps=3" AB_VARIANTS="deg_np_pre pre_trnt" AB_ROUNDS=3 bash tools/ab_proc.sh || exit $?
mv gpurun_out/ab gpurun_out/y/ab

# round 4, GPU session z: non-temporal G_A / G_B streams: transposes (tr_nt 1) and the stage's
# G_A stores as well (tr_nt 2)
set -o pipefail
mkdir -p gpurun_out/z
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "multi_row_chains or option_errors or rmat" > gpurun_out/z/pytest.log 2>&1 || exit $?
rm -rf gpurun_out/ab
AB_SPEC="rmat:scale=24,ef=16" AB_ARGS="--warm=3 --timed=20 --reps=3" AB_VARIANTS="deg_np_pre pre_trnt pre_trnt2" AB_ROUNDS=3 bash tools/ab_proc.sh || exit $?
mv gpurun_out/ab gpurun_out/z/ab

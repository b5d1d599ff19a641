# round 4, GPU session aa: the multi-row blocks' G_B loads non-temporal too (tr_nt 2): the
# (record of a measured session: tr_nt 2 was removed after it lost)
# kernel-9 parity tests first (a crash ends the session), then the R-MAT A/B against tr_nt 1
set -o pipefail
mkdir -p gpurun_out/aa
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "pregather or multi_row_chains or option_errors or lag or rmat" > gpurun_out/aa/pytest.log 2>&1 || exit $?
rm -rf gpurun_out/ab
AB_SPEC="rmat:scale=24,ef=16" AB_ARGS="--warm=3 --timed=20 --reps=3" AB_VARIANTS="deg_np_pre pre_trnt2" AB_ROUNDS=3 bash tools/ab_proc.sh || exit $?
mv gpurun_out/ab gpurun_out/aa/ab

# round 4, GPU session l: kernel 9's light tiles at 1024 x 256 (light_geo 2): parity, R-MAT-24 A/B
# (record of a measured session: option light_geo was removed after it lost)
set -o pipefail
mkdir -p gpurun_out/l
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "multi_row_chains or row_class or option_errors" > gpurun_out/l/pytest.log 2>&1 || exit $?
rm -rf gpurun_out/ab
AB_SPEC="rmat:scale=24,ef=16" AB_ARGS="--warm=3 --timed=20 --reps=3" AB_VARIANTS="deg_np_pre pre_lg2" AB_ROUNDS=3 bash tools/ab_proc.sh || exit $?
mv gpurun_out/ab gpurun_out/l/ab

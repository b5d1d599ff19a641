# round 4, GPU session i: fused rows, second form (isolated tail in k_isolated, rows of > 64
# (record of a measured session: option fuse was removed after it lost, profiles/r04/fuse/)
# edges on whole waves, unrolled short rows): parity, R-MAT-24 A/B, kernel traces
set -o pipefail
mkdir -p gpurun_out/i
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "fuse or row_class or multi_row_chains or option_errors or lag" > gpurun_out/i/pytest.log 2>&1 || exit $?
rm -rf gpurun_out/ab
AB_SPEC="rmat:scale=24,ef=16" AB_ARGS="--warm=3 --timed=20 --reps=3" AB_VARIANTS="deg_np_pre pre_fuse1 pre_fuse2 pre_fuse3" AB_ROUNDS=2 bash tools/ab_proc.sh || exit $?
mv gpurun_out/ab gpurun_out/i/ab
for m in 1 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/i/prof_fuse$m -o run -- python3 tools/prof_target.py --spec rmat:scale=24,ef=16 --layout degree --kernel pregather --warm 2 --rounds 20 --pack 0 --opt fuse=$m > gpurun_out/i/prof_fuse$m.log 2>&1 || exit $?
done

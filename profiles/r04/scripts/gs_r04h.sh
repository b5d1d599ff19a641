# round 4, GPU session h: kernel 9's fused rows (option fuse): GPU parity suite, then the
# (record of a measured session: option fuse was removed after it lost, profiles/r04/fuse/)
# R-MAT-24 A/B against the default, a kernel trace and PMC bytes of the best candidate
set -o pipefail
mkdir -p gpurun_out/h
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/h/pytest.log 2>&1 || exit $?
rm -rf gpurun_out/ab
AB_SPEC="rmat:scale=24,ef=16" AB_ARGS="--warm=3 --timed=20 --reps=3" AB_VARIANTS="deg_np_pre pre_fuse1 pre_fuse2 pre_fuse3 pre_fuse3_late" AB_ROUNDS=2 bash tools/ab_proc.sh || exit $?
mv gpurun_out/ab gpurun_out/h/ab
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/h/prof_fuse3 -o run -- python3 tools/prof_target.py --spec rmat:scale=24,ef=16 --layout degree --kernel pregather --warm 2 --rounds 20 --pack 0 --opt fuse=3 > gpurun_out/h/prof_fuse3.log 2>&1 || exit $?
rm -rf gpurun_out/pmc
PMC_GROUPS="FETCH_SIZE WRITE_SIZE" TARGET_ARGS="--spec rmat:scale=24,ef=16 --layout degree --kernel pregather --warm 2 --rounds 20 --pack 0 --opt fuse=3" bash tools/pmc.sh || exit $?
python3 tools/pmc_window.py gpurun_out/pmc 20 > gpurun_out/h/pmc_rmat_fuse3.json || exit $?
mv gpurun_out/pmc gpurun_out/h/pmc_fuse3

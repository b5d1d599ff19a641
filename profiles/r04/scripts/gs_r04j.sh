# round 4, GPU session j: where k_fused_rows' time goes (timing-only experiment builds):
# (record of a measured session: option fuse was removed after it lost, profiles/r04/fuse/)
# the default geometry, without the row phase (fzd1), 2048-edge buckets at four blocks per CU
# (fz2k, fz2kd1), one block per CU (fz1blk); kernel traces of fuse 1 on R-MAT-24
set -o pipefail
mkdir -p gpurun_out/j
export TMPDIR=/tmp
L=simgrid-flow-updating-implementation_amd/fu
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k "fuse or row_class" > gpurun_out/j/pytest.log 2>&1 || exit $?
FU_LIBRARY=$(pwd)/$L/libfu_fz2k.so timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k "fuse" > gpurun_out/j/pytest_fz2k.log 2>&1 || exit $?
for lib in libfu libfu_fzd1 libfu_fz2k libfu_fz2kd1 libfu_fz1blk; do
  export FU_LIBRARY=$(pwd)/$L/$lib.so
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/j/prof_$lib -o run -- python3 tools/prof_target.py --spec rmat:scale=24,ef=16 --layout degree --kernel pregather --warm 2 --rounds 10 --pack 0 --opt fuse=1 > gpurun_out/j/prof_$lib.log 2>&1 || exit $?
done
unset FU_LIBRARY

#!/bin/bash
# rocprofv3 kernel traces of R-MAT-24 kernel 9 variants (product and timing-only ablations,
# from the -DFU_DIAG library: make DIAG=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export FU_LIBRARY=$PWD/simgrid-flow-updating-implementation_amd/fu/libfu_diag.so
for v in ${RMAT_VARIANTS:-deg_np_pre pre_d5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prmat/$v -o run -- \
    python3 tools/sweep.py rmat:scale=24,ef=16 --variants=$v --warm=3 --timed=4 --reps=1 > gpurun_out/prmat_$v.log 2>&1 || exit $?
done

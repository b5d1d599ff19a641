#!/bin/bash
# RGG 2^23 (one GPU, kernel 4 at 1024x128): kernel trace, then FETCH_SIZE / WRITE_SIZE passes
# (tools/pmc.sh) over 20 rounds from the zero state.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--spec rgg:n=8388608,deg=8 --kernel recon --tile 1024 --warm 5 --rounds 20 --pack 0 ${RGG_EXTRA:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prgg -o run -- python3 tools/prof_target.py $ARGS > gpurun_out/prgg.log 2>&1 || exit $?
PMC_GROUPS="FETCH_SIZE WRITE_SIZE" TARGET_ARGS="$ARGS" bash tools/pmc.sh

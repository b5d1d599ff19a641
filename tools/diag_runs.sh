#!/bin/bash
# Timing-only ablations (libfu_diag.so, results WRONG by design): one rocprofv3 kernel-stats
# run of tools/prof_target.py per DIAG value. DIAGS="0 1 5" TARGET_ARGS="..." bash tools/diag_runs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/diag
mkdir -p "$OUT"
export TMPDIR=/tmp FU_LIBRARY=$(pwd)/simgrid-flow-updating-implementation_amd/fu/libfu_diag.so
for d in ${DIAGS:-0 1 5}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/d$d" -o run -- python3 tools/prof_target.py --diag $d ${TARGET_ARGS:-} > "$OUT/d$d.log" 2>&1
  rc=$?
  echo "diag $d rc=$rc" >> "$OUT/status.txt"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/d$d.log"; exit $rc; fi
done

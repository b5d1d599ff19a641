#!/bin/bash
# PMC passes (one rocprofv3 run per counter group; no trace domains) on tools/prof_target.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
i=0
for grp in ${PMC_GROUPS:-"FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES"}; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 tools/prof_target.py ${TARGET_ARGS:-} > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i [$grp] rc=$rc" >> "$OUT/status.txt"
  if [ $rc -ne 0 ]; then exit $rc; fi
done

#!/bin/bash
# PMC passes (one rocprofv3 run per counter group; no trace domains): the calibration
# program (known byte counts per access width) and tools/prof_target.py (the bench's timed
# region). Summarise with tools/pmc_summary.py. A group of several counters: "A:B:C".
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
i=0
for grp in ${PMC_GROUPS:-"FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"}; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc ${grp//:/ } --output-format csv -d "$OUT/c$i" -o run -- "$(pwd)/tools/bin/pmc_calib" > "$OUT/c$i.log" 2>&1
  rc=$?
  echo "calib pass $i [$grp] rc=$rc" >> "$OUT/status.txt"
  if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -k 10 300 rocprofv3 --pmc ${grp//:/ } --output-format csv -d "$OUT/p$i" -o run -- python3 tools/prof_target.py ${TARGET_ARGS:-} > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i [$grp] rc=$rc" >> "$OUT/status.txt"
  if [ $rc -ne 0 ]; then exit $rc; fi
done

#!/bin/bash
# Process-separated A/B: each variant of tools/sweep.py alone in its own process, alternating
# (AB_VARIANTS="a b", AB_ROUNDS times), so allocation order cannot favour one of them.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab
mkdir -p "$OUT"
i=0
for r in $(seq 1 "${AB_ROUNDS:-2}"); do
  for v in ${AB_VARIANTS}; do
    i=$((i+1))
    timeout -k 10 300 python tools/sweep.py ${AB_SPEC:-} --variants="$v" ${AB_ARGS:-} > "$OUT/$i.$v.log" 2>&1 || exit $?
  done
done

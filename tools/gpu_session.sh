#!/bin/bash
# One GPU session on the gpurun box: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout (rc not in {0,1}) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
OUT=$ROOTDIR/gpurun_out
mkdir -p "$OUT"
: > "$OUT/status.txt"
STEPS="${STEPS:-pytest smoke bench prof}"
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[$(date +%T)] start $name" >> "$OUT/status.txt"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> "$OUT/status.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc in $name; stopping"; tail -30 "$OUT/$name.log"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    pytest) step pytest 1100 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  step bench 600 python bench.py ${BENCH_ARGS:-} ;;
    prof)   export TMPDIR=/tmp
            step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$ROOTDIR/bench.py" --cpu-seconds 0 ${BENCH_ARGS:-} ;;
    sweep)  step sweep 900 python tools/sweep.py ${SWEEP_ARGS:-} ;;
    replay) step replay 400 python tools/bench_replay.py ;;
    rgg)    step bench_rgg 400 python bench.py --workload rgg --n 8388608 --no-conv --cpu-seconds 0 ;;
    rmat)   step bench_rmat 500 python bench.py --workload rmat --no-conv --cpu-seconds 0 --steps ${RMAT_STEPS:-20} --warmup 2 ${RMAT_ARGS:-} ;;
    profrmat) export TMPDIR=/tmp
            step profrmat 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profrmat" -o run -- python3 "$ROOTDIR/bench.py" --workload rmat --no-conv --cpu-seconds 0 --steps ${RMAT_STEPS:-20} --warmup 2 ${RMAT_ARGS:-} ;;
    ubench) step ubench 200 tools/bin/ubench_gather ;;
    rggdist) step bench_rggdist 500 python bench.py --workload rgg-dist --steps 100 --warmup 5 ;;
    rmatline) step bench_rmatline 900 python bench.py --workload rmat --steps 20 --warmup 5 ;;
    rgg23line) step bench_rgg23line 600 python bench.py --workload rgg --n 8388608 --steps 20 --warmup 5 ;;
    pairwise) step bench_pairwise 400 python bench.py --workload pairwise --steps 400 --warmup 50 ;;
    profpw) export TMPDIR=/tmp
            step profpw 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profpw" -o run -- python3 "$ROOTDIR/bench.py" --workload pairwise --steps 400 --warmup 50 --cpu-seconds 0 ;;
    pmc)    step pmc 900 bash tools/pmc.sh ;;
    *) echo "unknown step $s" ;;
  esac
done
tail -5 "$OUT/pytest.log" 2>/dev/null
cat "$OUT/bench.log" 2>/dev/null | tail -3
cat "$OUT/status.txt"

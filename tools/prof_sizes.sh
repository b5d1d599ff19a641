set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
for n in 1000000 400000; do
  m=$((4*n))
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/psz/$n -o run -- python3 tools/sweep.py er:n=$n,m=$m --variants=stage_nopack --warm=10 --timed=50 --reps=2 > gpurun_out/psz_$n.log 2>&1 || exit $?
done

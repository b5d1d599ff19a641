set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ptr$v -o run -- python3 tools/prof_target.py --spec rmat:scale=24,ef=16 --layout degree --kernel pregather --warm 2 --rounds 10 --pack 0 --opt tr_pipe=$v > gpurun_out/ptr$v.log 2>&1 || exit $?
done

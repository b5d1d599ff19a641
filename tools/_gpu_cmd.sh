set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_stage.log
for p in ab/s1024 ab/s1024x256 ab/s2048 ab/s1024 ab/s1024x256 ab/s2048; do
  timeout -k 10 200 python -u tools/_ab_stage.py $p >> gpurun_out/ab_stage.log 2>&1 || exit 1
done
echo rc=$?
cat gpurun_out/ab_stage.log

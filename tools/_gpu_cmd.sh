set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_stage.log
for p in abtest/cur abtest/nt abtest/cur abtest/nt; do
  timeout -k 10 120 python -u tools/_ab_stage.py $p >> gpurun_out/ab_stage.log 2>&1 || exit 1
done
echo rc=$?
grep '^{' gpurun_out/ab_stage.log

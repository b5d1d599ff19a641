# round 4, GPU session t: PMC bytes and the kernel trace of R-MAT-24 with the final round-4
# defaults (lag, k_isolated, multi_short)
set -o pipefail
mkdir -p gpurun_out/t
export TMPDIR=/tmp
rm -rf gpurun_out/pmc
PMC_GROUPS="FETCH_SIZE WRITE_SIZE" TARGET_ARGS="--spec rmat:scale=24,ef=16 --layout degree --kernel pregather --warm 2 --rounds 20 --pack 0" bash tools/pmc.sh || exit $?
python3 tools/pmc_window.py gpurun_out/pmc 20 > gpurun_out/t/pmc_rmat_final.json || exit $?
mv gpurun_out/pmc gpurun_out/t/pmc_rmat_final
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t/prof_rmat -o run -- python3 tools/prof_target.py --spec rmat:scale=24,ef=16 --layout degree --kernel pregather --warm 2 --rounds 20 --pack 0 > gpurun_out/t/prof_rmat.log 2>&1 || exit $?

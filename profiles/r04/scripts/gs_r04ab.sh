# round 4, GPU session ab: tr_nt on (the default) against off on another box, and the PMC bytes
# of R-MAT-24 with the final defaults
set -o pipefail
mkdir -p gpurun_out/ab2
export TMPDIR=/tmp
rm -rf gpurun_out/ab
AB_SPEC="rmat:scale=24,ef=16" AB_ARGS="--warm=3 --timed=20 --reps=3" AB_VARIANTS="deg_np_pre pre_trnt0" AB_ROUNDS=3 bash tools/ab_proc.sh || exit $?
mv gpurun_out/ab gpurun_out/ab2/ab
rm -rf gpurun_out/pmc
PMC_GROUPS="FETCH_SIZE WRITE_SIZE" TARGET_ARGS="--spec rmat:scale=24,ef=16 --layout degree --kernel pregather --warm 2 --rounds 20 --pack 0" bash tools/pmc.sh || exit $?
python3 tools/pmc_window.py gpurun_out/pmc 20 > gpurun_out/ab2/pmc_rmat_trnt.json || exit $?
mv gpurun_out/pmc gpurun_out/ab2/pmc_rmat_trnt

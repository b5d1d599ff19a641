# round 4, GPU session m: kernel 9's row-class thresholds re-checked with the round-4 kernels
# (lag, k_isolated): mega hubs above 4K / 16K edges, heavy rows above 256 edges
set -o pipefail
mkdir -p gpurun_out/m
export TMPDIR=/tmp
rm -rf gpurun_out/ab
AB_SPEC="rmat:scale=24,ef=16" AB_ARGS="--warm=3 --timed=20 --reps=3" AB_VARIANTS="deg_np_pre pre_mega4k pre_mega16k pre_ht256 pre_ht64" AB_ROUNDS=2 bash tools/ab_proc.sh || exit $?
mv gpurun_out/ab gpurun_out/m/ab

# round 4, GPU session q: multi_short with the light tiles on the side stream / with split_tr
set -o pipefail
mkdir -p gpurun_out/q
export TMPDIR=/tmp
rm -rf gpurun_out/ab
AB_SPEC="rmat:scale=24,ef=16" AB_ARGS="--warm=3 --timed=20 --reps=3" AB_VARIANTS="deg_np_pre pre_short pre_short_side1 pre_short_split" AB_ROUNDS=3 bash tools/ab_proc.sh || exit $?
mv gpurun_out/ab gpurun_out/q/ab

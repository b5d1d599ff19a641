# round 4, GPU session o: with lag and k_isolated the side stream ends ~1.1 ms before the main
# stream: the light tiles / rows of 129-256 edges behind the hub path (side_tiles), the heavy
# rows beside the last transposes (split_tr), re-checked
set -o pipefail
mkdir -p gpurun_out/o
export TMPDIR=/tmp
rm -rf gpurun_out/ab
AB_SPEC="rmat:scale=24,ef=16" AB_ARGS="--warm=3 --timed=20 --reps=3" AB_VARIANTS="deg_np_pre pre_side1 pre_side2 pre_split pre_split_side1" AB_ROUNDS=2 bash tools/ab_proc.sh || exit $?
mv gpurun_out/ab gpurun_out/o/ab

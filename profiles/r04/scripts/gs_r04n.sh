# round 4, GPU session n: kernel 9's transposes re-checked with the round-4 kernels: blocks per
# XCD (tr_bpx 48 / 64: up to two per CU) and the software-pipelined transpose
set -o pipefail
mkdir -p gpurun_out/n
export TMPDIR=/tmp
rm -rf gpurun_out/ab
AB_SPEC="rmat:scale=24,ef=16" AB_ARGS="--warm=3 --timed=20 --reps=3" AB_VARIANTS="deg_np_pre pre_tr48 pre_tr64 pre_pipe" AB_ROUNDS=2 bash tools/ab_proc.sh || exit $?
mv gpurun_out/ab gpurun_out/n/ab

# round 5, session ac: k_stage with 2 steps in flight per lane (libfu_su2) against 4: ER-1M
# kernel 8 rounds 1-19, four more alternations, and BASELINE config 2 as written (bench.py
# defaults: 1000 rounds through the packed widths) two alternations.
set -o pipefail
O=gpurun_out/ac
mkdir -p $O
export TMPDIR=/tmp
L=simgrid-flow-updating-implementation_amd/fu
for i in 1 2 3 4; do
  for lib in libfu libfu_su2; do
    timeout -k 10 200 env FU_LIBRARY=$PWD/$L/$lib.so python tools/sweep.py er:n=1000000,m=4000000 --variants=stage_nopack --warm=1 --timed=19 --reps=5 > $O/sweep_er_${lib}_$i.log 2>&1 || exit $?
  done
done
for i in 1 2; do
  for lib in libfu libfu_su2; do
    timeout -k 10 300 env FU_LIBRARY=$PWD/$L/$lib.so python bench.py --no-unit --no-conv --cpu-seconds 0 > $O/bench_default_${lib}_$i.log 2>&1 || exit $?
  done
done
exit 0

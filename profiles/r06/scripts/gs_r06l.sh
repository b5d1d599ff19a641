# round 6, session l: split-plane flows against the session-j library on BASELINE config 2 as
# written (ER-1M, rounds 0-999 timed from zero after a 400-round autotune pass), alternating.
set -o pipefail
O=gpurun_out/r06l
mkdir -p $O
B=simgrid-flow-updating-implementation_amd/fu/libfu_base.so
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 1000 --warmup 400 --no-unit --no-conv --cpu-seconds 0 > $O/c2_new_$i.log 2>&1 || exit $?
  FU_LIBRARY=$PWD/$B timeout -k 10 300 python bench.py --gpus 1 --steps 1000 --warmup 400 --no-unit --no-conv --cpu-seconds 0 > $O/c2_base_$i.log 2>&1 || exit $?
done
exit 0

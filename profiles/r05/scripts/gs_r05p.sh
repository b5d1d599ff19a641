# round 5, session p: non-temporal flow accesses (experiment builds on top of the now-default
# non-temporal stage stores): libfu_fnts (flow stores nt), libfu_fntl (flow loads nt),
# libfu_fntb (both). Bitwise checks of each, then ER-1M kernel 8 (rounds 1-19 unpacked) three
# alternations and R-MAT-24 kernel 9 one alternation against the default build.
set -o pipefail
O=gpurun_out/p
mkdir -p $O
export TMPDIR=/tmp
L=simgrid-flow-updating-implementation_amd/fu
for lib in libfu_fnts libfu_fntl libfu_fntb; do
  timeout -k 10 300 env FU_LIBRARY=$PWD/$L/$lib.so python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "er_vs_c_oracle or ca_sync_fixture_bitwise or headline_window or lag_flows" > $O/pytest_$lib.log 2>&1 || exit $?
done
for i in 1 2 3; do
  for lib in libfu libfu_fnts libfu_fntl libfu_fntb; do
    timeout -k 10 200 env FU_LIBRARY=$PWD/$L/$lib.so python tools/sweep.py er:n=1000000,m=4000000 --variants=stage_nopack --warm=1 --timed=19 --reps=5 > $O/sweep_er_${lib}_$i.log 2>&1 || exit $?
  done
done
for lib in libfu libfu_fnts libfu_fntl libfu_fntb; do
  timeout -k 10 300 env FU_LIBRARY=$PWD/$L/$lib.so python tools/sweep.py rmat:scale=24,ef=16 --variants=deg_np_pre --warm=3 --timed=20 --reps=3 > $O/sweep_rmat_${lib}_1.log 2>&1 || exit $?
done
exit 0

# round 5, session n: non-temporal hints on kernel 8's staged estimates (experiment builds):
# libfu_stnt (k_stage's G stores nt), libfu_glnt (k_round_staged's G loads nt), libfu_bothnt;
# bitwise checks of each, then tools/sweep.py on ER-1M (kernel 8, rounds 1-19 unpacked) in
# separate processes, alternating three times with the default build.
set -o pipefail
O=gpurun_out/n
mkdir -p $O
export TMPDIR=/tmp
L=simgrid-flow-updating-implementation_amd/fu
for lib in libfu_stnt libfu_glnt libfu_bothnt; do
  timeout -k 10 300 env FU_LIBRARY=$PWD/$L/$lib.so python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "er_vs_c_oracle and stage or ca_sync_fixture_bitwise and stage or headline_window" > $O/pytest_$lib.log 2>&1 || exit $?
done
for i in 1 2 3; do
  for lib in libfu libfu_stnt libfu_glnt libfu_bothnt; do
    timeout -k 10 200 env FU_LIBRARY=$PWD/$L/$lib.so python tools/sweep.py er:n=1000000,m=4000000 --variants=stage_nopack --warm=1 --timed=19 --reps=5 > $O/sweep_${lib}_$i.log 2>&1 || exit $?
  done
done
exit 0

# round 5, session c: kernel 8 option st_split (the next round's stage on a second stream in
# (the st_split option was removed after this session: profiles/r05/c)
# two slice groups, each behind the tiles of its rows; G double-buffered) on ER-1M: the
# parity test, then the driver's command with and without it, alternating in separate
# processes (x3), and a kernel trace of the split window.
set -o pipefail
O=gpurun_out/c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -s -x -v --timeout 250 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "stage_split or ca_sync_fixture or er_vs_c" > $O/pytest.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-conv --no-unit --cpu-seconds 0 > $O/base_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-conv --no-unit --cpu-seconds 0 --opt st_split=1 > $O/split_$i.log 2>&1 || exit $?
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_split -o run -- python3 bench.py --steps 20 --warmup 5 --no-conv --no-unit --cpu-seconds 0 --opt st_split=1 > $O/prof_split.log 2>&1 || exit $?

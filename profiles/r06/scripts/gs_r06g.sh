# round 6, session g: why kernel 8 with 7-byte codes ran 149 us per round: kernel traces of the
# bench with kernel 8 pinned, g56 = 0 (doubles), 1 (non-temporal code stores), 2 (plain stores).
set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
export TMPDIR=/tmp
for g in 0 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_g$g -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-unit --no-conv --cpu-seconds 0 --kernel stage --opt g56=$g > $O/bench_g$g.log 2>&1 || exit $?
done
exit 0

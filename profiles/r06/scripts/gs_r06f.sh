# round 6, session f: kernel 8's 7-byte staged codes for unpacked tables (option g56): the
# kernel-8 GPU tests, then the driver's command with g56 on and off, alternating processes.
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 600 python -u -m pytest -s -x -v --timeout 400 --timeout-method thread tests -m gpu -k "stage or staged or headline or config2 or fixture or marked or dist_ghost or option_errors" > $O/pytest.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-unit --cpu-seconds 0 > $O/bench_g56_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-unit --cpu-seconds 0 --opt g56=0 > $O/bench_g64_$i.log 2>&1 || exit $?
done
exit 0

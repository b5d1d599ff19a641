# round 5, session h: fu_get_estimates / fu_get_flows through pinned bounce buffers (copy_out);
# the GPU suite (capture off), smoke, the driver's command with host_io.
set -o pipefail
O=gpurun_out/h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || exit $?
exit 0

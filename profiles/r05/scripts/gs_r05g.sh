# round 5, session g: the driver's command with the host_io record (fu_create's upload and
# plans, fu_get_estimates' download: the PCIe-inclusive rate beside the value).
set -o pipefail
O=gpurun_out/g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || exit $?
exit 0

# round 5, session ae: kernel trace of BASELINE config 2 as written (bench.py defaults, 1000
# rounds): what the packed (8-bit) rounds spend per launch.
set -o pipefail
O=gpurun_out/ae
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_default -o run -- python3 bench.py --no-unit --no-conv --cpu-seconds 0 > $O/prof_default.log 2>&1 || exit $?
exit 0

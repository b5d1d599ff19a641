# round 5, session m: the part's streaming ceiling (tools/ubench_copy.hip): float4 copy
# variants, read-only, write-only and a 2-read/1-write mix over grid sizes, 512 MB and 2 GB
# per buffer.
set -o pipefail
O=gpurun_out/m
mkdir -p $O
timeout -k 10 120 tools/bin/ubench_copy 536870912 > $O/ubench_copy_512M.log 2>&1 || exit $?
timeout -k 10 200 tools/bin/ubench_copy 2147483648 > $O/ubench_copy_2G.log 2>&1 || exit $?
exit 0

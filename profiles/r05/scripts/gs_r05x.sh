# round 5, session x: the CLI on the reference inputs (python -m fu collectall / pairwise,
# --sync, bench-graph), test_cli_reference_inputs_watcher_lines.
set -o pipefail
O=gpurun_out/x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k cli_reference > $O/pytest.log 2>&1 || exit $?
exit 0

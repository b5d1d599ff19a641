# round 6, session c: the window's host side, A/B in one process (tools/ab_window.py): Python
# marks between run() calls against one fu_run_collectall_marked call.
set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 300 python tools/ab_window.py --reps 10 > $O/ab_window.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab_window.py --reps 10 > $O/ab_window_2.log 2>&1 || exit $?
exit 0

#!/usr/bin/env python3
"""A/B of the timed window's host side on one engine (ER-1M, the driver's 20 rounds): the
marks recorded from Python between run() calls ("py", bench.py before round 6) against one
fu_run_collectall_marked call ("marked": mark 0 is round 0's own start event), alternating,
each after fu_reset. Prints, per
variant, the wall time of the window (what `value` divides by) and the device time between
the first and last mark, and round 0's device time.

    python tools/ab_window.py [--reps 8] [--steps 20]
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "simgrid-flow-updating-implementation_amd"))

import numpy as np  # noqa: E402

import bench  # noqa: E402
import fu  # noqa: E402


def window(eng, b, how):
    ra = np.asarray(b, dtype=np.int32)
    eng.synchronize()
    t0 = time.perf_counter()
    if how == "py":
        eng.mark(0)
        for k in range(len(b) - 1):
            eng.run(b[k + 1] - b[k])
            eng.mark(k + 1)
    else:
        eng.run_marked(ra)
    eng.synchronize()
    wall = time.perf_counter() - t0
    return wall * 1e6, eng.elapsed(0, len(b) - 1) * 1e3, eng.elapsed(0, 1) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    g = fu.Graph.erdos_renyi(1_000_000, 4_000_000, seed=1)
    eng = fu.CollectAll(g, fu.uniform_values(g.n, seed=0))
    bench.prepare(eng, "auto", 5)
    b = bench.chunk_bounds(a.steps)
    res = {"py": [], "marked": []}
    for r in range(a.reps):
        for how in (("py", "marked") if r % 2 == 0 else ("marked", "py")):
            eng.reset()
            eng.run(64)  # the settle's part: the chip busy right before the window
            eng.synchronize()
            eng.reset()
            res[how].append(window(eng, b, how))
    for how, v in res.items():
        w = statistics.median(x[0] for x in v)
        d = statistics.median(x[1] for x in v)
        r0 = statistics.median(x[2] for x in v)
        print(f"{how:7s} wall {w:8.1f} us  device {d:8.1f} us  wall-device {w - d:6.1f} us  round0 {r0:5.1f} us  "
              f"(all walls: {[round(x[0]) for x in v]})", flush=True)
    eng.close()


if __name__ == "__main__":
    main()

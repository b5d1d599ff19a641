#!/usr/bin/env python3
"""Profiling target (for rocprofv3): the bench's timed region without the bench around it.
ER-1M, kernel "auto": `warm` rounds (autotune), reset, then `rounds` rounds from the zero
state, exactly as bench.py times them."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simgrid-flow-updating-implementation_amd"))
import fu  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--spec", default="er:n=1000000,m=4000000")
ap.add_argument("--kernel", default="auto")
ap.add_argument("--warm", type=int, default=20)
ap.add_argument("--rounds", type=int, default=1000)
ap.add_argument("--pack", type=int, default=1)
ap.add_argument("--tile", type=int, default=0, help="kernel 4 tile edges (2048/1024/512); 0 = default")
ap.add_argument("--layout", default="given")
ap.add_argument("--opt", action="append", default=[], help="extra engine option key=value (repeatable)")
ap.add_argument("--pairwise", default="", help="WARMUP:STEPS: bench.py's pairwise window instead (RR-64K "
                "tick replay: ticks 0..51+WARMUP in one launch, then the STEPS timed ticks in a second)")
ap.add_argument("--dist-rgg", type=int, default=0, help="N: bench.py's rgg-dist window instead (RGG of N "
                "nodes through the partitioned path at one RCCL rank, kernel auto: tune, --warm rounds, "
                "reset, --rounds rounds)")
a = ap.parse_args()
if a.dist_rgg:
    from fu.dist import DistCollectAll, RggPart, unique_id

    part = RggPart(a.dist_rgg, avg_deg=8.0, seed=1, nparts=1, part=0)
    eng = DistCollectAll(part.to_plan(), part.values(seed=0), unique_id(), kernel=a.kernel)
    if a.kernel == "auto":
        eng.tune()
    eng.run(a.warm)
    eng.reset()
    eng.run(a.rounds)
    eng.synchronize()
    print("rgg-dist", part.n_local, part.e_local, "info", eng.info())
    sys.exit(0)
if a.pairwise:
    warm, steps = (int(x) for x in a.pairwise.split(":"))
    g = fu.Graph.random_regular(65536, 8, seed=1)
    v = fu.uniform_values(g.n, seed=0)
    t0 = 51 + warm
    tr = fu.Trace(g.rowptr, g.col, "pairwise", t0 + steps, "rand:3")
    rep = fu.Replay(tr, v, persistent=True)
    rep.run(t0)
    rep.run(t0 + steps)
    print("pairwise", g.n, g.E, "ticks", t0, t0 + steps)
    sys.exit(0)
g = fu.Graph.from_spec(a.spec, seed=1)
v = fu.uniform_values(g.n, seed=0)
eng = fu.CollectAll(g, v, kernel=a.kernel, layout=a.layout)
eng.set_option("pack", a.pack)
if a.tile:
    eng.set_option("tile_edges", a.tile)
for kv in a.opt:
    k, _, val = kv.partition("=")
    eng.set_option(k, int(val))
if a.kernel == "auto":
    eng.tune()  # as bench.py: one untimed autotune pass
eng.run(a.warm)
eng.reset()
eng.run(a.rounds)
eng.synchronize()
print("n", g.n, "E", g.E, "alg_bytes", 24 * g.E + 28 * g.n, "info", eng.info(), "pack", eng.pack_widths())

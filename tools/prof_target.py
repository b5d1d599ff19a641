#!/usr/bin/env python3
"""Small profiling target: ER-1M, `rounds` rounds of one kernel variant (for rocprofv3)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simgrid-flow-updating-implementation_amd"))
import fu  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--spec", default="er:n=1000000,m=4000000")
ap.add_argument("--kernel", default="recon")
ap.add_argument("--rounds", type=int, default=50)
ap.add_argument("--nt", type=int, default=0)
ap.add_argument("--diag", type=int, default=0)
a = ap.parse_args()
g = fu.Graph.from_spec(a.spec, seed=1)
v = fu.uniform_values(g.n, seed=0)
eng = fu.CollectAll(g, v, kernel=a.kernel)
eng.set_option("nt", a.nt)
eng.run(2)
eng.set_option("diag", a.diag)
eng.run(a.rounds)
eng.synchronize()
print("n", g.n, "E", g.E, "alg_bytes", 24 * g.E + 28 * g.n)

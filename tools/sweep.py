#!/usr/bin/env python3
"""Kernel-variant sweep on the headline workload (ER-1M): device time per round for each
round-kernel variant, interleaved in one process (cdna guide §5.4 rule 24)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simgrid-flow-updating-implementation_amd"))
import fu  # noqa: E402

specs = sys.argv[1:] or ["er:n=1000000,m=4000000"]
for spec in specs:
    g = fu.Graph.from_spec(spec, seed=1)
    v = fu.uniform_values(g.n, seed=0)
    engs = {k: fu.CollectAll(g, v, kernel=k) for k in ("thread", "tile", "push", "recon")}
    engs["recon_nt"] = fu.CollectAll(g, v, kernel="recon")
    engs["recon_nt"].set_option("nt", 1)
    for d in (1, 2):  # timing-only ablations (wrong results): price the gather / the flows
        engs[f"recon_diag{d}"] = fu.CollectAll(g, v, kernel="recon")
    for k, e in engs.items():
        e.run(10)
        if k.startswith("recon_diag"):
            e.set_option("diag", int(k[-1]))
    res = {k: [] for k in engs}
    for rep in range(5):
        for k, e in engs.items():
            res[k].append(e.run_timed(200) / 200 * 1e3)
    alg = 24 * g.E + 28 * g.n
    out = {"spec": spec, "n": g.n, "E": g.E, "max_deg": g.max_deg}
    for k, ts in res.items():
        med = sorted(ts)[len(ts) // 2]
        out[k] = {"us_per_round_med": med, "us_min": min(ts),
                  "alg_GBs": alg / (med * 1e-6) / 1e9, "edge_updates_per_s": g.E / (med * 1e-6)}
    print(json.dumps(out), flush=True)
    for e in engs.values():
        e.close()

"""Exact-chain speed: one star hub of L leaves (kernel 4's mega-hub path), device us/round."""
import sys, os, json
sys.path.insert(0, sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "simgrid-flow-updating-implementation_amd"))
import numpy as np
import fu
for L in (100_000, 1_000_000):
    hub = L
    g = fu.Graph.from_edges(L + 1, np.full(L, hub, dtype=np.int32), np.arange(L, dtype=np.int32))
    v = fu.uniform_values(g.n, seed=1)
    out = {"pkg": sys.argv[1] if len(sys.argv) > 1 else "", "leaves": L}
    for name, opts in (("chain", {}), ("diag5", {"diag": 5})):
        e = fu.CollectAll(g, v, kernel="recon")
        e.run(5)
        for k, val in opts.items():
            e.set_option(k, val)
        ts = sorted(e.run_timed(10) / 10 * 1e3 for _ in range(3))
        out[name] = round(ts[1], 1)
        e.close()
    out["ns_per_element"] = round((out["chain"] - out["diag5"]) * 1e3 / L, 2)
    print(json.dumps(out), flush=True)

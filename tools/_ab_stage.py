"""A/B timing of kernel 8 (stage) on ER-1M across builds: python tools/_ab_stage.py <pkgdir>"""
import sys, json
sys.path.insert(0, sys.argv[1])
import fu
g = fu.Graph.erdos_renyi(1_000_000, 4_000_000, seed=1)
v = fu.uniform_values(g.n, seed=0)
out = {"pkg": sys.argv[1]}
for name, warm, timed, opts in (("early", 20, 20, {}), ("steady", 400, 200, {}), ("pipe_steady", 400, 200, {"k": "pipe_stage"})):
    e = fu.CollectAll(g, v, kernel=opts.get("k", "stage"))
    e.run(warm)
    ts = []
    for _ in range(3):
        ts.append(e.run_timed(timed) / timed * 1e3)
    out[name] = round(sorted(ts)[1], 2)
    a = e.estimates()
    out[name + "_chk"] = float(a[:1000].sum())
    e.close()
print(json.dumps(out), flush=True)

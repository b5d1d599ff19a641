"""A/B timing of kernel 4 on one graph across builds: python tools/_ab.py <pkgdir> <spec>"""
import sys, json
sys.path.insert(0, sys.argv[1])
import fu
spec = sys.argv[2]
g = fu.Graph.from_spec(spec, seed=1)
v = fu.uniform_values(g.n, seed=0)
out = {"pkg": sys.argv[1], "spec": spec}
for te in (2048, 1024, 512):
    e = fu.CollectAll(g, v, kernel="recon")
    e.set_option("tile_edges", te)
    e.run(400)
    ts = sorted(e.run_timed(200) / 200 * 1e3 for _ in range(3))
    out[te] = round(ts[1], 1)
    e.close()
print(json.dumps(out), flush=True)

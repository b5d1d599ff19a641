#!/usr/bin/env python3
"""Kernel-variant sweep: device time per round for each round-kernel variant, interleaved
in one process (cdna guide §5.4 rule 24).

    python tools/sweep.py [spec ...] [--variants a,b,c]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simgrid-flow-updating-implementation_amd"))
import fu  # noqa: E402

VARIANTS = {
    "recon": ("recon", {"tile_edges": 2048}),
    "recon_1024": ("recon", {"tile_edges": 1024}),
    "recon_1024_c16off": ("recon", {"tile_edges": 1024, "c16": 0}),
    "recon_1024x256": ("recon", {"tile_edges": 1024, "tile_nodes": 256}),
    "recon_512": ("recon", {"tile_edges": 512}),
    "recon_nopack": ("recon", {"pack": 0}),
    "recon_1024_nopack": ("recon", {"tile_edges": 1024, "pack": 0}),
    "recon_nofork": ("recon", {"fork_heavy": 0}),
    "recon_blockheavy": ("recon", {"wave_heavy": 0}),
    "recon_deg": ("recon", {"layout": "degree"}),
    "recon_deg_mega2048": ("recon", {"mega_hub": 2048, "layout": "degree"}),
    "deg_np": ("recon", {"layout": "degree", "pack": 0}),
    "deg_np_pre": ("pregather", {"layout": "degree", "pack": 0}),
    "pre_mid0": ("pregather", {"layout": "degree", "pack": 0, "mid_heavy": 0}),
    "pre_multi0": ("pregather", {"layout": "degree", "pack": 0, "multi_heavy": 0}),
    "pre_multimid0": ("pregather", {"layout": "degree", "pack": 0, "multi_mid": 0}),
    "pre_lag": ("pregather", {"layout": "degree", "pack": 0, "lag": 1}),
    "pre_iso0": ("pregather", {"layout": "degree", "pack": 0, "iso_rows": 0}),
    "pre_short": ("pregather", {"layout": "degree", "pack": 0, "multi_short": 1}),
    "pre_trnt": ("pregather", {"layout": "degree", "pack": 0, "tr_nt": 1}),
    "pre_trnt0": ("pregather", {"layout": "degree", "pack": 0, "tr_nt": 0}),
    "pre_short_ht64": ("pregather", {"layout": "degree", "pack": 0, "multi_short": 1, "hub_threshold": 64}),
    "pre_short_ht96": ("pregather", {"layout": "degree", "pack": 0, "multi_short": 1, "hub_threshold": 96}),
    "pre_mega4k": ("pregather", {"layout": "degree", "pack": 0, "mega_hub": 4096}),
    "pre_mega16k": ("pregather", {"layout": "degree", "pack": 0, "mega_hub": 16384}),
    "pre_mega32k": ("pregather", {"layout": "degree", "pack": 0, "mega_hub": 32768}),
    "pre_mega64k": ("pregather", {"layout": "degree", "pack": 0, "mega_hub": 65536}),
    "pre_tr0": ("pregather", {"layout": "degree", "pack": 0, "tr_bpx": 0}),
    "pre_tr16": ("pregather", {"layout": "degree", "pack": 0, "tr_bpx": 16}),
    "pre_tr48": ("pregather", {"layout": "degree", "pack": 0, "tr_bpx": 48}),
    "pre_tr64": ("pregather", {"layout": "degree", "pack": 0, "tr_bpx": 64}),
    "pre_tr128": ("pregather", {"layout": "degree", "pack": 0, "tr_bpx": 128}),
    "pre_mega4k": ("pregather", {"layout": "degree", "pack": 0, "mega_hub": 4096}),
    "pre_mega16k": ("pregather", {"layout": "degree", "pack": 0, "mega_hub": 16384}),
    "pre_mega32k": ("pregather", {"layout": "degree", "pack": 0, "mega_hub": 32768}),
    "pre_mega64k": ("pregather", {"layout": "degree", "pack": 0, "mega_hub": 65536}),
    "pre_ht128": ("pregather", {"layout": "degree", "pack": 0, "hub_threshold": 128}),
    "pre_ht256": ("pregather", {"layout": "degree", "pack": 0, "hub_threshold": 256}),
    "pre_ht512": ("pregather", {"layout": "degree", "pack": 0, "hub_threshold": 512}),
    "deg_np_ht128": ("recon", {"layout": "degree", "pack": 0, "hub_threshold": 128}),
    "deg_np_ht256": ("recon", {"layout": "degree", "pack": 0, "hub_threshold": 256}),
    "deg_np_nosplit": ("recon", {"layout": "degree", "pack": 0, "split_hubs": 0}),
    "stage": ("stage", {}),
    "stage_nopack": ("stage", {"pack": 0}),
    "stage_lo0": ("stage", {"staged_lo": 0}),
    "stage_pe64": ("stage", {"pack_every": 64}),
}

args = [a for a in sys.argv[1:] if not a.startswith("--")]
opts = [a for a in sys.argv[1:] if a.startswith("--variants=")]
names = opts[0].split("=", 1)[1].split(",") if opts else list(VARIANTS)
warm = [int(a.split("=", 1)[1]) for a in sys.argv[1:] if a.startswith("--warm=")]
warm = warm[0] if warm else 10  # rounds before timing (packing engages after ~100-300)
timed = [int(a.split("=", 1)[1]) for a in sys.argv[1:] if a.startswith("--timed=")]
timed = timed[0] if timed else 200  # rounds per timed repetition
reps = [int(a.split("=", 1)[1]) for a in sys.argv[1:] if a.startswith("--reps=")]
reps = reps[0] if reps else 5
specs = args or ["er:n=1000000,m=4000000"]
for spec in specs:
    g = fu.Graph.from_spec(spec, seed=1)
    v = fu.uniform_values(g.n, seed=0)
    engs = {}
    for nm in names:
        kern, o = VARIANTS[nm]
        e = fu.CollectAll(g, v, kernel=kern, layout=o.get("layout", "given"))
        for k, val in o.items():
            if k != "layout":
                e.set_option(k, val)
        e.run(warm)
        engs[nm] = e
    res = {k: [] for k in engs}
    for rep in range(reps):
        for k, e in engs.items():
            res[k].append(e.run_timed(timed) / timed * 1e3)
    alg = 24 * g.E + 28 * g.n
    out = {"spec": spec, "n": g.n, "E": g.E, "max_deg": g.max_deg, "warm": warm}
    for k, ts in res.items():
        med = sorted(ts)[len(ts) // 2]
        out[k] = {"us_per_round_med": med, "us_min": min(ts),
                  "alg_GBs": alg / (med * 1e-6) / 1e9, "edge_updates_per_s": g.E / (med * 1e-6),
                  "pack": engs[k].pack_widths(),
                  "info": {k2: engs[k].info()[k2] for k2 in ("kernel", "tile", "mega_hubs")}}
    print(json.dumps(out), flush=True)
    for e in engs.values():
        e.close()

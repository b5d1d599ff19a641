#!/usr/bin/env python3
"""profiles/pmc_traffic.json from pmc_summary.py outputs: the HBM-side bytes per round of the
round's launches (one summary per launch kind, summed), read by bench.py for
roofline.traffic when (n, E, kernel_selected, rounds_timed) match its own run.

    python tools/pmc_summary.py gpurun_out/pmc "<kernel name>" > s1.json   (per launch kind)
    python tools/make_pmc_traffic.py <n> <E> <selected> <rounds_timed> <all|last40> s1.json [s2.json ...]

Records for other (graph, kernel, window) keys already in profiles/pmc_traffic.json are kept.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
n, E, selected, rounds_timed, window = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), sys.argv[5]
key = "all_launches" if window == "all" else "steady_state_last40pct"
parts = []
for path in sys.argv[6:]:
    s = json.load(open(path))
    st = s[key]
    parts.append({"kernel_filter": s["kernel_filter"], "launches": st["launches"],
                  "fetch_bytes": st["fetch_bytes"], "write_bytes": st["write_bytes"],
                  "bytes_per_launch": st["hbm_bytes_per_launch"], "l2_hit_rate": st.get("l2_hit_rate")})
cal = json.load(open(sys.argv[6]))["calibration"]
rec = {
    "n": n, "E": E, "kernel_selected": selected, "rounds_timed": rounds_timed, "window": key,
    "bytes_per_launch": sum(p["bytes_per_launch"] for p in parts),
    "fetch_bytes": sum(p["fetch_bytes"] for p in parts),
    "write_bytes": sum(p["write_bytes"] for p in parts),
    "per_launch_kind": parts,
    "calibration": {k: v for k, v in cal.items() if k.endswith("_SIZE")},
    "note": ("rocprofv3 --pmc, one counter group per pass (tools/pmc.sh), kernel pinned to the "
             "bench's choice; per round = the sum over the round's launch kinds, each averaged over "
             f"the window '{key}'. FETCH_SIZE is corrected by the calibration program's factor for "
             "8-B-per-lane reads (0.5 counter bytes per true byte, tools/pmc_calib.hip); WRITE_SIZE "
             "needs no correction. Both count L2 <-> fabric traffic (Infinity Cache hits included)."),
}
path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
recs = []
if os.path.exists(path):
    old = json.load(open(path))
    recs = [r for r in (old if isinstance(old, list) else [old])
            if (r.get("n"), r.get("E"), r.get("kernel_selected"), r.get("rounds_timed")) !=
            (n, E, selected, rounds_timed)]
recs.append(rec)
json.dump(recs, open(path, "w"), indent=1)
print(json.dumps(rec, indent=1))

#!/usr/bin/env python3
"""profiles/pmc_traffic.json from pmc_summary.py outputs: the steady-state HBM bytes per
round of the selected round kernel(s) (one summary per launch of the round, summed), read
by bench.py for roofline.traffic.

    python tools/pmc_summary.py gpurun_out/pmc "<kernel name>" > s1.json   (per launch kind)
    python tools/make_pmc_traffic.py <n> <E> <selected> s1.json [s2.json ...] > profiles/pmc_traffic.json
"""
import json
import sys

n, E, selected = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
parts = []
for path in sys.argv[4:]:
    s = json.load(open(path))
    st = s["steady_state_last40pct"]
    parts.append({"kernel_filter": s["kernel_filter"], "launches": st["launches"],
                  "fetch_bytes": st["fetch_bytes"], "write_bytes": st["write_bytes"],
                  "bytes_per_launch": st["hbm_bytes_per_launch"], "l2_hit_rate": st.get("l2_hit_rate")})
cal = json.load(open(sys.argv[4]))["calibration"]
print(json.dumps({
    "n": n, "E": E, "kernel": "auto", "kernel_selected": selected,
    "bytes_per_launch": sum(p["bytes_per_launch"] for p in parts),
    "fetch_bytes": sum(p["fetch_bytes"] for p in parts),
    "write_bytes": sum(p["write_bytes"] for p in parts),
    "per_launch_kind": parts,
    "calibration": {k: v for k, v in cal.items() if k.endswith("_SIZE")},
    "note": ("rocprofv3 --pmc, one counter group per pass (tools/pmc.sh), kernel pinned to the "
             "bench's steady-state choice; per round = the sum over the round's launches, each "
             "averaged over the last 40 % of its launches (packed steady state). FETCH_SIZE is "
             "corrected by the calibration program's factor for 8-B-per-lane reads (0.5 counter "
             "bytes per true byte, tools/pmc_calib.hip), which makes fetch_bytes an upper bound. "
             "WRITE_SIZE needs no correction (factor 1.0)."),
}, indent=1))

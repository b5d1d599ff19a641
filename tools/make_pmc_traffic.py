#!/usr/bin/env python3
"""profiles/pmc_traffic.json from a pmc_summary.py output: the steady-state HBM bytes per
launch of the dominant round kernel, read by bench.py for roofline.traffic.

    python tools/pmc_summary.py gpurun_out/pmc "<kernel name>" > s.json
    python tools/make_pmc_traffic.py s.json <n> <E> <kernel name> > profiles/pmc_traffic.json
"""
import json
import sys

s = json.load(open(sys.argv[1]))
n, E, name = int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
st = s["steady_state_last40pct"]
print(json.dumps({
    "n": n, "E": E, "kernel": "auto", "kernel_name": name,
    "bytes_per_launch": st["hbm_bytes_per_launch"],
    "fetch_bytes": st["fetch_bytes"], "write_bytes": st["write_bytes"],
    "fetch_bytes_raw": st["fetch_bytes_raw"], "l2_hit_rate": st["l2_hit_rate"],
    "launches": st["launches"],
    "all_launches_bytes_per_launch": s["all_launches"]["hbm_bytes_per_launch"],
    "calibration": {k: v for k, v in s["calibration"].items() if k.endswith("_SIZE")},
    "note": ("rocprofv3 --pmc, one counter group per pass (tools/pmc.sh); the last 40 % of the "
             "kernel's launches (packed steady state). FETCH_SIZE is corrected by the calibration "
             "program's factor for 8-B-per-lane reads (0.5 counter bytes per true byte, "
             "tools/pmc_calib.hip), which makes fetch_bytes an upper bound: L2-miss gathers "
             "(64-B requests) are not under-counted, so their share is doubled too. WRITE_SIZE "
             "needs no correction (factor 1.0)."),
}, indent=1))

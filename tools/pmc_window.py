#!/usr/bin/env python3
"""PMC bytes per round of a multi-launch round (kernel 9 on R-MAT): every dispatch after the
last k_round0 of the profiled run (tools/prof_target.py: warmup, reset, then the timed rounds
0..R-1), summed per kernel name and divided by the R - 1 rounds after round 0. FETCH_SIZE is
corrected by the calibration program's 8-B-per-lane factor (as tools/pmc_summary.py).

    python tools/pmc_window.py gpurun_out/pmc ROUNDS
"""
import collections
import csv
import glob
import json
import os
import re
import sys

root, rounds = sys.argv[1], int(sys.argv[2])
CAL = 512 << 20


def rows(pattern):
    for f in sorted(glob.glob(os.path.join(root, pattern, "run_counter_collection.csv"))):
        yield from csv.DictReader(open(f))


fac = {}
for r in rows("c*"):
    n = r["Kernel_Name"]
    w = "read8" if "k_read<double>" in n else "write8" if "k_write8" in n else None
    if w:
        fac[(w, r["Counter_Name"])] = float(r["Counter_Value"]) * 1024.0 / CAL
out = {}
for cname, wkey in (("FETCH_SIZE", "read8"), ("WRITE_SIZE", "write8")):
    recs = sorted(((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])) for r in rows("p*")
                   if r["Counter_Name"] == cname), key=lambda x: x[0])
    last0 = max(i for i, (_, n, _) in enumerate(recs) if "k_round0" in n and "flows" not in n)
    per = collections.defaultdict(float)
    for _, n, val in recs[last0 + 1:]:
        m = re.search(r"(k_\w+(<[^>]*>)?)", n)
        per[m.group(1) if m else n[:40]] += val * 1024.0 / fac[(wkey, cname)] / (rounds - 1)
    out[cname] = dict(per)
kinds = sorted(set(out["FETCH_SIZE"]) | set(out["WRITE_SIZE"]))
res = {"per_launch_kind": [{"kernel_filter": k, "fetch_bytes_per_round": out["FETCH_SIZE"].get(k, 0.0),
                            "write_bytes_per_round": out["WRITE_SIZE"].get(k, 0.0)} for k in kinds]}
res["fetch_bytes"] = sum(out["FETCH_SIZE"].values())
res["write_bytes"] = sum(out["WRITE_SIZE"].values())
res["bytes_per_launch"] = res["fetch_bytes"] + res["write_bytes"]
print(json.dumps(res, indent=1))

#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (gpurun_out/pmc/p*/run_counter_collection.csv) for the round
kernel: per-launch averages. FETCH_SIZE/WRITE_SIZE are KB; per MI355X_MICROARCH.md §HBM,
gfx950 FETCH_SIZE counts 64 B per TCC_EA0_RDREQ (128-B streaming requests are tallied at
64 B), so the read side is also reported as TCC_EA0_RDREQ x 64 B and the streaming-corrected
upper bound (x2 for the streamed share)."""
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
kern = sys.argv[2] if len(sys.argv) > 2 else "k_round_recon"
agg = {}
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
out = {k: sum(v) / len(v) for k, v in agg.items()}
out["launches"] = max(len(v) for v in agg.values()) if agg else 0
if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
    out["fetch_bytes"] = out["FETCH_SIZE"] * 1024
    out["write_bytes"] = out["WRITE_SIZE"] * 1024
    out["hbm_bytes_per_launch"] = out["fetch_bytes"] + out["write_bytes"]
if "TCC_HIT_sum" in out:
    out["l2_hit_rate"] = out["TCC_HIT_sum"] / (out["TCC_HIT_sum"] + out["TCC_MISS_sum"])
print(json.dumps(out, indent=1))

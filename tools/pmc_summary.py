#!/usr/bin/env python3
"""Summarise the PMC passes of tools/pmc.sh: per-launch averages of the round kernel
(k_round_recon, all geometries; or the kernel-name filter given), over all launches and over
the last 40 % (the packed steady state), with FETCH_SIZE / WRITE_SIZE corrected by the
calibration program's 8-B-per-lane factors (MI355X_MICROARCH.md § HBM: FETCH_SIZE is
calibrated there only for 16-B-per-lane streams, so calibrate on our own access width).

    python tools/pmc_summary.py [gpurun_out/pmc] [kernel-filter]
"""
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
kern = sys.argv[2] if len(sys.argv) > 2 else "k_round_recon"
CAL_BYTES = 512 << 20


def rows(pattern):
    for f in sorted(glob.glob(os.path.join(root, pattern, "run_counter_collection.csv"))):
        yield from csv.DictReader(open(f))


# calibration: counter value per true byte, per access width
cal = {}
for r in rows("c*"):
    name = r["Kernel_Name"]
    w = "read8" if "k_read<double>" in name else "read4" if "k_read<int>" in name else \
        "write8" if "k_write8" in name else None
    if w:
        cal.setdefault(w, {})[r["Counter_Name"]] = float(r["Counter_Value"])
factors = {}
for w, c in cal.items():
    for k, val in c.items():
        unit = 1024.0 if k in ("FETCH_SIZE", "WRITE_SIZE") else 1.0
        factors[f"{w}:{k}"] = val * unit / CAL_BYTES  # counter bytes (or requests) per true byte

per = {}
for r in rows("p*"):
    if kern in r["Kernel_Name"]:
        per.setdefault(r["Counter_Name"], []).append((int(r.get("Dispatch_Id", 0) or 0), float(r["Counter_Value"])))


def summarise(sel):
    out = {k: sum(v for _, v in xs) / len(xs) for k, xs in sel.items() if xs}
    out["launches"] = max((len(xs) for xs in sel.values()), default=0)
    if "FETCH_SIZE" in out:
        out["fetch_bytes_raw"] = out["FETCH_SIZE"] * 1024
        f8 = factors.get("read8:FETCH_SIZE")
        out["fetch_bytes"] = out["fetch_bytes_raw"] / f8 if f8 else None
    if "WRITE_SIZE" in out:
        out["write_bytes_raw"] = out["WRITE_SIZE"] * 1024
        w8 = factors.get("write8:WRITE_SIZE")
        out["write_bytes"] = out["write_bytes_raw"] / w8 if w8 else None
    if out.get("fetch_bytes") is not None and out.get("write_bytes") is not None:
        out["hbm_bytes_per_launch"] = out["fetch_bytes"] + out["write_bytes"]
    if "TCC_HIT_sum" in out and "TCC_MISS_sum" in out:
        out["l2_hit_rate"] = out["TCC_HIT_sum"] / max(1.0, out["TCC_HIT_sum"] + out["TCC_MISS_sum"])
    return out


whole = summarise(per)
steady = summarise({k: sorted(xs)[int(len(xs) * 0.6):] for k, xs in per.items()})
print(json.dumps({"kernel_filter": kern, "calibration": factors, "all_launches": whole,
                  "steady_state_last40pct": steady}, indent=1))

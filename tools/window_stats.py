#!/usr/bin/env python3
"""Per-kernel durations inside bench.py's timed window (rounds 0..K-1 from the zero state:
from the second k_round0 launch to the third, i.e. after the warmup's reset and before the
convergence run) from a rocprofv3 --kernel-trace CSV.

    python tools/window_stats.py gpurun_out/prof/run_kernel_trace.csv [out.json]
"""
import collections
import csv
import json
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
seq = []
for r in rows:
    m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
    seq.append((m.group(1) if m else r["Kernel_Name"][:40], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
r0 = [i for i, s in enumerate(seq) if s[0].startswith("k_round0")]
w = seq[r0[1]:r0[2]] if len(r0) >= 3 else seq[r0[-1]:]
per = collections.defaultdict(list)
for nm, a, b in w:
    per[nm].append((b - a) / 1e3)
out = {k: {"calls": len(v), "mean_us": round(sum(v) / len(v), 2), "min_us": round(min(v), 2),
           "max_us": round(max(v), 2)} for k, v in per.items()}
rounds = [s for s in w if s[0].startswith(("k_round_staged", "k_round_recon"))]
first = next((s for s in w[1:]), None)
if rounds and first:
    out["_rounds_1_on_wall_us_per_round"] = round((rounds[-1][2] - first[1]) / 1e3 / len(rounds), 2)
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    json.dump({"source": sys.argv[1], "window": out}, open(sys.argv[2], "w"), indent=1)

#!/usr/bin/env python3
"""Per-round wall span from a rocprofv3 kernel trace: rounds are delimited by the launches of
the given marker kernel (default: the first kernel of each round). Prints the span of every
round and the kernels' [start, end) offsets within the last one.

    python tools/round_times.py gpurun_out/diag/d0/run_kernel_trace.csv [marker]"""
import csv
import sys

tr = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
tr = [r for r in tr if "rocclr" not in r["Kernel_Name"] and "k_round0" not in r["Kernel_Name"]]
marker = sys.argv[2] if len(sys.argv) > 2 else None
if marker is None:  # the kernel that opens a round: the first one after the last k_round0
    marker = tr[0]["Kernel_Name"]
starts = [k for k, r in enumerate(tr) if r["Kernel_Name"] == marker]
spans = []
for a, b in zip(starts, starts[1:] + [len(tr)]):
    rs = tr[a:b]
    t0 = min(int(r["Start_Timestamp"]) for r in rs)
    t1 = max(int(r["End_Timestamp"]) for r in rs)
    spans.append((t1 - t0) / 1e3)
print("round spans (us):", [round(s, 1) for s in spans])
rs = tr[starts[-1]:]
t0 = min(int(r["Start_Timestamp"]) for r in rs)
for r in rs:
    n = r["Kernel_Name"]
    tag = n.split("(")[0].split("::")[-1] + ("<" + n.split("<", 1)[1].split(">")[0] + ">" if "<" in n else "")
    print(f"  {tag[:70]:70s} q{r['Queue_Id']} {(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {(int(r['End_Timestamp']) - t0) / 1e3:9.1f}")

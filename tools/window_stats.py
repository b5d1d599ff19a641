#!/usr/bin/env python3
"""Per-kernel durations inside bench.py's timed window (rounds 0..K-1 from the zero state) from
a rocprofv3 --kernel-trace CSV of the same command, as the record bench.py quotes
(`roofline.archived_window_profile`, marked archival: another run's record) when n, E, kernel
and K match its run.

    python tools/window_stats.py TRACE.csv --n N --E E --kernel KNAME --steps K [--which I]
                                 [--copy-GBs C] [--commit SHA] [--out profiles/r06/NAME_window_stats.json]
                                 [--dump profiles/r05/NAME_window_trace.csv]

The window starts at the (I+1)-th k_round0 launch of the process (I = 1 by default: the first
k_round0 is the autotune / warmup run, the second the timed run; the R-MAT unit of the N = 1
line is a later engine: pass its index) and spans K rounds: round 0, then the launches up to
the next k_round0 or the K-1 rounds that follow. avg_round_us = (end of the last launch of
round K-1 - start of the first launch of round 1) / (K - 1), the device time the bench's HIP
events span; frac = (24 E + 28 N) / avg_round_us / 8 TB/s.
"""
import argparse
import collections
import csv
import json
import re

ROUND_KERNELS = {"k_stage", "k_round_staged", "k_round_recon", "k_transpose", "k_heavy_multi", "k_hub_flows",
                 "k_hub_stage", "k_isolated", "k_pack_plan", "k_lag_final", "k_max_err"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--E", type=int, required=True)
    ap.add_argument("--kernel", required=True, help="the bench line's kernel_selected")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--which", type=int, default=1, help="index of the k_round0 launch that starts the window")
    ap.add_argument("--copy-GBs", type=float, default=None, help="the same run's roofline.copy_GBs")
    ap.add_argument("--commit", default=None, help="git commit of the tree the trace ran")
    ap.add_argument("--out")
    ap.add_argument("--dump", help="write the window's launches (name, start, end ns) as CSV, so that the "
                                   "record can be recomputed from a tracked file")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    seq = []
    for r in rows:
        m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
        seq.append((m.group(1) if m else r["Kernel_Name"][:40], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    r0 = [i for i, s in enumerate(seq) if s[0].startswith("k_round0(") or s[0] == "k_round0"]
    start = r0[a.which]
    stop = r0[a.which + 1] if a.which + 1 < len(r0) else len(seq)
    w = seq[start:stop]
    # round boundaries: each round after round 0 begins with its stage launch (kernels 8, 9) or
    # its first tile launch (kernel 4); the first launch after round 0's launches opens round 1
    r0_end = 1
    while r0_end < len(w) and w[r0_end][0].startswith(("k_round0", "k_max_err")):
        r0_end += 1
    body = w[r0_end:]
    head = body[0][0].split("<")[0] if body else None
    starts = [i for i, s in enumerate(body) if s[0].split("<")[0] == head]
    rounds = starts[: a.steps - 1]
    if len(rounds) < a.steps - 1:
        raise SystemExit(f"window holds {len(rounds)} rounds after round 0, expected {a.steps - 1}")
    # round K-1 ends before the next round's head or the first launch that is no round kernel
    # (the bench's copy benchmark, a memset, the next phase's k_round0)
    end_idx = starts[a.steps - 2] + 1
    while end_idx < len(body) and body[end_idx][0].split("<")[0] in ROUND_KERNELS \
            and body[end_idx][0].split("<")[0] != head:
        end_idx += 1
    win = body[: end_idx]
    per = collections.defaultdict(list)
    for nm, s0, s1 in win:
        per[nm].append((s1 - s0) / 1e3)
    t0 = win[0][1]
    t1 = max(s[2] for s in win)
    avg = (t1 - t0) / 1e3 / (a.steps - 1)
    alg = 24 * a.E + 28 * a.n
    rec = {
        "source": a.trace, "n": a.n, "E": a.E, "kernel_selected": a.kernel, "rounds_timed": a.steps,
        "window": f"rounds 1-{a.steps - 1} (launches {len(win)})",
        "avg_round_us": round(avg, 3), "alg_bytes_per_round": alg,
        "frac": alg / (avg * 1e-6) / 1e9 / 8000.0,
        "round0_us": round((w[r0_end - 1][2] - w[0][1]) / 1e3, 3),
        "per_kernel_per_round": {k: round(sum(v) / (a.steps - 1), 3) for k, v in per.items()},
        "per_kernel": {k: {"calls": len(v), "mean_us": round(sum(v) / len(v), 3), "min_us": round(min(v), 3),
                           "max_us": round(max(v), 3)} for k, v in per.items()},
        "copy_GBs": a.copy_GBs, "commit": a.commit,
    }
    if a.dump:
        with open(a.dump, "w") as f:
            f.write("kernel,start_ns,end_ns\n")
            for nm, s0, s1 in w[:r0_end] + win:
                f.write(f'"{nm}",{s0},{s1}\n')
        rec["window_trace"] = a.dump
    print(json.dumps(rec, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()

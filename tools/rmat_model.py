#!/usr/bin/env python3
"""R-MAT-24 (BASELINE config 4) byte-and-time model: the round-5 verdict's gate for one
structural alternative to kernel 9's propagation blocking (CA:106-113 on rows of up to
406,598 edges). CPU only; reads the real graph (this repository's generator, seed 1).

    python tools/rmat_model.py [--scale 24] [--out profiles/r06/rmat24_model.json]

It prices, from the graph's own row-length x slice histogram:
  1. kernel 9 as shipped (degree layout): per launch, the byte model next to the PMC record
     (profiles/pmc_traffic.json), and the floor of this design (every heavy row in one pass);
  2. alternative S, the verdict's slice-outer heavy rows: under layout "given" a row's
     neighbours are sorted by id, so slice order is summation order; a task (slice, row
     group) holds the slice in LDS and continues each row's exact (S, T) chains from the
     previous slice's task, carried through memory; a second slice-outer pass writes the flows
     (f_r = (fr + a) - er needs every er again, CA:117-118);
  3. alternative W, the same idea without LDS tasks: the heavy rows' edges stored per window
     of slices in 64-lane SELL order, every CU sweeping the windows in step so that the
     window's estimates sit in each XCD's L2, the chains in registers (no carried state),
     a second sweep for the flows.
Gate: build only if a model gives <= 24 GB and <= 5.5 ms per round.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simgrid-flow-updating-implementation_amd"))

PEAK_GBS = 8000.0
SLICE = 1 << 14          # nodes per 128 KB slice of doubles (kernel 8 / 9 staging, LDS)
TR_BE = 8192             # kernel 9 transpose bucket (csrc/fu_tuning.h)
XCDS, CUS = 8, 256
CHAIN_NS = 7.2           # one exact chain element, one wave alone
L2_REQ_PER_S = XCDS * 16 * 2.4e9   # 16 L2 channels per XCD, one 64-B request per clock each


def classes(deg):
    """Row classes of kernel 9 (degree bounds) -> (name, mask)."""
    return [("isolated", deg == 0), ("light <=128", (deg >= 1) & (deg <= 128)),
            ("short 129-256", (deg > 128) & (deg <= 256)), ("mid 257-1024", (deg > 256) & (deg <= 1024)),
            ("heavy 1025-8192", (deg > 1024) & (deg <= 8192)), ("mega >8192", deg > 8192)]


def segments(rp, col, rows, shift):
    """(row, bucket) pairs with at least one edge, bucket = col >> shift, over `rows` (rows'
    neighbours sorted by id: a row's bucket sequence is non-decreasing)."""
    nseg = 0
    for r in rows:
        b = col[rp[r]:rp[r + 1]] >> shift
        nseg += 1 + int(np.count_nonzero(b[1:] != b[:-1])) if len(b) else 0
    return nseg


def sell_padding(rp, col, rows, shift, lanes=64):
    """Rows (sorted by degree) in waves of `lanes`; per window (col >> shift) a wave runs as
    many steps as its longest segment: padded slots / real edges."""
    nb = (int(col.max()) >> shift) + 1
    real = padded = 0
    for w0 in range(0, len(rows), lanes):
        grp = rows[w0:w0 + lanes]
        m = np.zeros((len(grp), nb), dtype=np.int64)
        for k, r in enumerate(grp):
            m[k] = np.bincount(col[rp[r]:rp[r + 1]] >> shift, minlength=nb)
        real += int(m.sum())
        padded += int(m.max(axis=0).sum()) * lanes
    return padded / max(real, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--out", default=None)
    ap.add_argument("--window-slices", type=int, default=16, help="alternative W: slices per window")
    a = ap.parse_args()
    import fu

    g = fu.Graph.rmat(a.scale, 16, seed=1)
    rp, col = g.rowptr, g.col
    n, E = g.n, g.E
    deg = np.diff(rp)
    P = (n + SLICE - 1) // SLICE
    alg = 24 * E + 28 * n
    rep = {"graph": f"rmat:scale={a.scale},ef=16,seed=1", "n": n, "E": E, "alg_bytes_per_round": alg,
           "slices": P}
    cls = {}
    for nm, m in classes(deg):
        cls[nm] = {"rows": int(m.sum()), "edges": int(deg[m].sum()), "edge_share": float(deg[m].sum() / E)}
    rep["classes"] = cls

    # ---- 1. kernel 9 as shipped, per launch: byte model vs PMC ------------------------------
    pmc = None
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
        for rec in json.load(f):
            if rec.get("n") == n and rec.get("E") == E and rec.get("kernel_selected") == "pregather":
                pmc = rec
    nbk = (E + TR_BE - 1) // TR_BE
    e_light = cls["light <=128"]["edges"]
    e_multi = cls["short 129-256"]["edges"] + cls["mid 257-1024"]["edges"] + cls["heavy 1025-8192"]["edges"]
    e_mega = cls["mega >8192"]["edges"]
    n_nz = n - cls["isolated"]["rows"]
    model = {
        "k_stage": {"fetch": 2 * E + n * 8, "write": 8 * E,
                    "what": "u16 column offsets in slice order + the slices into LDS / G_A (8 B per edge)"},
        "k_transpose": {"fetch": 8 * E + 2 * E + 4 * nbk * P, "write": 8 * E,
                        "what": "G_A + u16 positions + per-bucket run starts (buckets x slices x 4 B) / G_B"},
        "light tiles (k_round_recon)": {"fetch": 16 * e_light + 20 * n_nz, "write": 8 * e_light + 8 * n_nz,
                                        "what": "own flow + G_B per edge, rowptr / v / a_{r-2} per row / flow, a_r"},
        "k_heavy_multi (rows 129-8192, lag)": {"fetch": 24 * e_multi, "write": 8 * e_multi,
                                               "what": "chain pass: f, G_B; lagged flow pass: G_B of r-2 / f"},
        "mega hubs (chains + k_hub_flows)": {"fetch": 24 * e_mega, "write": 8 * e_mega,
                                             "what": "chains: f, G_B; k_hub_flows: f, G_B again / f"},
        "k_isolated": {"fetch": 12 * cls["isolated"]["rows"], "write": 8 * cls["isolated"]["rows"], "what": "v / a"},
    }
    tot_model = sum(v["fetch"] + v["write"] for v in model.values())
    rep["kernel9_model"] = {k: {"GB": (v["fetch"] + v["write"]) / 1e9, "what": v["what"]} for k, v in model.items()}
    rep["kernel9_model_total_GB"] = tot_model / 1e9
    if pmc:
        rep["kernel9_pmc_total_GB"] = pmc["bytes_per_launch"] / 1e9
        rep["kernel9_pmc_per_launch_GB"] = {x["kernel_filter"]: (x["fetch_bytes_per_round"] + x["write_bytes_per_round"]) / 1e9
                                            for x in pmc["per_launch_kind"]}
    t_meas_ms = 6.740  # BENCH_r05 rmat24_unit (driver), rounds 1-19
    rate = (pmc["bytes_per_launch"] if pmc else tot_model) / (t_meas_ms * 1e-3)
    rep["kernel9_measured"] = {"ms": t_meas_ms, "frac": alg / (t_meas_ms * 1e-3) / 1e9 / PEAK_GBS,
                               "traffic_rate_GBs": rate / 1e9, "record": "BENCH_r05.json rmat24_unit; profiles/pmc_traffic.json"}
    # the design's floor: staging (10 B) + transpose (18 B + run starts) + one pass over every row
    floor = (model["k_stage"]["fetch"] + model["k_stage"]["write"] + model["k_transpose"]["fetch"]
             + model["k_transpose"]["write"] + 24 * (E - 0) + 28 * n)
    rep["kernel9_floor"] = {"GB": floor / 1e9, "ms_at_measured_rate": floor / rate * 1e3,
                            "frac": alg / (floor / rate) / 1e9 / PEAK_GBS,
                            "what": "propagation blocking's 28 B per edge + every row in one pass (24 B per edge) "
                                    "+ 28 B per node, at the rate the shipped round streams its traffic"}

    rest_pb = lambda rest: (10 + 18) * rest + 24 * rest + 4 * nbk * P * rest / E  # noqa: E731
    per_cu = rate / CUS  # one CU's share of the streaming rate
    for lo in (256, 2048):
        rows = np.nonzero((deg > lo) & (deg <= 8192))[0]
        rows = rows[np.argsort(-deg[rows], kind="stable")]
        eh = int(deg[rows].sum())
        if eh == 0:  # a small graph may have no rows in this class
            continue
        nseg = segments(rp, col, rows, 14)
        hist = np.zeros(P, dtype=np.int64)
        for r in rows:
            hist += np.bincount(col[rp[r]:rp[r + 1]] >> 14, minlength=P)
        key = f"rows_{lo + 1}_8192"
        rep.setdefault("given_layout_heavy", {})[key] = {
            "rows": int(len(rows)), "edges": eh, "row_slice_segments": nseg,
            "edges_per_segment": eh / max(nseg, 1), "hottest_slice_share": float(hist.max() / hist.sum())}
        rest = E - eh

        # ---- 2. alternative S: slice-outer tasks, LDS slices, (S, T) carried -------------
        # per heavy edge: chain pass u16 offset 2 + f 8; flow pass 2 + f 8 + f write 8 = 28 B;
        # per (row, slice) segment: (S, T) written and read (32 B) + a descriptor (row, start:
        # 8 B) per pass; the other rows keep kernel 9 (staging 28 B + one pass 24 B per edge).
        s_bytes = 28 * eh + (32 + 16) * nseg + rest_pb(rest) + 28 * n
        # time: a row's exact chain meets its slices in order. Either one CU carries a row group
        # through all P slices (it streams the whole 8n-byte table into its LDS, per pass, at one
        # CU's share of the chip's rate), or the chain hops between CUs at every slice (>= 1 us per
        # hand-off through L2 / the fabric, P hops per pass): the cheaper of the two, twice
        walk = min(2 * 8 * n / per_cu, 2 * P * 1e-6)
        s_ms = max(s_bytes / rate, walk) * 1e3
        rep[f"alt_S_slice_outer_{key}"] = {
            "GB": s_bytes / 1e9, "ms_bytes_at_measured_rate": s_bytes / rate * 1e3,
            "ms_chain_walk_lower_bound": walk * 1e3, "ms": s_ms,
            "note": "carried (S, T) and descriptors: %.1f B per heavy edge; a chain walks %d slices in order "
                    "per pass: one CU streaming the table (%.2f ms per pass) or %d cross-CU hand-offs "
                    "(>= %.2f ms per pass)" % (48 * nseg / eh, P, 8 * n / per_cu * 1e3, P, P * 1e-3)}

        # ---- 3. alternative W: window sweep through L2, SELL-64 rows, chains in registers --
        ws = a.window_slices
        shift = 14 + int(np.log2(ws))
        pad = sell_padding(rp, col, rows, shift)
        table = XCDS * 8 * n * 2  # every XCD streams the whole table through its L2, twice
        w_bytes = (12 + 20) * eh * pad + table + rest_pb(rest) + 28 * n
        gathers = 2 * eh * pad
        w_ms = max(w_bytes / rate, gathers / L2_REQ_PER_S) * 1e3
        rep[f"alt_W_window_sweep_{key}"] = {
            "window_slices": ws, "sell64_padding": pad, "GB": w_bytes / 1e9, "GB_table_through_L2": table / 1e9,
            "ms_bytes_at_measured_rate": w_bytes / rate * 1e3, "ms_L2_gather_requests": gathers / L2_REQ_PER_S * 1e3,
            "ms_longest_chain_alone": int(deg.max()) * CHAIN_NS * 1e-6, "ms": w_ms,
            "note": "lower bounds: the byte time at the shipped round's streaming rate and the L2 request time "
                    "of the gathers; the window barriers, the gathers' L2 hit rate and the SELL chains' "
                    "latency hiding are not priced"}
    gate = {"GB": 24.0, "ms": 5.5}
    rep["gate"] = gate
    rep["verdict"] = {k: (rep[k]["GB"] <= gate["GB"] and rep[k]["ms"] <= gate["ms"])
                      for k in list(rep) if k.startswith("alt_")}
    txt = json.dumps(rep, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()

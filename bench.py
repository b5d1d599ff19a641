#!/usr/bin/env python3
"""Headline benchmark: directed-edge flow updates/s + % HBM roofline; rounds to 1e-9 error.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload auto|er|rgg-dist|pairwise|...]

N = 1 (default workload "er", BASELINE.json configs[1]): Erdos-Renyi G(n=1,000,000,
m=4,000,000), self-loops dropped, deduplicated, symmetrised (E ~ 8.0e6 directed edges); node
values U[0,100) (SplitMix64, seed 0); collect-all generation-synchronous rounds in fp64 on one
MI355X. A step = one round = Peer.on_receive for every directed edge + Peer.avg_and_send for
every node (flowupdating-collectall.py:93-128). The timed region is rounds 0 .. K-1 of the job
from the zero state, exactly the first K rounds of the BASELINE 1000-round run.

N > 1 (default workload "rgg-dist", BASELINE.json configs[4], weak scaling): one random
geometric graph of 2^23 nodes per GPU (avg degree 8), cut into x-slabs, one rank per GPU,
estimates-only RCCL halo exchange every round (fu_dist.hip). Without WORLD_SIZE in the
environment, `--gpus N` starts the N ranks itself (torch.distributed.run, 127.0.0.1) before
anything touches a GPU; a box with fewer than N visible GPUs is an error, never a silent
1-GPU line.

Setup outside the timed region: graph generation, handle creation, one autotune pass
(fu_tune: the candidate kernels timed on real rounds at the unpacked width), W warmup rounds
(in chunks, so the autotuner also sees every packing width the warmup reaches), fu_reset.
Timed: HIP events on the engine's stream around round 0 and every chunk, one host sync at the
end, between barriers; value = edge updates of all ranks / max-over-ranks wall time.

Printed by rank 0: ONE JSON line, with `roofline` (the round kernel's algorithmic bytes
24E + 28N per launch, §8(d), / the mean device time of rounds 1 .. K-1 from those events,
against 8 TB/s; `traffic` from the PMC passes in profiles/ when they match this command) and
`cpu_baseline` (the C port of the oracle on the host, single thread, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "simgrid-flow-updating-implementation_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md)
METRIC = "directed-edge flow updates/sec + % HBM roofline; rounds to 1e-9 error"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000, help="timed rounds (ticks for pairwise)")
    ap.add_argument("--warmup", type=int, default=400,
                    help="untimed rounds after the autotune pass (the autotuner also times the "
                         "candidates at every packing width these reach), then fu_reset")
    ap.add_argument("--n", type=int, default=0,
                    help="nodes (er: 1e6; rgg-dist: per GPU, 2^23; rmat: scale, 24; rr: 65536)")
    ap.add_argument("--m", type=int, default=4_000_000)
    ap.add_argument("--workload", default="auto",
                    choices=["auto", "er", "rgg", "rmat", "rr", "rgg-dist", "pairwise", "rgg-parts"],
                    help="auto = er at N = 1, rgg-dist at N > 1; rgg / rmat / rr = exploratory "
                         "single-GPU graphs; pairwise = RR-64K tick replay (BASELINE configs[2]); "
                         "rgg-parts = one GPU, RGG(--n, 2^28 by default) as --parts in-process "
                         "partitions (graphs beyond one handle's 2^31 directed edges)")
    ap.add_argument("--parts", type=int, default=2, help="rgg-parts: partitions on the one GPU")
    ap.add_argument("--deg", type=float, default=9.0,
                    help="rgg-parts: average degree (9: RGG 2^28 has 2.4e9 directed edges, beyond 2^31)")
    ap.add_argument("--kernel", default="auto")
    ap.add_argument("--layout", default="auto", choices=["auto", "given", "degree"],
                    help="device node numbering: degree = relabelled by degree (hot estimates "
                         "share cache lines; outputs keep the caller's numbering); auto = "
                         "degree for rmat, given otherwise")
    ap.add_argument("--conv-rounds", type=int, default=1000,
                    help="rounds of the (untimed) convergence run for rounds-to-1e-9")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target length of the CPU baseline sample (0 = skip)")
    ap.add_argument("--no-conv", action="store_true")
    ap.add_argument("--strong", action="store_true",
                    help="rgg-dist: strong scaling, --n nodes in all (2^26 by default) split over the ranks")
    ap.add_argument("--opt", action="append", default=[], metavar="KEY=VALUE",
                    help="engine option for the headline engine (fu_set_option; A/B runs)")
    ap.add_argument("--settle-ms", type=float, default=None,
                    help="untimed rounds run back to back right before a timed window, at least this "
                         "long (default 25 ms; at N > 1 a fixed round count, the same on every rank)")
    ap.add_argument("--no-unit", action="store_true",
                    help="N = 1 default line without its weak_scaling_unit (config 5's per-GPU RGG)")
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args) -> int:
    """--gpus N without a launcher: start N rank processes (one per GPU) as children and
    return their exit status. Runs before this process touches HIP."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] starting {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def chunk_bounds(steps: int, nchunk: int = 10):
    """Round 0 alone (the timeout fire on zero state), then rounds 1..K-1: one chunk up to
    100 rounds, else nchunk chunks (each event mark costs the stream ~6 us)."""
    if steps <= 1:
        return [0, steps]
    rest = steps - 1
    k = 1 if steps <= 100 else min(nchunk, rest)
    return [0] + [1 + rest * q // k for q in range(k + 1)]


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world != args.gpus:
        print(f"[bench] error: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr, flush=True)
        sys.exit(2)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo", init_method="env://", world_size=world, rank=rank)

    import fu

    print(f"[bench] rank {rank}/{world} (local {local})", file=sys.stderr, flush=True)
    ndev = fu.device_count()
    if ndev < local_world or ndev == 0:
        # never share a GPU between ranks or report a scaling line for GPUs that do not exist
        print(f"[bench] error: {local_world} rank(s) on this node need {local_world} GPU(s), "
              f"{ndev} visible", file=sys.stderr, flush=True)
        sys.exit(3)

    wl = args.workload
    if wl == "auto":
        wl = "er" if world == 1 else "rgg-dist"
    if wl == "rgg-dist":
        return run_dist(args, world, rank, local, dist)
    if wl == "pairwise" and world > 1:  # the tick replay does not shard: replicas
        return run_pairwise_replicas(args, world, rank, local, dist)
    if world > 1:
        print(f"[bench] error: workload {wl} is single-GPU (use rgg-dist at N > 1)", file=sys.stderr, flush=True)
        sys.exit(2)
    if wl == "pairwise":
        return run_pairwise(args)
    if wl == "rgg-parts":
        return run_parts(args)
    return run_single(args, wl)


def timed_rounds(eng, steps: int):
    """Rounds 0..steps-1 from the zero state; HIP event marks on the engine's stream around
    round 0 and each chunk, one host sync at the end. Returns (wall_s, per-chunk device ms,
    bounds)."""
    b = chunk_bounds(steps)
    ra = np.asarray(b, dtype=np.int32)  # ready before the clock starts
    eng.synchronize()
    t0 = time.perf_counter()
    # one host call for the whole window (fu_run_collectall_marked); mark 0 is round 0's own
    # start (the kernel's start event), not an event on the idle stream ahead of its dispatch
    eng.run_marked(ra)
    eng.synchronize()
    wall = time.perf_counter() - t0
    dev = [eng.elapsed(k, k + 1) for k in range(len(b) - 1)]
    return wall, dev, b


def roofline(alg_bytes: int, dev_ms, b, traffic=None, kernel=""):
    """Dominant kernel = the round kernel of rounds >= 1: its mean launch time from the
    events; round 0 (k_round0 + k_round0_flows) is reported beside it."""
    steps = b[-1]
    r1 = sum(dev_ms[1:]) / max(1, steps - 1) if steps > 1 else dev_ms[0]
    achieved = alg_bytes / (r1 * 1e-3) / 1e9
    whole = sum(dev_ms) / max(1, steps)
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "alg_bytes_per_launch": alg_bytes,
            "kernel": kernel, "avg_launch_us": r1 * 1e3, "launch_window": f"rounds 1-{steps - 1}",
            "round0_us": dev_ms[0] * 1e3, "whole_region_avg_round_us": whole * 1e3,
            "whole_region_frac": alg_bytes / (whole * 1e-3) / 1e9 / HBM_PEAK_GBS}


def round_kernels(kinfo):
    """The launches one round of the selected kernel consists of (the roofline's unit)."""
    k = kinfo["kernel"]
    if k == "recon":
        return "k_round_recon %dx%d" % (kinfo["tile"][0], kinfo["tile"][1])
    if k == "stage":
        return "k_stage + k_round_staged 1024x128"
    if k == "pregather":
        return ("k_stage + k_transpose (hub buckets, rest) + k_round_recon<PRE> 1024x128 (heavy rows, "
                "register-resident rows, light tiles) + mega-hub chains + k_hub_flows (side stream)")
    return k


def pmc_traffic(n, E, kernel_selected, steps, per_gpu=False):
    """HBM bytes per round from profiles/pmc_traffic.json (tools/pmc.sh + tools/make_pmc_traffic.py),
    only when it was measured on this graph, kernel and timed window. per_gpu: the rgg-dist
    record of the per-GPU slab (n = nodes per GPU; E not compared: it is the slab's)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        pmc = json.load(f)
    for rec in pmc if isinstance(pmc, list) else [pmc]:
        if rec.get("n") == n and (per_gpu or rec.get("E") == E) \
                and rec.get("kernel_selected") == kernel_selected and rec.get("rounds_timed") == steps:
            return rec.get("bytes_per_launch")
    return None


def make_graph(wl, n_arg, m_arg):
    """The single-GPU workloads' graphs (seeded): (graph, description)."""
    import fu

    if wl == "er":
        n = n_arg or 1_000_000
        return fu.Graph.erdos_renyi(n, m_arg, seed=1), f"er:n={n},m={m_arg} collect-all generation-synchronous rounds"
    if wl == "rgg":
        n = n_arg or (1 << 20)
        return fu.Graph.random_geometric(n, avg_deg=8.0, seed=1), f"rgg:n={n},deg=8 collect-all generation-synchronous rounds"
    if wl == "rmat":
        scale = n_arg or 24
        return fu.Graph.rmat(scale, 16, seed=1), f"rmat:scale={scale},ef=16 collect-all generation-synchronous rounds"
    n = n_arg or 65536
    return fu.Graph.random_regular(n, 8, seed=1), f"rr:n={n},d=8 collect-all generation-synchronous rounds"


SETTLE_MS = 25.0  # untimed rounds right before a timed window, at least this long (wall)


def prepare(eng, kernel, warmup, widths=None, tune=True, settle_ms=None):
    """Untimed setup: one autotune pass (kernel auto; tune=False: the engine was tuned at this
    width already), `warmup` rounds in chunks of 64 (the host sees each packing plan's width
    between calls, so the autotuner also covers every width the warmup reaches; winners are
    kept across fu_reset; at most four passes per engine), then rounds until the GPU has
    run at least settle_ms (default SETTLE_MS) of them back to back right before the window
    (with 5 warmup rounds of 60 us the chip starts the window cold: rounds 1-19 of ER-1M
    took 59.7 us against 58.1 after 25 ms of rounds, four alternating pairs,
    profiles/r05/ag), fu_reset. widths: a list that receives (rounds done, packing plan
    width) after each warmup chunk. Returns the settle rounds run."""
    if kernel == "auto" and tune:
        eng.tune()
    done = 0
    for w0 in range(0, warmup, 64):
        eng.run(min(64, warmup - w0))
        done += min(64, warmup - w0)
        eng.synchronize()
        if widths is not None:
            widths.append((done, eng.pack_widths()[2]))
    settle = SETTLE_MS if settle_ms is None else settle_ms
    n_settle, t0 = 0, time.perf_counter()
    while settle > 0 and (time.perf_counter() - t0) * 1e3 < settle:
        eng.run(16)
        eng.synchronize()
        n_settle += 16
    # the window's own host path once, untimed (rounds 0-1 from the zero state): its first
    # call in a process costs ~50 us of host time (profiles/r06/d: 1180 against 1148 us)
    eng.reset()
    eng.run_marked(np.asarray(chunk_bounds(2), dtype=np.int32))
    eng.synchronize()
    eng.reset()
    return n_settle


def measure_window(eng, g, steps):
    """The timed region (rounds 0..steps-1 from the zero state) of an engine already tuned and
    reset: wall time, per-chunk device times, the roofline of rounds 1..steps-1, the kernel
    that ran them."""
    wall, dev_ms, b = timed_rounds(eng, steps)
    kinfo = eng.info()
    kname = kinfo["kernel"]
    phases = [{"rounds": [b[k], b[k + 1]], "us_per_round": dev_ms[k] * 1e3 / max(1, b[k + 1] - b[k])}
              for k in range(len(b) - 1)]
    alg_bytes = 24 * g.E + 28 * g.n
    roof = roofline(alg_bytes, dev_ms, b, pmc_traffic(g.n, g.E, kname, steps), round_kernels(kinfo))
    ws = window_stats(g.n, g.E, kname, steps)
    if ws:  # an archived record of another run (possibly another tree): never this run's numbers
        roof["archived_window_profile"] = ws
    value_r1 = g.E * (steps - 1) / (sum(dev_ms[1:]) * 1e-3) if steps > 1 else None
    return wall, phases, roof, value_r1, kinfo, kname


def run_single(args, wl):
    import fu

    t_gen = time.perf_counter()
    g, desc = make_graph(wl, args.n, args.m)
    v = fu.uniform_values(g.n, seed=0)
    t_gen = time.perf_counter() - t_gen
    print(f"[bench] graph {desc}: n={g.n} E={g.E} generated in {t_gen:.1f} s", file=sys.stderr, flush=True)
    layout = args.layout if args.layout != "auto" else ("degree" if wl == "rmat" else "given")
    device = 0
    t_create = time.perf_counter()  # host CSR and values -> HBM, the launch plans, the tables
    eng = fu.CollectAll(g, v, device=device, kernel=args.kernel, layout=layout)
    eng.synchronize()
    t_create = time.perf_counter() - t_create
    for kv in args.opt:
        k, val = kv.split("=", 1)
        eng.set_option(k, int(val))
    t_setup = time.perf_counter()
    n_settle = prepare(eng, args.kernel, args.warmup, settle_ms=args.settle_ms)
    t_setup = time.perf_counter() - t_setup

    wall, phases, roof, value_r1, kinfo, kname = measure_window(eng, g, args.steps)
    t_down = time.perf_counter()  # the K-round job's result back to the host (fu_get_estimates)
    eng.estimates()
    t_down = time.perf_counter() - t_down
    t_down2 = time.perf_counter()  # again: a snapshot's cost once the bounce buffers exist
    eng.estimates()
    t_down2 = time.perf_counter() - t_down2
    pack_after = eng.pack_widths()[2]
    value = g.E * args.steps / wall
    host_io = {"create_s": t_create, "estimates_to_host_s": t_down, "estimates_to_host_again_s": t_down2,
               "host_bytes_in": 8 * (g.n + 1) + 4 * g.E + 8 * g.n, "host_bytes_out": 8 * g.n,
               "value_with_create_and_download": g.E * args.steps / (wall + t_create + t_down),
               "note": "not the metric: the handle is created once per job (fu_create: the CSR and values "
                       "cross PCIe, the launch plans are built on the host) and the estimates return once"}
    companions = args.workload == "auto" and not args.no_unit
    extra = {}
    if companions and args.steps != 1000:  # BASELINE config 2 as written, on the same engine
        extra["config2_1000"] = guarded("config2_1000", config2_1000, eng, g, args.kernel)

    conv = {"rounds_to_1e-9": None, "err_after_conv_rounds": None, "conv_rounds": None,
            "components": None}
    if not args.no_conv:  # rounds to 1e-9 vs the per-component means (untimed)
        conv = convergence(eng, g.rowptr, g.col, v, args.conv_rounds)
    eng.close()
    # the box's own streaming rate, measured in this run (untimed, after the timed region and
    # with the engine freed): a float4 copy of 1 GB, so a slow box shows as a slow copy as well
    # as a slow round
    try:
        roof["copy_GBs"] = fu.copy_bandwidth(device, 1 << 30, 5)
        roof["frac_of_copy"] = roof["achieved"] / roof["copy_GBs"]
    except Exception as ex:  # noqa: BLE001  (the headline line must survive)
        print(f"[bench] copy_bandwidth failed: {ex!r}", file=sys.stderr, flush=True)
        roof["copy_GBs"] = None
        roof["copy_error"] = repr(ex)
    cpu = cpu_baseline(g, v, args.cpu_seconds) if args.cpu_seconds > 0 else None
    out = {
        "metric": METRIC, "value": value, "unit": "edge-updates/s", "n_gpus": 1,
        "value_rounds_1_on": value_r1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall * 1e3 / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": f"synthetic (seeded {wl} graph, U[0,100) values)",
        "config": {
            "workload": desc, "n": g.n, "E_directed": g.E, "max_deg": g.max_deg, "graph_seed": 1,
            "value_seed": 0, "rounds_timed": f"0-{args.steps - 1} from the zero state",
            "kernel": args.kernel, "layout": layout, "kernel_selected": kname,
            "tile_selected": kinfo["tile"], "autotune_passes": kinfo["tune_passes"],
            "autotune_us_per_round": kinfo["tune_us_per_round"],
            "autotune_winner_by_width": kinfo["tune_winner_by_width"],
            "pack_width_after": pack_after, "setup_s": t_setup, "phases": phases,
            "settle": {"rounds": n_settle, "ms": SETTLE_MS if args.settle_ms is None else args.settle_ms,
                       "note": "untimed rounds back to back right before the window (bench.prepare)"},
            "options": args.opt,
            "parallelism": "single GPU",
        },
        "roofline": roof, "cpu_baseline": cpu, "graph_gen_s": t_gen, "host_io": host_io,
    }
    out.update(conv)
    del g
    if companions:
        # BASELINE configs 5, 4 and 3 measured live beside the headline (each guarded: a
        # failure of a companion measurement must not lose the headline line)
        out["weak_scaling_unit"] = guarded("weak_scaling_unit", weak_unit, args)
        out["rmat24_unit"] = guarded("rmat24_unit", rmat24_unit, args)
        out["pairwise_unit"] = guarded("pairwise_unit", pairwise_unit, args)
    out.update(extra)
    print(json.dumps(out), flush=True)


def guarded(name, fn, *a):
    t = time.perf_counter()
    try:
        r = fn(*a)
    except Exception as ex:  # noqa: BLE001
        print(f"[bench] {name} failed: {ex!r}", file=sys.stderr, flush=True)
        return {"error": repr(ex)}
    r["wall_s"] = time.perf_counter() - t
    print(f"[bench] {name}: {r.get('wall_s'):.1f} s", file=sys.stderr, flush=True)
    return r


def config2_1000(eng, g, kernel):
    """BASELINE config 2 as written (ER-1M, 1000 rounds) on the headline's engine: an untimed
    400-round pass in chunks (the autotuner sees the 32-, 16- and 8-bit packing widths; the
    width schedule is recorded), fu_reset, then rounds 0-999 timed from the zero state
    without any error check, HIP events around round 0 and ten chunks."""
    widths = []
    eng.reset()  # the width schedule is counted from the zero state, as in the timed run
    prepare(eng, kernel, 400, widths, tune=False)  # the headline's pass covered width 0
    wall, phases, roof, value_r1, info, kname = measure_window(eng, g, 1000)
    sched, last = [], None
    for r, w in widths:  # rounds at which the plan's width changed (deterministic: the same
        if w != last:    # rounds and values give the same plans in the timed run)
            sched.append({"from_round_le": r, "width": w})
            last = w
    return {"workload": "er:n=%d,m=%d, rounds 0-999 from the zero state (BASELINE config 2)" % (g.n, g.E // 2),
            "value": g.E * 1000 / wall, "unit": "edge-updates/s", "ms_total": wall * 1e3,
            "value_rounds_1_on": value_r1, "avg_round_us": roof["avg_launch_us"], "frac": roof["frac"],
            "roofline": roof, "phases": phases, "pack_width_schedule": sched,
            "autotune_winner_by_width": info["tune_winner_by_width"],
            "note": "measured in this run; the 20-round headline window is rounds 0-19 of this job"}


def rmat24_unit(args):
    """BASELINE config 4 (R-MAT scale 24, ef 16, degree layout) beside the headline: kernel
    auto tuned outside the window (kernel 9 wins), 20 rounds timed from the zero state."""
    import fu

    steps = 20
    t = time.perf_counter()
    g, desc = make_graph("rmat", 24, 0)
    v = fu.uniform_values(g.n, seed=0)
    t_gen = time.perf_counter() - t
    eng = fu.CollectAll(g, v, device=0, kernel="auto", layout="degree")
    try:
        prepare(eng, "auto", 2)
        wall, phases, roof, value_r1, kinfo, kname = measure_window(eng, g, steps)
    finally:
        eng.close()
    return {"workload": desc + ", degree layout (BASELINE config 4)", "n": g.n, "E_directed": g.E,
            "max_deg": g.max_deg, "value": g.E * steps / wall, "unit": "edge-updates/s",
            "value_rounds_1_on": value_r1, "steps": steps, "ms_per_step": wall * 1e3 / steps,
            "kernel_selected": kname, "autotune_us_per_round": kinfo["tune_us_per_round"],
            "avg_round_us": roof["avg_launch_us"], "frac": roof["frac"], "traffic": roof["traffic"],
            "roofline": roof, "phases": phases, "graph_gen_s": t_gen}


def pairwise_unit(args):
    """BASELINE config 3 beside the headline: RR-64K pairwise tick replay, ticks 101-500."""
    a = argparse.Namespace(**vars(args))
    a.n, a.steps, a.warmup, a.cpu_seconds = 0, 400, 50, 0
    line = pairwise_line(a)
    return {"workload": line["config"]["workload"], "value": line["value"], "unit": line["unit"],
            "ms_per_step": line["ms_per_step"],
            "us_per_tick": line["roofline"]["avg_launch_us"] / a.steps,  # device time (HIP events)
            "frac": line["roofline"]["frac"], "traffic": line["roofline"]["traffic"],
            "roofline": line["roofline"], "pairwise_updates": line["config"]["pairwise_updates"]}


def dist_line(*, world, steps, warmup, wall, dev1_ms, e_tot, n_tot, halo, n_total, per, kinfo,
              halo_us, round_us, t_gen, conv, strong=False, rccl_parity=None, traffic=None):
    """The N > 1 (rgg-dist) JSON line. Per GPU and round the algorithmic bytes are the §8(d)
    figure of the rank's rows (24 E + 28 N) plus the halo: 8 B per ghost estimate received
    (the RCCL payload written into the ghost slots; halo = ghost slots over all ranks)."""
    alg = (24 * e_tot + 28 * n_tot + 8 * halo) // world  # per GPU, per round
    r1 = dev1_ms / max(1, steps - 1)
    achieved = alg / (r1 * 1e-3) / 1e9
    line = {
        "metric": METRIC, "value": e_tot * steps / wall, "unit": "edge-updates/s",
        "n_gpus": world, "steps": steps, "warmup": warmup,
        "ms_per_step": wall * 1e3 / steps, "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (seeded RGG, U[0,100) values)",
        "config": {"workload": f"rgg-dist:n={n_total} ({per} per GPU{', strong scaling' if strong else ''}), "
                               "deg=8, x-slabs, "
                               "RCCL estimates-only halo every round",
                   "n_total": n_total, "E_directed": e_tot,
                   "rounds_timed": f"0-{steps - 1} from the zero state",
                   "kernel_selected": kinfo["kernel"], "tile_selected": kinfo["tile"],
                   "halo_estimates_per_round": halo, "halo_bytes_per_round": 8 * halo,
                   "parallelism": f"graph partition x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "per_gpu": True,
                     # HBM bytes per GPU and round from the PMC passes of this window on the
                     # partitioned path (profiles/pmc_traffic.json, measured at one rank: the
                     # same kernels on the same per-GPU slab; the halo adds 8 B per ghost)
                     "traffic": traffic,
                     "alg_bytes_per_launch": alg, "avg_launch_us": r1 * 1e3,
                     "kernel": "k_round_recon (heavy, boundary tiles) -> k_pack + RCCL group on the "
                               "comm stream beside the interior tiles",
                     "launch_window": f"rounds 1-{steps - 1}, max over ranks, the last halo included "
                                      "(events inside the timed region)"},
        # halo: device time on the comm stream from the start of the pack (boundary tiles
        # done) to the ghost slots written, max over ranks; it overlaps the interior tiles
        "halo": {"us_per_round": halo_us, "share_of_round": (halo_us / round_us) if round_us else None,
                 "overlapped_with": "interior tiles of the same round",
                 "sample": "20 rounds after the timed region (outside it), one halo read per round"},
        # the RCCL halo's correctness, checked in this run before the timed region
        "rccl_parity": rccl_parity["status"] if rccl_parity else ("n/a (one rank: no halo)" if world == 1 else None),
        "rccl_parity_check": rccl_parity,
        "cpu_baseline": None,
        "cpu_baseline_note": "reported on the N = 1 line only (rank 0 at N = 1)",
        "graph_gen_s": t_gen,
        "value_per_gpu": e_tot * steps / wall / world,
    }
    line.update(conv)
    return line


def window_stats(n, E, kernel_selected, steps):
    """The kernel-trace record of this exact window (tools/window_stats.py over a rocprofv3
    --kernel-trace of the same command, committed under profiles/), when one matches: the
    per-kernel mean durations and the window's round time, from which the roofline fraction
    can be recomputed."""
    import glob

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "*window_stats.json")), reverse=True):
        try:
            with open(path) as f:
                rec = json.load(f)
        except (OSError, ValueError):
            continue
        if rec.get("n") == n and rec.get("E") == E and rec.get("kernel_selected") == kernel_selected \
                and rec.get("rounds_timed") == steps:
            return {"file": os.path.relpath(path, ROOT), "avg_round_us": rec.get("avg_round_us"),
                    "frac": rec.get("frac"), "per_kernel": rec.get("per_kernel_per_round"),
                    "box_copy_GBs": rec.get("copy_GBs"), "commit": rec.get("commit"),
                    "note": "archival: the kernel-trace record of this window committed under profiles/ "
                            "(another run, maybe another tree and box), for recomputing the fraction from "
                            "tracked files; this run's own numbers are the fields above"}
    return None


def run_dist(args, world, rank, local, dist):
    """BASELINE config 5 (weak scaling): RGG with --n nodes per GPU (2^23 by default), one
    global graph cut into x-slabs (fu_part_gen_rgg: no rank builds the global graph), kernel 4
    with the estimates-only RCCL halo. value = all ranks' edge updates / max-over-ranks time."""
    line = measure_dist(args, world, rank, local, dist)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def run_parts(args):
    """One GPU, one process: RGG(--n) cut into --parts x-slabs (fu_part_gen_rgg, no global
    graph), each an in-process partition (fu_dist_create_local: its own handle and streams on
    the same GPU, the halo copied into the neighbours' ghost slots on the comm streams beside
    the interior tiles, fu_dist_run_local). For graphs beyond one handle's 2^31 directed edges
    (RGG 2^28: 2.15e9). value = all partitions' edge updates / wall time of rounds 0..K-1."""
    import fu
    from fu.dist import DistCollectAll, RggPart, run_local

    n = args.n or (1 << 28)
    k = args.parts
    deg = args.deg
    t = time.perf_counter()
    parts = [RggPart(n, avg_deg=deg, seed=1, nparts=k, part=r) for r in range(k)]
    vals = [p.values(seed=0) for p in parts]
    t_gen = time.perf_counter() - t
    e_tot = sum(p.e_local for p in parts)
    print(f"[bench] rgg:n={n} as {k} partitions: E={e_tot} generated in {t_gen:.1f} s", file=sys.stderr, flush=True)
    t = time.perf_counter()
    engs = []
    for p, v in zip(parts, vals):
        engs.append(DistCollectAll(p.to_plan(), v, None, device=0))
    for e in engs:
        e.synchronize()
    t_create = time.perf_counter() - t
    if args.warmup:
        run_local(engs, args.warmup)
    for e in engs:
        e.reset()
    for e in engs:
        e.synchronize()
    for e in engs:
        e.mark(0)
    t = time.perf_counter()
    run_local(engs, args.steps)
    for e in engs:
        e.mark(1)
    for e in engs:
        e.synchronize()
    wall = time.perf_counter() - t
    dev_ms = max(e.elapsed(0, 1) for e in engs)  # each partition's stream, events around the window
    halo = sum(p.n_ghost_a for p in parts)
    alg = 24 * e_tot + 28 * n + 8 * halo
    per_round = dev_ms * 1e-3 / args.steps
    kinfo = engs[0].info()
    fr, tot = fu.mem_info(0)  # while the partitions are resident
    free = [fr / 2 ** 30, tot / 2 ** 30]
    for e in engs:
        e.close()
    line = {
        "metric": METRIC, "value": e_tot * args.steps / wall, "unit": "edge-updates/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall * 1e3 / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded RGG, U[0,100) values)",
        "config": {"workload": f"rgg-parts:n={n},deg={deg:g} as {k} in-process x-slab partitions on one GPU "
                               "(halo by device copies every round)",
                   "n": n, "E_directed": e_tot, "parts": k, "E_per_part": [p.e_local for p in parts],
                   "halo_estimates_per_round": halo, "kernel_selected": kinfo["kernel"],
                   "tile_selected": kinfo["tile"], "rounds_timed": f"0-{args.steps - 1} from the zero state",
                   "graph_gen_s": t_gen, "create_s": t_create, "hbm_free_total_GiB": free,
                   "parallelism": f"{k} partitions, one GPU"},
        "roofline": {"bound": "hbm", "achieved": alg / per_round / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": alg / per_round / 1e9 / HBM_PEAK_GBS, "traffic": None,
                     "alg_bytes_per_launch": alg, "avg_launch_us": per_round * 1e6,
                     "kernel": "k_round_recon per partition (own streams), halo copies on the comm streams",
                     "launch_window": f"rounds 0-{args.steps - 1} (round 0 included), the slowest partition's events"},
        "cpu_baseline": None,
    }
    print(json.dumps(line), flush=True)


def weak_unit(args):
    """The N = 1 line's companion: BASELINE config 5's per-GPU unit (RGG 2^23 through the
    partitioned path, one rank, the same steps and warmup), measured live in the same run, so
    that the driver's N > 1 lines (which run that workload) have their one-GPU counterpart."""
    a = argparse.Namespace(**vars(args))
    a.n, a.kernel, a.no_conv, a.strong = 0, "auto", True, False
    line = measure_dist(a, 1, 0, 0, None)
    return {"workload": line["config"]["workload"], "value": line["value"], "unit": line["unit"],
            "ms_per_step": line["ms_per_step"], "E_directed": line["config"]["E_directed"],
            "kernel_selected": line["config"]["kernel_selected"],
            "tile_selected": line["config"]["tile_selected"],
            "roofline_frac": line["roofline"]["frac"], "avg_round_us": line["roofline"]["avg_launch_us"],
            "note": "measured in this run: compare the driver's N > 1 lines (value_per_gpu) with this"}


def measure_dist(args, world, rank, local, dist):
    """One rgg-dist measurement; returns rank 0's JSON line (None on other ranks)."""
    import torch

    import fu
    from fu.dist import DistCollectAll, RggPart, unique_id

    if args.strong:  # BASELINE config 5 as written: 2^26 nodes in all, split over the ranks
        n_total = args.n or (1 << 26)
        per = n_total // world
    else:  # weak scaling: 2^23 nodes per GPU
        per = args.n or (1 << 23)
        n_total = per * world
    def shared_uid():
        if world == 1:
            return unique_id()
        buf = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            buf = torch.frombuffer(bytearray(unique_id()), dtype=torch.uint8)
        dist.broadcast(buf, 0)
        return bytes(buf.tolist())

    # correctness of the RCCL halo first (untimed, before the measured graph exists): a
    # small RGG over the same ranks against the single-GPU engine on rank 0, bitwise
    parity = rccl_parity(world, rank, local, dist, shared_uid) if world > 1 else None
    t = time.perf_counter()
    part = RggPart(n_total, avg_deg=8.0, seed=1, nparts=world, part=rank)
    v = part.values(seed=0)
    t_gen = time.perf_counter() - t
    uid = shared_uid()
    eng = DistCollectAll(part.to_plan(), v, uid, device=local, kernel=args.kernel)
    if args.kernel == "auto":
        eng.tune()  # collective: the same rounds on every rank
    if args.warmup:
        eng.run(args.warmup)
    # settle: a fixed round count (the same on every rank: each round is a halo exchange),
    # about SETTLE_MS of rounds for the 2^23-node slab (~0.3 ms per round)
    n_settle = 0 if args.settle_ms == 0 else 80
    if n_settle:
        eng.run(n_settle)
    eng.reset()
    eng.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    wall, dev_ms, b = timed_rounds(eng, args.steps)
    barrier()
    # the halo's device time per round (untimed): one round per call, then its halo events
    hs = []
    for _ in range(20):
        eng.run(1)
        hs.append(eng.halo_ms())
    halo_us = 1e3 * sum(hs) / len(hs)
    t3 = torch.tensor([wall, sum(dev_ms[1:]), halo_us, float(part.e_local), float(part.n_local),
                       float(part.n_ghost_a)], dtype=torch.float64)
    if dist is not None:
        mx = t3[:3].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t3[3:].clone()
        dist.all_reduce(sm)
        wall, dev1, halo_us = (float(x) for x in mx.tolist())
        e_tot, n_tot, halo = (int(x) for x in sm.tolist())
    else:
        dev1 = sum(dev_ms[1:])
        e_tot, n_tot, halo = part.e_local, part.n_local, part.n_ghost_a
    kinfo = eng.info()
    # rounds to 1e-9 against the per-component means (math.fsum over each component of the
    # global graph, joined across the ranks without any rank holding it; untimed), the
    # error all-reduced (max) over the ranks by RCCL every round
    conv = {"rounds_to_1e-9": None, "err_after_conv_rounds": None, "conv_rounds": None,
            "components": None}
    if not args.no_conv:
        conv = convergence_dist(eng, part, v, args.conv_rounds, rank, world, dist)
    line = None
    if rank == 0:
        traffic = pmc_traffic(per, None, "rgg-dist", args.steps, per_gpu=True) if not args.strong else None
        line = dist_line(world=world, steps=args.steps, warmup=args.warmup, wall=wall, dev1_ms=dev1,
                         e_tot=e_tot, n_tot=n_tot, halo=halo, n_total=n_total, per=per, kinfo=kinfo,
                         halo_us=halo_us, round_us=1e3 * dev1 / max(1, args.steps - 1), t_gen=t_gen,
                         conv=conv, strong=args.strong, rccl_parity=parity, traffic=traffic)
        line["config"]["settle_rounds"] = n_settle  # untimed, right before the window, every rank
    eng.close()
    return line


def convergence_dist(eng, part, v, rounds, rank, world, dist):
    """convergence() for one rank of a partitioned graph: the per-component means from
    fu.dist.component_means_dist (bitwise those of the global graph), each rank's slice as
    its targets, one untimed run with the error check every round (RCCL max over ranks)."""
    from fu.dist import component_means_dist

    tgt, ncomp = component_means_dist(part.n_local, part.rowptr, part.col, part.send_a_off,
                                      part.send_a_idx, part.recv_a_off, v, rank, world, dist)
    eng.reset()
    eng.set_targets(tgt)
    tr = eng.run(rounds, err_every=1)
    below = np.nonzero(tr < 1e-9)[0]
    return {"rounds_to_1e-9": int(below[0]) + 1 if len(below) else None,
            "err_after_conv_rounds": float(tr[-1]), "conv_rounds": rounds, "components": int(ncomp)}


RCCL_PARITY_N = 1 << 18     # nodes of the parity graph (all ranks together)
RCCL_PARITY_ROUNDS = 30


def parity_verdict(a_parts, f_parts, a_ref, f_ref):
    """Rank 0's comparison of the gathered partitioned run with the single-GPU engine:
    (True, "bitwise") or (False, what differs)."""
    a = np.concatenate(a_parts)
    f = np.concatenate(f_parts)
    if a.shape != a_ref.shape or f.shape != f_ref.shape:
        return False, f"shape: estimates {a.shape} vs {a_ref.shape}, flows {f.shape} vs {f_ref.shape}"
    bad_a = int(np.sum(a.view(np.uint64) != a_ref.view(np.uint64)))
    bad_f = int(np.sum(f.view(np.uint64) != f_ref.view(np.uint64)))
    if bad_a or bad_f:
        return False, f"{bad_a} estimates and {bad_f} flows differ from the single-GPU engine"
    return True, "bitwise"


def rccl_parity_arrays(world, rank, local, dist, shared_uid, n=RCCL_PARITY_N, rounds=RCCL_PARITY_ROUNDS):
    """Every rank runs its slab of RGG(n) through fu_dist_create + RCCL for `rounds` rounds
    (halo exchange every round); rank 0 gathers the estimates and flows and runs the same
    rounds on the global graph with the single-GPU engine (pinned to the C oracle by the
    -m gpu suite). Returns (a_parts, f_parts, a_ref, f_ref) on rank 0, None elsewhere."""
    import fu
    from fu.dist import DistCollectAll, RggPart

    part = RggPart(n, avg_deg=8.0, seed=11, nparts=world, part=rank)
    eng = DistCollectAll(part.to_plan(), part.values(seed=12), shared_uid(), device=local)
    eng.run(rounds)
    mine = (eng.estimates(), eng.flows())
    eng.close()
    got = [None] * world if rank == 0 else None
    if dist is not None:
        dist.gather_object(mine, got, dst=0)
    else:
        got = [mine]
    if rank != 0:
        return None
    g = fu.Graph.random_geometric(n, avg_deg=8.0, seed=11)
    ref = fu.CollectAll(g, fu.uniform_values(g.n, seed=12), device=local)
    ref.run(rounds)
    out = ([x[0] for x in got], [x[1] for x in got], ref.estimates(), ref.flows())
    ref.close()
    return out


def rccl_parity(world, rank, local, dist, shared_uid):
    """The N > 1 line's correctness bit for the RCCL halo (CA:74 get_async, CA:124 put_async
    become ncclRecv/ncclSend into ghost slots): "bitwise", or every rank exits with status 5."""
    arrs = rccl_parity_arrays(world, rank, local, dist, shared_uid)
    verdict = [None]
    if rank == 0:
        verdict = [parity_verdict(*arrs)]
    if dist is not None:
        dist.broadcast_object_list(verdict, src=0)
    ok, detail = verdict[0]
    if not ok:
        print(f"[bench] RCCL parity FAILED at {world} ranks (RGG n={RCCL_PARITY_N}, "
              f"{RCCL_PARITY_ROUNDS} rounds): {detail}", file=sys.stderr, flush=True)
        sys.exit(5)
    return {"status": detail, "graph": f"rgg:n={RCCL_PARITY_N},deg=8,seed=11 over {world} ranks",
            "rounds": RCCL_PARITY_ROUNDS,
            "against": "single-GPU engine on the global graph (rank 0), estimates and flows"}


def convergence(eng, rowptr, col, v, rounds):
    """Rounds to max |a - mean of the node's component| < 1e-9 (per-component means with
    math.fsum; the watcher's last_avg, CA:139-142), from an untimed run of `rounds` rounds
    from the zero state with the fused error check every round; the error reached if never."""
    import fu

    tgt, comp = fu.component_means(rowptr, col, v)
    eng.reset()
    eng.set_targets(tgt)
    tr = eng.run(rounds, err_every=1)
    below = np.nonzero(tr < 1e-9)[0]
    return {"rounds_to_1e-9": int(below[0]) + 1 if len(below) else None,
            "err_after_conv_rounds": float(tr[-1]), "conv_rounds": rounds,
            "components": int(comp.max()) + 1}


def pairwise_bytes(events, rowptr, tasks):
    """Algorithmic bytes of a slice of replay events (per event type):
    RECV 32 (message in 16, est + flow 16); FIRE_PW 8k + 56 (k flows summed, est, v, then
    flow/est/last writes and a 16-B message out; 136 B at k = 8 with its receive);
    FIRE_CA 48k + 16."""
    kind = events[:, 0]
    k_pw = events[kind == 2, 2].astype(np.int64)
    k_ca = events[kind == 1, 1].astype(np.int64)
    return int(32 * np.sum(kind == 0) + np.sum(8 * k_pw + 56) + np.sum(48 * k_ca + 16))


def run_pairwise(args):
    print(json.dumps(pairwise_line(args)), flush=True)


def run_pairwise_replicas(args, world, rank, local, dist):
    """Pairwise mode at N > 1: "replicas only" (the tick replay is latency-bound
    and is not sharded): every rank replays the same RR-64K trace on its own GPU, between
    barriers; value = the updates of all replicas / the slowest rank's wall time."""
    import torch

    line = pairwise_line(args, device=local, barrier=dist.barrier)
    t = torch.tensor([line["ms_per_step"] * args.steps * 1e-3, line["roofline"]["avg_launch_us"]],
                     dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        wall = float(t[0])
        upd = line["config"]["pairwise_updates"]
        line.update({"value": upd * world / wall, "n_gpus": world, "ms_per_step": wall * 1e3 / args.steps,
                     "value_per_gpu": upd / wall, "scaling": "weak", "cpu_baseline": None,
                     "cpu_baseline_note": "reported on the N = 1 line only"})
        line["config"]["parallelism"] = f"replicas x{world} (the tick replay does not shard)"
        line["roofline"]["per_gpu"] = True
        line["roofline"]["avg_launch_us_max_over_ranks"] = float(t[1])
        print(json.dumps(line), flush=True)
    dist.destroy_process_group()


def pairwise_line(args, device=0, barrier=None):
    """BASELINE config 3: pairwise mode on a 64K-node random regular graph (d = 8), the
    SimGrid event order (Peer.loop, mailbox rendez-vous; App. B) replayed on the GPU by the
    persistent dataflow kernel. A step = one tick (PW:69-84 for every actor); the timed ticks
    start after the 51-tick timeout that starts the exchanges (PW:86-91) and the warmup."""
    import fu

    n = args.n or 65536
    g = fu.Graph.random_regular(n, 8, seed=1)
    v = fu.uniform_values(g.n, seed=0)
    t0_tick = 51 + args.warmup
    ticks = t0_tick + args.steps
    t = time.perf_counter()
    tr = fu.Trace(g.rowptr, g.col, "pairwise", ticks, "rand:3")
    t_build = time.perf_counter() - t
    a = tr.arrays()
    tto, tasks, ev = a["tick_task_off"], a["tasks"], a["events"]
    e0, e1 = int(tasks[tto[t0_tick], 1]) if tto[t0_tick] < len(tasks) else len(ev), len(ev)
    win = ev[e0:e1]
    upd = int(np.sum(win[:, 0] == 2))
    alg = pairwise_bytes(win, a["rowptr"], tasks)
    rep = fu.Replay(tr, v, device=device, persistent=True)
    rep.run(t0_tick)
    if barrier:
        barrier()
    t = time.perf_counter()
    ms = rep.run_timed(ticks)
    wall = time.perf_counter() - t
    if barrier:
        barrier()
    rep.close()
    cpu = None
    if args.cpu_seconds > 0 and device == 0 and barrier is None:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import coracle

        t = time.perf_counter()
        coracle.replay(a["rowptr"], v, tto, tasks, ev, a["out_ids"], tr.n_msgs)
        dt = time.perf_counter() - t
        upd_all = int(np.sum(ev[:, 0] == 2))
        cpu = {"value": upd_all / dt, "unit": "flow-updates/s", "cores": 1, "kind": "port",
               "sample": f"oracle/fu_oracle.c replay of the same trace, all {ticks} ticks ({dt:.2f} s, 1 thread)"}
    return {
        "metric": METRIC, "value": upd / wall, "unit": "flow-updates/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall * 1e3 / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded random regular graph, U[0,100) values)",
        "config": {"workload": f"pairwise tick replay: rr:n={n},d=8, tie order rand:3, ticks "
                               f"{t0_tick}-{ticks - 1}, persistent dataflow kernel",
                   "events": int(len(win)), "pairwise_updates": upd, "trace_build_s": t_build},
        "roofline": {"bound": "hbm", "achieved": alg / (ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     # the PMC passes of this window (tools/pmc.sh, prof_target.py --pairwise
                     # WARMUP:STEPS), when they match it
                     "traffic": pmc_traffic(g.n, g.E, "pairwise", args.steps) if args.warmup == 50 else None,
                     "alg_bytes_per_launch": alg, "kernel": "k_replay_persist_reg",
                     "avg_launch_us": ms * 1e3, "launch_window": f"one launch, {args.steps} ticks"},
        "cpu_baseline": cpu}


def cpu_baseline(g, v, seconds):
    """C port of the oracle (oracle/fu_oracle.c) on the host, 1 thread, bounded sample:
    the same graph and values, steady-state rounds, about `seconds` of CPU work."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle

    a, f = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 1, nthreads=1)  # round 0
    t = time.perf_counter()
    coracle.ca_rounds(g.rowptr, g.col, g.rev, v, 2, a, f, nthreads=1)
    per = (time.perf_counter() - t) / 2
    rounds = max(2, int(seconds / max(per, 1e-6)))
    t = time.perf_counter()
    coracle.ca_rounds(g.rowptr, g.col, g.rev, v, rounds, a, f, nthreads=1)
    dt = time.perf_counter() - t
    # the same restatement with OpenMP across nodes (rows stay sequential), on the host cores
    # this process may use (16 on a gpurun box; os.cpu_count() reports the whole machine)
    try:
        mt = len(os.sched_getaffinity(0))
    except AttributeError:
        mt = os.cpu_count() or 1
    mt = max(1, min(mt, int(os.environ.get("OMP_NUM_THREADS", mt))))
    coracle.ca_rounds(g.rowptr, g.col, g.rev, v, 2, a, f, nthreads=mt)
    rounds_mt = max(4, int(rounds * 2))
    t = time.perf_counter()
    coracle.ca_rounds(g.rowptr, g.col, g.rev, v, rounds_mt, a, f, nthreads=mt)
    dt_mt = time.perf_counter() - t
    return {
        "value": g.E * rounds / dt, "unit": "edge-updates/s", "cores": 1,
        "cores_available": os.cpu_count(), "kind": "port",
        "sample": f"{rounds} collect-all rounds on the same graph ({dt:.1f} s, oracle/fu_oracle.c, "
                  f"gcc -O2, single thread like SimGrid's DES)",
        "multicore": {"value": g.E * rounds_mt / dt_mt, "cores": mt,
                      "sample": f"{rounds_mt} rounds ({dt_mt:.1f} s), OpenMP across nodes"},
    }


if __name__ == "__main__":
    main()

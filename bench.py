#!/usr/bin/env python3
"""Headline benchmark: directed-edge flow updates/s + % HBM roofline; rounds to 1e-9 error.

Workload (BASELINE.json configs[1]): Erdos-Renyi G(n=1,000,000, m=4,000,000), self-loops
dropped, deduplicated, symmetrised (E ~ 8.0e6 directed edges); node values U[0,100)
(SplitMix64, seed 0); collect-all generation-synchronous rounds in fp64 on one MI355X.
A "step" = one round = Peer.on_receive for every directed edge + Peer.avg_and_send for
every node (flowupdating-collectall.py:93-128) = one launch of the round kernel.

    python bench.py [--gpus N] [--steps K] [--warmup W]

At N > 1 (torch.distributed.run, one process per GPU) every rank runs its own ER-1M
instance (graph seed 1 + rank), the weak-scaling "independent graphs" mode: the ER graph
has no locality, so partitioning it would put ~7/8 of its edges on the halo.
Ranks synchronise with a barrier around the timed region; time = max over ranks; value =
edge updates of all ranks / that time. torch.distributed (gloo, CPU) is used only for the
barrier and the max; the hot path is libfu.so.

Printed by rank 0: ONE JSON line (contract in the task statement), with `roofline` (the
round kernel's algorithmic bytes 24E + 28N per launch / average launch time from HIP
events on the library's stream, against 8 TB/s) and `cpu_baseline` (the C port of the
oracle on the host, single thread, on a bounded sample of the same workload).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "simgrid-flow-updating-implementation_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000, help="timed rounds")
    ap.add_argument("--warmup", type=int, default=400,
                    help="untimed rounds first: the autotuner times the candidate kernels at every "
                         "packing width the run reaches (0, 32, 16, 8 bits), then fu_reset")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--m", type=int, default=4_000_000)
    ap.add_argument("--workload", default="er", choices=["er", "rgg", "rmat", "rr", "rgg-dist"],
                    help="er = the headline ER-1M (default); others are exploratory: rgg "
                         "(--n nodes, avg deg 8), rmat (scale = --n, edge factor 16), rr (d = 8), "
                         "rgg-dist (ONE random geometric graph of --n nodes per GPU, partitioned "
                         "into slabs across the ranks, RCCL halo exchange every round)")
    ap.add_argument("--kernel", default="auto")
    ap.add_argument("--layout", default="auto", choices=["auto", "given", "degree"],
                    help="device node numbering: degree = relabelled by degree (hot estimates "
                         "share cache lines; outputs keep the caller's numbering); auto = "
                         "degree for rmat, given otherwise")
    ap.add_argument("--tile-edges", type=int, default=0, help="kernel 4 tile (2048/1024/512); 0 = default")
    ap.add_argument("--pack-every", type=int, default=0, help="rounds between packing plans; 0 = engine default (16)")
    ap.add_argument("--conv-rounds", type=int, default=1000,
                    help="rounds of the (untimed) convergence run for rounds-to-1e-9")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target length of the CPU baseline sample (0 = skip)")
    ap.add_argument("--no-conv", action="store_true")
    return ap.parse_args()


def round_kernels(kinfo):
    """The launches one round of the selected kernel consists of (the roofline's unit)."""
    k = kinfo["kernel"]
    if k == "recon":
        return "k_round_recon %dx%d%s" % (kinfo["tile"][0], kinfo["tile"][1], "+nt" if kinfo["nt"] else "")
    if k == "stage":
        return "k_stage + k_round_staged 1024x128"
    if k == "pipe_stage":
        return "k_stage + k_round_pipe<staged> 1024x128"
    if k == "pipe":
        return "k_round_pipe<recon> 1024x128"
    if k == "split2":
        return "k_gather_part0 + k_round_split"
    return k


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        dist.init_process_group("gloo", init_method="env://", world_size=world, rank=rank)

    import fu

    # one rank per GPU; on a box with fewer GPUs than ranks (a functional check of the N > 1
    # path) ranks share devices round-robin
    ndev = fu.device_count()
    if ndev > 0:
        local = local % ndev

    def barrier():
        if dist is not None:
            dist.barrier()

    def allmax(x: float) -> float:
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    if args.workload == "rgg-dist":
        return run_dist(args, world, rank, local, dist, barrier, allmax)
    t_gen = time.perf_counter()
    if args.workload == "er":
        g = fu.Graph.erdos_renyi(args.n, args.m, seed=1 + rank)
        wl = f"er:n={args.n},m={args.m} collect-all generation-synchronous rounds"
    elif args.workload == "rgg":
        g = fu.Graph.random_geometric(args.n, avg_deg=8.0, seed=1 + rank)
        wl = f"rgg:n={args.n},deg=8 collect-all generation-synchronous rounds"
    elif args.workload == "rmat":
        g = fu.Graph.rmat(args.n, 16, seed=1 + rank)
        wl = f"rmat:scale={args.n},ef=16 collect-all generation-synchronous rounds"
    else:
        g = fu.Graph.random_regular(args.n, 8, seed=1 + rank)
        wl = f"rr:n={args.n},d=8 collect-all generation-synchronous rounds"
    v = fu.uniform_values(g.n, seed=0)
    t_gen = time.perf_counter() - t_gen
    print(f"[bench] graph {wl}: n={g.n} E={g.E} generated in {t_gen:.1f} s", file=sys.stderr, flush=True)
    layout = args.layout if args.layout != "auto" else ("degree" if args.workload == "rmat" else "given")
    eng = fu.CollectAll(g, v, device=local, kernel=args.kernel, layout=layout)
    if args.tile_edges:
        eng.set_option("tile_edges", args.tile_edges)
    if args.pack_every:
        eng.set_option("pack_every", args.pack_every)
    # with kernel "auto" the warmup rounds also pick the kernel for each packing width; run in
    # chunks so the host sees each plan's width (an asynchronous copy) while the rounds run
    # (a pass needs 9 rounds per candidate within one call)
    for w0 in range(0, args.warmup, 64):
        eng.run(min(64, args.warmup - w0))
        eng.synchronize()
    eng.reset()           # the timed region is rounds 0 .. steps-1 from the zero state
    eng.synchronize()

    # Timed in <= 10 chunks (HIP events on the engine's own stream) to show how the round
    # time evolves: the packed estimate table engages as the estimates converge, and the
    # autotuner re-runs (on real rounds, inside the timed region) when its width changes.
    nchunk = min(10, args.steps)
    bounds = [args.steps * k // nchunk for k in range(nchunk + 1)]
    barrier()
    eng.synchronize()
    t0 = time.perf_counter()
    chunk_ms, chunk_pack = [], []
    for k in range(nchunk):
        chunk_ms.append(eng.run_timed(bounds[k + 1] - bounds[k]))
        chunk_pack.append(eng.pack_widths()[2])
    eng.synchronize()
    t1 = time.perf_counter()
    barrier()
    wall = allmax(t1 - t0)
    kern_ms = allmax(sum(chunk_ms))
    kinfo = eng.info()
    phases = [{"rounds": [bounds[k], bounds[k + 1]],
               "us_per_round": chunk_ms[k] * 1e3 / max(1, bounds[k + 1] - bounds[k]),
               "pack_width_after": chunk_pack[k]} for k in range(nchunk)]

    edges_total = g.E  # every rank has its own graph (seed 1 + rank): sum their edges
    if dist is not None:
        te = torch.tensor([float(g.E)], dtype=torch.float64)
        dist.all_reduce(te)
        edges_total = int(te.item())
    value = edges_total * args.steps / wall
    ms_per_step = wall * 1e3 / args.steps
    # roofline of the dominant round kernel (one launch per round): its average launch time
    # is the mean round time over the second half of the timed region, where the autotuned
    # kernel runs alone (plus the packing plan every 16 rounds, so this is conservative);
    # the whole-region average (incl. the unpacked early rounds and autotune passes) beside it
    alg_bytes = 24 * g.E + 28 * g.n
    avg_round_s = kern_ms / 1e3 / args.steps
    tail = phases[len(phases) // 2:]
    dom_s = sum(p["us_per_round"] * (p["rounds"][1] - p["rounds"][0]) for p in tail) * 1e-6 / \
        max(1, sum(p["rounds"][1] - p["rounds"][0] for p in tail))
    achieved = alg_bytes / dom_s / 1e9

    # rounds to 1e-9 vs the per-component means (untimed)
    rounds_to = None
    final_err = None
    if not args.no_conv:
        tgt, comp = fu.component_means(g.rowptr, g.col, v)
        eng.reset()
        eng.set_targets(tgt)
        tr = eng.run(args.conv_rounds, err_every=1)
        below = np.nonzero(tr < 1e-9)[0]
        rounds_to = int(below[0]) + 1 if len(below) else None
        final_err = float(tr[-1])
        n_comp = int(comp.max()) + 1

    out = None
    if rank == 0:
        cpu = None
        if world == 1 and args.cpu_seconds > 0:
            cpu = cpu_baseline(g, v, args.cpu_seconds)
        traffic = None
        pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc_path):
            with open(pmc_path) as f:
                pmc = json.load(f)
            if pmc.get("n") == g.n and pmc.get("E") == g.E and pmc.get("kernel") == args.kernel and \
                    pmc.get("kernel_selected") == kinfo["kernel"]:
                traffic = pmc.get("bytes_per_launch")  # per round, all of the round's launches
        out = {
            "metric": "directed-edge flow updates/sec + % HBM roofline; rounds to 1e-9 error",
            "value": value,
            "unit": "edge-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic (seeded {args.workload} graph, U[0,100) values)",
            "config": {
                "workload": wl,
                "n": g.n, "E_directed": g.E, "max_deg": g.max_deg, "graph_seed": "1+rank",
                "value_seed": 0, "rounds_timed": args.steps, "kernel": args.kernel, "layout": layout,
                "kernel_selected": kinfo["kernel"] + ("+nt" if kinfo["nt"] else ""),
                "tile_selected": kinfo["tile"],
                "autotune_passes": kinfo["tune_passes"],
                "autotune_us_per_round": kinfo["tune_us_per_round"],
                "autotune_winner_by_width": kinfo["tune_winner_by_width"],
                "phases": phases,
                "parallelism": "independent graph per GPU" if world > 1 else "single GPU",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "alg_bytes_per_launch": alg_bytes,
                "kernel": round_kernels(kinfo),
                "avg_launch_us": dom_s * 1e6,
                "launch_window": "rounds %d-%d" % (tail[0]["rounds"][0], tail[-1]["rounds"][1]),
                "whole_region_avg_round_us": avg_round_s * 1e6,
                "whole_region_frac": alg_bytes / avg_round_s / 1e9 / HBM_PEAK_GBS,
            },
            "cpu_baseline": cpu,
            "rounds_to_1e-9": rounds_to,
            "err_after_conv_rounds": final_err,
            "conv_rounds": args.conv_rounds,
            "components": None if args.no_conv else n_comp,
            "graph_gen_s": t_gen,
        }
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def run_dist(args, world, rank, local, dist, barrier, allmax):
    """BASELINE config 5 (weak scaling): RGG with --n nodes per GPU, one global graph split
    into slabs (fu_part_gen_rgg, no rank builds the global graph), kernel 4 with the
    estimates-only RCCL halo. value = all ranks' edge updates / max-over-ranks time."""
    import fu  # noqa: F401
    from fu.dist import DistCollectAll, RggPart, unique_id

    n_total = args.n * world
    t = time.perf_counter()
    part = RggPart(n_total, avg_deg=8.0, seed=1, nparts=world, part=rank)
    v = part.values(seed=0)
    t_gen = time.perf_counter() - t
    if world > 1:
        import torch

        buf = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            buf = torch.frombuffer(bytearray(unique_id()), dtype=torch.uint8)
        dist.broadcast(buf, 0)
        uid = bytes(buf.tolist())
    else:
        uid = unique_id()
    eng = DistCollectAll(part.to_plan(), v, uid, device=local, kernel="auto")
    eng.run(args.warmup)
    eng.synchronize()
    barrier()
    eng.synchronize()
    t0 = time.perf_counter()
    kern_ms = eng.run_timed(args.steps)
    eng.synchronize()
    t1 = time.perf_counter()
    barrier()
    wall = allmax(t1 - t0)
    kern_ms = allmax(kern_ms)
    e_tot = part.e_local
    if dist is not None:
        import torch

        te = torch.tensor([float(part.e_local), float(part.n_local), float(part.n_ghost_a)],
                          dtype=torch.float64)
        dist.all_reduce(te)
        e_tot = int(te[0].item())
        n_tot, halo = int(te[1].item()), int(te[2].item())
    else:
        n_tot, halo = part.n_local, part.n_ghost_a
    alg = 24 * e_tot + 28 * n_tot
    kinfo = eng.info()
    if rank == 0:
        avg_s = kern_ms / 1e3 / args.steps
        achieved = alg / avg_s / 1e9 / world  # per GPU, against one GPU's peak
        print(json.dumps({
            "metric": "directed-edge flow updates/sec + % HBM roofline; rounds to 1e-9 error",
            "value": e_tot * args.steps / wall, "unit": "edge-updates/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall * 1e3 / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded RGG, U[0,100) values)",
            "config": {"workload": f"rgg-dist:n={n_total} ({args.n} per GPU), deg=8, slabs, "
                                   "RCCL estimates-only halo", "E_directed": e_tot,
                       "kernel_selected": kinfo["kernel"], "tile_selected": kinfo["tile"],
                       "halo_estimates_per_round": halo, "parallelism": f"graph partition x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "alg_bytes_per_launch": alg // world, "avg_launch_us": avg_s * 1e6},
            "cpu_baseline": None, "graph_gen_s": t_gen}), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(g, v, seconds):
    """C port of the oracle (oracle/fu_oracle.c) on the host, 1 thread, bounded sample:
    the same ER-1M graph and values, steady-state rounds, about `seconds` of CPU work."""
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
        "value": g.E * rounds / dt,
        "unit": "edge-updates/s",
        "cores": 1,
        "cores_available": os.cpu_count(),
        "kind": "port",
        "sample": f"{rounds} steady-state collect-all rounds on the same ER-1M graph "
                  f"({dt:.1f} s, oracle/fu_oracle.c, gcc -O2, single thread like SimGrid's DES)",
        "multicore": {"value": g.E * rounds_mt / dt_mt, "cores": mt,
                      "sample": f"{rounds_mt} rounds ({dt_mt:.1f} s), OpenMP across nodes"},
    }


if __name__ == "__main__":
    main()

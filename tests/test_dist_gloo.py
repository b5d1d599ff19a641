"""Multi-rank partition + halo plan (fu.dist.partition), exercised on the CPU with
torch.distributed/gloo at world_size 2, 3 and 8 (the driver's scaling node).

Each rank runs the collect-all rounds on its local CSR in the ghost-slot numbering that
fu_dist_create consumes, and exchanges the halo exactly as fu_dist.hip does: it packs
send_*_idx in order and receives into the contiguous ghost ranges recv_*_off. The gathered
per-node estimates and flows must equal the single-process oracle bitwise, for both halo
contents: pull (ghost flows + ghost estimates) and recon (ghost estimates only). Only the
transport (RCCL instead of gloo) and the kernels differ on the GPU.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from fu.dist import partition, split_ranges


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rows(rowptr, fr, er, v):
    """Sequential row sums (CA:106-113) on per-edge fr/er; returns (a, f_new)."""
    n = len(rowptr) - 1
    a = np.empty(n)
    f = np.empty(len(fr))
    for i in range(n):
        b, e = rowptr[i], rowptr[i + 1]
        S = 0.0
        T = 0.0
        for k in range(b, e):
            S = S + fr[k]
            T = T + er[k]
        a[i] = ((v[i] - S) + T) / (e - b + 1)
        for k in range(b, e):
            f[k] = (fr[k] + a[i]) - er[k]
    return a, f


def _exchange(plan, src_local, ghost_out, send_off, send_idx, recv_off):
    """Pack send_idx from src_local per peer, receive into ghost_out[recv_off[p]:...]."""
    reqs = []
    for p in range(plan.nranks):
        if p == plan.rank:
            continue
        s = torch.from_numpy(np.ascontiguousarray(src_local[send_idx[send_off[p]:send_off[p + 1]]]))
        r = torch.empty(int(recv_off[p + 1] - recv_off[p]), dtype=torch.float64)
        if len(s):
            reqs.append(dist.isend(s, p))
        if len(r):
            reqs.append((dist.irecv(r, p), r, p))
    for q in reqs:
        if isinstance(q, tuple):
            q[0].wait()
            ghost_out[recv_off[q[2]]:recv_off[q[2] + 1]] = q[1].numpy()
        else:
            q.wait()


def _worker(rank, world, port, rowptr, col, rev, v, rounds, mode, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    plan = partition(rowptr, col, rev, world, rank)
    nl, el = plan.n_local, plan.e_local
    rp = plan.rowptr
    vl = v[plan.lo:plan.hi]
    deg = np.diff(rp)
    src = np.repeat(np.arange(nl), deg)
    # round 0 (CA:87-91)
    a = ((vl - 0.0) + 0.0) / (deg + 1)
    f = (0.0 + a[src]) - 0.0
    a_ext = np.zeros(nl + plan.n_ghost_a)
    f_ext = np.zeros(el + plan.n_ghost_f)
    a_prev2 = np.zeros(nl)  # a_{r-2}; a_{-1} = 0.0
    F = np.full(el, -0.0)   # recon: f_{r-2}; f_{-1} = -0.0
    hist_f = [F, f.copy()]
    for r in range(1, rounds):
        a_ext[:nl] = a
        f_ext[:el] = f
        _exchange(plan, a, a_ext[nl:], plan.send_a_off, plan.send_a_idx, plan.recv_a_off)
        if mode == "pull":
            _exchange(plan, f, f_ext[el:], plan.send_f_off, plan.send_f_idx, plan.recv_f_off)
            fr = -f_ext[plan.rev]
            er = a_ext[plan.col]
        else:  # recon: rebuild -f_{r-1}[j->i] from f_{r-2}[i->j], a_{r-1}[j], a_{r-2}[i]
            er = a_ext[plan.col]
            fr = -(((-hist_f[0]) + er) - a_prev2[src])
        a_new, f_new = _rows(rp, fr, er, vl)
        a_prev2 = a
        hist_f = [hist_f[1], f_new]
        a, f = a_new, f_new
    out_q.put((rank, plan.lo, plan.hi, a, f))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("mode", ["pull", "recon"])
@pytest.mark.parametrize("kind", ["er", "rgg"])
def test_partitioned_rounds_match_oracle(world, mode, kind):
    import fu

    g = (fu.Graph.erdos_renyi(600, 2400, seed=4) if kind == "er"
         else fu.Graph.random_geometric(900, avg_deg=7, seed=4))
    v = fu.uniform_values(g.n, seed=2)
    rounds = 12
    a_ref, f_ref = oracle.ca_sync(g.rowptr, g.col, v, rounds)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, g.rowptr, g.col, g.rev, v, rounds,
                                               mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    a = np.empty(g.n)
    f = np.empty(g.E)
    for rank, lo, hi, al, fl in res:
        a[lo:hi] = al
        f[g.rowptr[lo]:g.rowptr[hi]] = fl
    assert np.array_equal(a, a_ref)
    assert np.array_equal(f, f_ref)


def test_plan_shapes_and_symmetry():
    import fu

    g = fu.Graph.random_geometric(3000, avg_deg=8, seed=9)
    world = 4
    plans = [partition(g.rowptr, g.col, g.rev, world, r) for r in range(world)]
    b = split_ranges(g.rowptr, world)
    assert b[0] == 0 and b[-1] == g.n
    for p in plans:
        for q in plans:
            if p.rank == q.rank:
                continue
            # what p sends to q is exactly what q expects from p, in q's slot order
            nf = p.send_f_off[q.rank + 1] - p.send_f_off[q.rank]
            assert nf == q.recv_f_off[p.rank + 1] - q.recv_f_off[p.rank]
            sent_gidx = p.send_f_idx[p.send_f_off[q.rank]:p.send_f_off[q.rank + 1]] + g.rowptr[p.lo]
            exp = q.ghost_f_gidx[q.recv_f_off[p.rank]:q.recv_f_off[p.rank + 1]]
            assert np.array_equal(sent_gidx, exp)
            sent_a = p.send_a_idx[p.send_a_off[q.rank]:p.send_a_off[q.rank + 1]] + p.lo
            exp_a = q.ghost_a_gid[q.recv_a_off[p.rank]:q.recv_a_off[p.rank + 1]]
            assert np.array_equal(sent_a, exp_a)
        # local numbering in range
        assert p.col.max() < p.n_local + p.n_ghost_a
        assert p.rev.max() < p.e_local + p.n_ghost_f


@pytest.mark.parametrize("nparts", [1, 2, 3, 5, 8])
def test_rgg_slab_generator_matches_global_and_partition(nparts):
    """fu_part_gen_rgg: each rank's slab (built without the global graph) has the global
    generator's rows, and the same ghost numbering / halo plan as fu.dist.partition with the
    same node ranges."""
    import fu
    from fu.dist import RggPart

    n, avg = 20000, 8.0
    g = fu.Graph.random_geometric(n, avg_deg=avg, seed=7)
    parts = [RggPart(n, avg_deg=avg, seed=7, nparts=nparts, part=p) for p in range(nparts)]
    assert parts[0].lo == 0 and parts[-1].hi == n
    bounds = [p.lo for p in parts] + [n]
    for p in parts:
        assert np.array_equal(p.rowptr, g.rowptr[p.lo:p.hi + 1] - g.rowptr[p.lo])
        assert np.array_equal(p.global_col(), g.col[g.rowptr[p.lo]:g.rowptr[p.hi]])
        ref = partition(g.rowptr, g.col, g.rev, nparts, p.part, bounds=bounds)
        assert np.array_equal(p.col, ref.col)
        assert np.array_equal(p.ghost_gid, ref.ghost_a_gid)
        assert np.array_equal(p.send_a_off, ref.send_a_off)
        assert np.array_equal(p.send_a_idx, ref.send_a_idx)
        assert np.array_equal(p.recv_a_off, ref.recv_a_off)
        assert np.array_equal(p.values(seed=3), fu.uniform_values(n, seed=3)[p.lo:p.hi])


def _cm_worker(rank, world, port, kind, n, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import fu
    from fu.dist import RggPart, component_means_dist

    if kind == "rgg":
        p = RggPart(n, avg_deg=3.0, seed=5, nparts=world, part=rank)
        v = p.values(seed=6)
        args = (p.n_local, p.rowptr, p.col, p.send_a_off, p.send_a_idx, p.recv_a_off)
        lo = p.lo
    else:
        g = fu.Graph.erdos_renyi(n, n, seed=5)  # average degree 2: many small components
        v = fu.uniform_values(g.n, seed=6)
        p = partition(g.rowptr, g.col, g.rev, world, rank)
        args = (p.n_local, p.rowptr, p.col, p.send_a_off, p.send_a_idx, p.recv_a_off)
        v, lo = v[p.lo:p.hi], p.lo
    mean, nc = component_means_dist(*args, v, rank, world, dist)
    out_q.put((rank, lo, mean, nc))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("kind", ["rgg", "er"])
def test_component_means_dist_bitwise(world, kind):
    """The N > 1 line's convergence targets: per-component exact means of a partitioned graph
    (each rank's own components + expansions, joined on rank 0 across the cut edges) equal
    fu.component_means on the global graph bitwise, with components that span several ranks
    (sparse RGG at average degree 3, ER at average degree 2)."""
    import fu

    n = 6000
    g = (fu.Graph.random_geometric(n, avg_deg=3.0, seed=5) if kind == "rgg"
         else fu.Graph.erdos_renyi(n, n, seed=5))
    v = fu.uniform_values(g.n, seed=6)
    ref, comp = fu.component_means(g.rowptr, g.col, v)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cm_worker, args=(r, world, port, kind, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = np.empty(g.n)
    for rank, lo, mean, nc in res:
        got[lo:lo + len(mean)] = mean
        assert nc == int(comp.max()) + 1
    assert np.array_equal(got, ref)
    assert len(np.unique(comp)) > 50  # many components, several across the cuts

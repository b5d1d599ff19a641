"""Multi-GPU collect-all: contiguous node-range partitions with a per-round halo exchange.

The reference simulates every node on one SimGrid host thread; its messages are mailbox
transfers (Mailbox.put_async CA:124, get_async CA:74). Here a graph that needs more than
one GPU (for memory or bandwidth) is split into contiguous node ranges, one per rank. A
message between nodes on different ranks becomes a slot in a packed halo buffer, moved once
per round by RCCL (fu_dist_create / fu_run_collectall; see fu_dist.hip).

`partition(rowptr, col, rev, nranks, rank)` builds one rank's local CSR in the ghost-slot
numbering that fu_dist_create expects:

* local rows = global nodes [lo, hi); local edge k = global edge rowptr[lo] + k;
* col[k] < n_local: a local node; col[k] = n_local + g: ghost estimate slot g. Ghosts are
  grouped by owner rank, and sorted by global id inside each group;
* rev[k] < e_local: a local edge; rev[k] = e_local + q: ghost flow slot q. Ghost flows are
  grouped by owner rank, and sorted by the global index of the remote edge inside each group;
* the send lists to rank p are this rank's edges into p's range (ascending global edge
  index) and this rank's nodes adjacent to p's range (ascending id). That is exactly the
  order in which p stores them, so no unpack pass is needed.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib as L


def split_ranges(rowptr, nranks: int, balance: str = "edges") -> np.ndarray:
    """Boundaries b[0..nranks] of contiguous node ranges, balanced by edges+nodes."""
    rowptr = np.asarray(rowptr, dtype=np.int64)
    n = len(rowptr) - 1
    if balance == "nodes":
        return np.array([(n * p) // nranks for p in range(nranks + 1)], dtype=np.int64)
    work = rowptr + np.arange(n + 1, dtype=np.int64)  # edges + nodes prefix
    targets = [(work[-1] * p) // nranks for p in range(nranks + 1)]
    b = np.searchsorted(work, targets, side="left").astype(np.int64)
    b[0], b[-1] = 0, n
    return np.maximum.accumulate(b)


@dataclass
class Plan:
    rank: int
    nranks: int
    lo: int
    hi: int
    rowptr: np.ndarray       # int64 [n_local+1]
    col: np.ndarray          # int32 [e_local], ghost-extended numbering
    rev: np.ndarray          # int32 [e_local], ghost-extended numbering
    n_ghost_a: int
    n_ghost_f: int
    ghost_a_gid: np.ndarray  # global node id of each ghost estimate slot
    ghost_f_gidx: np.ndarray  # global edge index of each ghost flow slot
    send_f_off: np.ndarray
    send_f_idx: np.ndarray
    recv_f_off: np.ndarray
    send_a_off: np.ndarray
    send_a_idx: np.ndarray
    recv_a_off: np.ndarray

    @property
    def n_local(self):
        return self.hi - self.lo

    @property
    def e_local(self):
        return int(self.rowptr[-1])


def partition(rowptr, col, rev, nranks: int, rank: int, bounds=None) -> Plan:
    rowptr = np.asarray(rowptr, dtype=np.int64)
    col = np.asarray(col, dtype=np.int64)
    rev = np.asarray(rev, dtype=np.int64)
    b = split_ranges(rowptr, nranks) if bounds is None else np.asarray(bounds, dtype=np.int64)
    lo, hi = int(b[rank]), int(b[rank + 1])
    e0, e1 = int(rowptr[lo]), int(rowptr[hi])
    n_local, e_local = hi - lo, e1 - e0
    lcol = col[e0:e1]
    lrev = rev[e0:e1]
    owner_of_col = np.searchsorted(b, lcol, side="right") - 1
    remote = (lcol < lo) | (lcol >= hi)

    # ghost estimates: remote neighbours, grouped by owner (ascending id == grouped by owner,
    # since ranges are contiguous and ordered)
    ghost_a_gid = np.unique(lcol[remote])
    owner_a = np.searchsorted(b, ghost_a_gid, side="right") - 1
    recv_a_off = np.zeros(nranks + 1, dtype=np.int64)
    np.add.at(recv_a_off, owner_a + 1, 1)
    recv_a_off = np.cumsum(recv_a_off)
    new_col = np.where(remote, 0, lcol - lo)
    new_col[remote] = n_local + np.searchsorted(ghost_a_gid, lcol[remote])

    # ghost flows: the reverse edges of cut edges, sorted by their global index (owner order
    # follows, because edge ranges are contiguous per rank)
    ghost_f_gidx = np.sort(lrev[remote])
    recv_f_off = np.zeros(nranks + 1, dtype=np.int64)
    np.add.at(recv_f_off, (np.searchsorted(b, ghost_f_gidx_owner_nodes(rowptr, ghost_f_gidx),
                                           side="right") - 1) + 1, 1)
    recv_f_off = np.cumsum(recv_f_off)
    new_rev = np.where(remote, 0, lrev - e0)
    new_rev[remote] = e_local + np.searchsorted(ghost_f_gidx, lrev[remote])

    # send lists: my edges into p's range, ascending (== local index order)
    send_f_idx = []
    send_a_idx = []
    send_f_off = [0]
    send_a_off = [0]
    src_local = np.repeat(np.arange(n_local, dtype=np.int64), np.diff(rowptr[lo:hi + 1]))
    for p in range(nranks):
        if p == rank:
            send_f_off.append(send_f_off[-1])
            send_a_off.append(send_a_off[-1])
            continue
        m = owner_of_col == p
        ef = np.nonzero(m)[0]
        na = np.unique(src_local[m])
        send_f_idx.append(ef)
        send_a_idx.append(na)
        send_f_off.append(send_f_off[-1] + len(ef))
        send_a_off.append(send_a_off[-1] + len(na))
    cat = lambda xs: (np.concatenate(xs) if xs else np.zeros(0, dtype=np.int64))  # noqa: E731
    return Plan(rank, nranks, lo, hi, rowptr[lo:hi + 1] - e0, new_col.astype(np.int32),
                new_rev.astype(np.int32), len(ghost_a_gid), len(ghost_f_gidx), ghost_a_gid,
                ghost_f_gidx, np.array(send_f_off, dtype=np.int64),
                cat(send_f_idx).astype(np.int32), recv_f_off,
                np.array(send_a_off, dtype=np.int64), cat(send_a_idx).astype(np.int32),
                recv_a_off)


def ghost_f_gidx_owner_nodes(rowptr, gidx):
    """Source node of each global edge index."""
    return np.searchsorted(rowptr, gidx, side="right") - 1


class RggPart:
    """One rank's slab of the random geometric graph fu_graph_gen_rgg(n_total, radius, seed),
    generated natively without the global graph (fu_part_gen_rgg), with the estimates-only
    halo plan (kernel 4)."""

    def __init__(self, n_total: int, radius: float | None = None, avg_deg: float = 8.0,
                 seed: int = 1, nparts: int = 1, part: int = 0):
        if radius is None:
            radius = float(np.sqrt(avg_deg / (np.pi * n_total)))
        out = L.vp()
        L.call("fu_part_gen_rgg", int(n_total), float(radius), int(seed), int(nparts), int(part),
               ctypes.byref(out))
        self._h = out
        info = np.zeros(8, dtype=np.int64)
        L.call("fu_part_info", self._h, L.ptr(info))
        (self.n_local, self.e_local, self.lo, self.hi, self.n_ghost_a, _, self.max_deg,
         self.n_total) = (int(x) for x in info)
        self.nparts, self.part, self.radius = nparts, part, radius
        self.rowptr = np.empty(self.n_local + 1, dtype=np.int64)
        self.col = np.empty(max(self.e_local, 1), dtype=np.int32)
        self.ghost_gid = np.empty(max(self.n_ghost_a, 1), dtype=np.int64)
        self.send_a_off = np.empty(nparts + 1, dtype=np.int64)
        self.send_a_idx = np.empty(max(int(info[5]), 1), dtype=np.int32)
        self.recv_a_off = np.empty(nparts + 1, dtype=np.int64)
        L.call("fu_part_export", self._h, L.ptr(self.rowptr), L.ptr(self.col), L.ptr(self.ghost_gid),
               L.ptr(self.send_a_off), L.ptr(self.send_a_idx), L.ptr(self.recv_a_off))
        self.col = self.col[:self.e_local]
        self.ghost_gid = self.ghost_gid[:self.n_ghost_a]
        self.send_a_idx = self.send_a_idx[:int(info[5])]
        L.lib.fu_part_free(self._h)
        self._h = None

    def global_col(self):
        """Neighbour ids in global numbering (for checks)."""
        c = self.col.astype(np.int64)
        ghost = c >= self.n_local
        out = c + self.lo
        out[ghost] = self.ghost_gid[c[ghost] - self.n_local]
        return out

    def values(self, seed: int = 0, lo: float = 0.0, hi: float = 100.0):
        out = np.empty(self.n_local)
        L.call("fu_values_uniform_range", self.lo, self.n_local, int(seed), float(lo), float(hi),
               L.ptr(out))
        return out

    def to_plan(self) -> Plan:
        z = np.zeros(self.nparts + 1, dtype=np.int64)
        return Plan(self.part, self.nparts, self.lo, self.hi, self.rowptr, self.col, None,
                    self.n_ghost_a, 0, self.ghost_gid, np.zeros(0, dtype=np.int64), z,
                    np.zeros(0, dtype=np.int32), z.copy(), self.send_a_off, self.send_a_idx,
                    self.recv_a_off)


def _exact_expansion(vals) -> list:
    """Non-overlapping doubles whose exact sum is the exact sum of `vals`: math.fsum's
    correctly rounded sum, then the correctly rounded residual of the rest, until nothing is
    left (each step takes 53 more bits; 3-4 steps for millions of values)."""
    import math

    vals = list(vals)
    out = []
    while True:
        s = math.fsum(vals + [-x for x in out])
        if s == 0.0 or len(out) > 40:
            return out
        out.append(s)


def component_means_dist(n_local, rowptr, col, send_a_off, send_a_idx, recv_a_off, values,
                         rank, nranks, dist=None):
    """fu.component_means for a partitioned graph, without any rank holding the global graph:
    the per-node exact mean of its connected component (math.fsum over the component, divided
    by its size; the convergence target of SURVEY.md §8(d)). Bitwise equal to
    fu.component_means on the global graph.

    Every rank labels the components of its own rows (edges to ghost slots left out) and
    the exact sum of each as a double expansion; rank 0 joins the labels across the cut edges
    (a ghost slot of this rank from peer p is p's node send_a_idx[send_a_off[me] + k], the
    slot order of the halo plan) with a union-find and fsums the expansions of each global
    component; the means go back to the ranks. `dist` is torch.distributed (any backend
    with object collectives) or None at one rank."""
    import math

    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import connected_components

    rowptr = np.asarray(rowptr, dtype=np.int64)
    col = np.asarray(col, dtype=np.int64)
    values = np.asarray(values, dtype=np.float64)
    send_a_off = np.asarray(send_a_off, dtype=np.int64)
    recv_a_off = np.asarray(recv_a_off, dtype=np.int64)
    src = np.repeat(np.arange(n_local, dtype=np.int64), np.diff(rowptr))
    own = col < n_local
    m = csr_matrix((np.ones(int(own.sum()), dtype=np.int8), (src[own], col[own])), shape=(n_local, n_local))
    nc, lab = connected_components(m, directed=False)
    # exact sums per local component (sizes 1 and 2 without a Python loop, as fu.component_means)
    order = np.argsort(lab, kind="stable")
    bounds = np.searchsorted(lab[order], np.arange(nc + 1))
    vs = values[order]
    size = np.diff(bounds)
    exp = [None] * nc
    for k in np.nonzero(size == 1)[0]:
        exp[k] = [float(vs[bounds[k]])]
    for k in np.nonzero(size >= 2)[0]:
        exp[k] = _exact_expansion(vs[bounds[k]:bounds[k + 1]].tolist())
    # cut edges: (my label, peer, index into the peer's send list)
    ghost = ~own
    slot = col[ghost] - n_local
    peer = np.searchsorted(recv_a_off, slot, side="right") - 1
    cut = np.unique(np.stack([lab[src[ghost]], peer, slot - recv_a_off[peer]]), axis=1) \
        if ghost.any() else np.zeros((3, 0), dtype=np.int64)
    send_lab = lab[np.asarray(send_a_idx, dtype=np.int64)] if len(send_a_idx) else np.zeros(0, dtype=np.int64)
    mine = {"nc": nc, "size": size, "exp": exp, "cut": cut, "send_lab": send_lab, "send_a_off": send_a_off}
    if dist is not None and nranks > 1:
        allr = [None] * nranks if rank == 0 else None
        dist.gather_object(mine, allr, dst=0)
    else:
        allr = [mine]
    result = [None]
    if rank == 0:
        base = np.cumsum([0] + [r["nc"] for r in allr])
        parent = np.arange(base[-1])

        def find(x):
            while parent[x] != x:
                parent[x] = parent[parent[x]]
                x = parent[x]
            return x

        for q, r in enumerate(allr):
            for mylab, p, k in r["cut"].T:
                pr = allr[int(p)]
                other = base[int(p)] + pr["send_lab"][pr["send_a_off"][q] + int(k)]
                x, y = find(base[q] + int(mylab)), find(int(other))
                if x != y:
                    parent[max(x, y)] = min(x, y)
        roots = np.array([find(x) for x in range(base[-1])], dtype=np.int64)
        sizes = np.concatenate([r["size"] for r in allr]).astype(np.int64)
        exps = [e for r in allr for e in r["exp"]]
        groups = {}
        for x, rt in enumerate(roots):
            groups.setdefault(int(rt), []).append(x)
        mean = np.empty(base[-1])
        for rt, members in groups.items():
            tot = int(sizes[members].sum())
            if len(members) == 1 and len(exps[members[0]]) == 1:
                mean[members] = exps[members[0]][0] / tot if tot > 1 else exps[members[0]][0]
            else:
                mean[members] = math.fsum([x for mbr in members for x in exps[mbr]]) / tot
        ncomp = len(groups)
        result = [[(mean[base[q]:base[q + 1]], ncomp) for q in range(len(allr))]]
    if dist is not None and nranks > 1:
        dist.broadcast_object_list(result, src=0)
    lmean, ncomp = result[0][rank]
    return lmean[lab], ncomp


def unique_id() -> bytes:
    buf = (ctypes.c_uint8 * 128)()
    L.call("fu_dist_unique_id", buf)
    return bytes(buf)


class DistCollectAll:
    """One rank of a partitioned collect-all run (RCCL halo exchange every round)."""

    def __init__(self, plan: Plan, values_local, uid: bytes | None, device: int = 0,
                 kernel: str = "auto"):
        """uid = the RCCL unique id shared by all ranks; None = the local test transport
        (all ranks in this process; rounds driven by run_local)."""
        from .engine import KERNELS

        self.plan = plan
        self.values = np.ascontiguousarray(values_local, dtype=np.float64)
        if len(self.values) != plan.n_local:
            raise ValueError("values_local must have n_local entries")
        # estimates-only halo: the round kernels rebuild the neighbours' flows, so the plan's
        # ghost-flow part (rev, send_f_*, recv_f_off) is not sent to the device
        zf = np.zeros(plan.nranks + 1, dtype=np.int64)
        keep = [plan.rowptr, plan.col, zf, plan.send_a_off, plan.send_a_idx, plan.recv_a_off]
        self._keep = [np.ascontiguousarray(x) for x in keep]
        (rp, c, zf, sao, sai, rao) = self._keep
        out = L.vp()
        if uid is None:  # local test transport (exchange_local), no communicator
            L.call("fu_dist_create_local", plan.n_local, plan.e_local, L.ptr(rp), L.ptr(c),
                   L.ptr(self.values), plan.n_ghost_a, plan.nranks, plan.rank, L.ptr(sao),
                   L.ptr(sai) if len(sai) else None, L.ptr(rao), int(device), ctypes.byref(out))
        else:
            idbuf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
            L.call("fu_dist_create", plan.n_local, plan.e_local, L.ptr(rp), L.ptr(c), None,
                   L.ptr(self.values), plan.n_ghost_a, 0, plan.nranks, plan.rank,
                   L.ptr(zf), None, L.ptr(zf), L.ptr(sao),
                   L.ptr(sai) if len(sai) else None, L.ptr(rao), idbuf, int(device),
                   ctypes.byref(out))
        self._h = out
        self.n = plan.n_local
        self.E = plan.e_local
        k = KERNELS[kernel]
        if k:
            L.call("fu_set_option", self._h, b"kernel", k)

    def run(self, rounds: int, err_every: int = 0):
        if err_every > 0:
            trace = np.empty(max(rounds // err_every, 1))
            L.call("fu_run_collectall", self._h, int(rounds), int(err_every), L.ptr(trace))
            return trace[:rounds // err_every]
        L.call("fu_run_collectall", self._h, int(rounds), 0, None)
        return None

    def run_timed(self, rounds: int) -> float:
        ms = L.f32()
        L.call("fu_run_collectall_timed", self._h, int(rounds), ctypes.byref(ms))
        return float(ms.value)

    def tune(self):
        """One autotune pass (collective: every rank calls it; same rounds on each)."""
        L.call("fu_tune", self._h)

    def reset(self):
        L.call("fu_reset", self._h)

    def run_marked(self, rounds_at):
        ra = np.ascontiguousarray(rounds_at, dtype=np.int32)
        L.call("fu_run_collectall_marked", self._h, len(ra), L.ptr(ra))

    def mark(self, slot: int):
        L.call("fu_mark", self._h, int(slot))

    def elapsed(self, a: int, b: int) -> float:
        ms = L.f32()
        L.call("fu_mark_elapsed", self._h, int(a), int(b), ctypes.byref(ms))
        return float(ms.value)

    def set_targets(self, target_local):
        self._target = np.ascontiguousarray(target_local, dtype=np.float64)
        L.call("fu_set_targets", self._h, L.ptr(self._target))

    def estimates(self):
        a = np.empty(self.n)
        L.call("fu_get_estimates", self._h, L.ptr(a))
        return a

    def flows(self):
        f = np.empty(max(self.E, 1))
        L.call("fu_get_flows", self._h, L.ptr(f))
        return f[:self.E]

    def synchronize(self):
        L.call("fu_synchronize", self._h)

    def halo_ms(self) -> float:
        """Device time of the last round's halo on the comm stream (pack start to ghost
        slots written; it overlaps the interior tiles). Waits for that halo."""
        ms = L.f32()
        L.call("fu_dist_halo_time", self._h, ctypes.byref(ms))
        return float(ms.value)

    def info(self) -> dict:
        from .engine import handle_info

        return handle_info(self._h)

    def close(self):
        if getattr(self, "_h", None):
            L.lib.fu_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


def run_local(engines, rounds: int):
    """In-process transport: `rounds` rounds of every rank (DistCollectAll(..., uid=None)),
    each followed by its halo exchange (fu_dist_run_local). Everything is queued
    asynchronously on the ranks' main and comm streams, as with RCCL: the copies into the
    ghost slots run beside each round's interior tiles, and no host sync happens between
    rounds."""
    arr = (ctypes.c_void_p * len(engines))(*[e._h.value for e in engines])
    L.call("fu_dist_run_local", arr, len(engines), int(rounds))

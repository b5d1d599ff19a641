"""Host graphs: CSR + reverse-edge index, built natively in libfu (fu_graph_*).

The reference builds its topology from the deployment file: each Peer splits its neighbour
string into an insertion-ordered dict (flowupdating-collectall.py:29-31, CA:38-40). That
order is the summation order of avg_and_send (CA:106, CA:110). `Graph.from_csr` keeps row
order as given. Generators return rows sorted by neighbour id.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L


class Graph:
    """Owns a native fu_graph*. Arrays are exported lazily (`rowptr`, `col`, `rev`)."""

    def __init__(self, handle):
        self._h = handle
        n = L.i32()
        e = L.i64()
        md = L.i32()
        sym = L.i32()
        L.call("fu_graph_info", self._h, ctypes.byref(n), ctypes.byref(e), ctypes.byref(md),
               ctypes.byref(sym))
        self.n = int(n.value)
        self.E = int(e.value)
        self.max_deg = int(md.value)
        self.symmetric = bool(sym.value)
        self._arrays = None

    # ---------------- constructors ----------------
    @staticmethod
    def _make(fn, *args) -> "Graph":
        out = L.vp()
        L.call(fn, *args, ctypes.byref(out))
        return Graph(out)

    @classmethod
    def from_edges(cls, n: int, src, dst) -> "Graph":
        """Undirected edge list -> symmetric CSR (self-loops dropped, deduplicated)."""
        s = np.ascontiguousarray(src, dtype=np.int32)
        d = np.ascontiguousarray(dst, dtype=np.int32)
        if s.shape != d.shape:
            raise ValueError("src and dst must have the same length")
        return cls._make("fu_graph_from_edges", int(n), len(s), L.ptr(s), L.ptr(d))

    @classmethod
    def from_csr(cls, rowptr, col, require_symmetric: bool = True) -> "Graph":
        rp = np.ascontiguousarray(rowptr, dtype=np.int64)
        c = np.ascontiguousarray(col, dtype=np.int32)
        return cls._make("fu_graph_from_csr", len(rp) - 1, L.ptr(rp), L.ptr(c),
                         1 if require_symmetric else 0)

    @classmethod
    def erdos_renyi(cls, n: int, m: int, seed: int = 1) -> "Graph":
        return cls._make("fu_graph_gen_er", int(n), int(m), int(seed))

    @classmethod
    def random_regular(cls, n: int, d: int, seed: int = 1) -> "Graph":
        return cls._make("fu_graph_gen_rr", int(n), int(d), int(seed))

    @classmethod
    def rmat(cls, scale: int, edge_factor: int = 16, a=0.57, b=0.19, c=0.19,
             seed: int = 1) -> "Graph":
        return cls._make("fu_graph_gen_rmat", int(scale), int(edge_factor), float(a), float(b),
                         float(c), int(seed))

    @classmethod
    def random_geometric(cls, n: int, radius: float | None = None, avg_deg: float = 8.0,
                         seed: int = 1) -> "Graph":
        if radius is None:
            radius = float(np.sqrt(avg_deg / (np.pi * n)))
        return cls._make("fu_graph_gen_rgg", int(n), float(radius), int(seed))

    @classmethod
    def from_spec(cls, spec: str, seed: int = 1) -> "Graph":
        """'er:n=1000000,m=4000000' | 'rr:n=65536,d=8' | 'rmat:scale=24,ef=16' |
        'rgg:n=67108864,deg=8'"""
        kind, _, rest = spec.partition(":")
        kv = {}
        for part in filter(None, rest.split(",")):
            k, _, v = part.partition("=")
            kv[k.strip()] = v.strip()
        if kind == "er":
            return cls.erdos_renyi(int(float(kv["n"])), int(float(kv["m"])), seed)
        if kind == "rr":
            return cls.random_regular(int(float(kv["n"])), int(kv["d"]), seed)
        if kind == "rmat":
            return cls.rmat(int(kv["scale"]), int(kv.get("ef", 16)), float(kv.get("a", 0.57)),
                            float(kv.get("b", 0.19)), float(kv.get("c", 0.19)), seed)
        if kind == "rgg":
            return cls.random_geometric(int(float(kv["n"])), avg_deg=float(kv.get("deg", 8)),
                                        seed=seed)
        raise ValueError(f"unknown graph spec {spec!r}")

    def relabel(self, order="degree", new_of_old=None):
        """(relabelled Graph, new_of_old): node i becomes new_of_old[i]; rows keep their
        neighbour order (fu_graph_relabel). order "degree" (descending, ties by id) or
        "given" with new_of_old a permutation."""
        if order == "degree":
            perm, mode = np.empty(self.n, dtype=np.int32), 1
        elif order == "given":
            perm, mode = np.ascontiguousarray(new_of_old, dtype=np.int32).copy(), 0
            if perm.shape != (self.n,):
                raise ValueError("new_of_old must have n entries")
        else:
            raise ValueError(f"unknown order {order!r}")
        out = L.vp()
        L.call("fu_graph_relabel", self._h, mode, L.ptr(perm), ctypes.byref(out))
        return Graph(out), perm

    # ---------------- arrays ----------------
    def arrays(self):
        if self._arrays is None:
            rp = np.empty(self.n + 1, dtype=np.int64)
            col = np.empty(max(self.E, 1), dtype=np.int32)
            rev = np.empty(max(self.E, 1), dtype=np.int32) if self.symmetric else None
            L.call("fu_graph_export", self._h, L.ptr(rp), L.ptr(col), L.ptr(rev))
            self._arrays = (rp, col[:self.E], None if rev is None else rev[:self.E])
        return self._arrays

    @property
    def rowptr(self):
        return self.arrays()[0]

    @property
    def col(self):
        return self.arrays()[1]

    @property
    def rev(self):
        return self.arrays()[2]

    @property
    def degrees(self):
        return np.diff(self.rowptr)

    def free(self):
        if getattr(self, "_h", None):
            L.lib.fu_graph_free(self._h)
            self._h = None

    def __del__(self):
        self.free()


def uniform_values(n: int, seed: int = 0, lo: float = 0.0, hi: float = 100.0) -> np.ndarray:
    """value[i] = lo + (hi - lo) * U_i, SplitMix64 counter stream (include/fu.h)."""
    out = np.empty(n, dtype=np.float64)
    L.call("fu_values_uniform", int(n), int(seed), float(lo), float(hi), L.ptr(out))
    return out


def component_means(rowptr, col, values):
    """(per-node exact mean of its connected component, component id per node).

    The convergence target of max |e_i - mean|. Uses scipy's connected
    components and exact summation (math.fsum) per component."""
    import math

    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import connected_components

    n = len(rowptr) - 1
    m = csr_matrix((np.ones(len(col), dtype=np.int8), np.asarray(col), np.asarray(rowptr)),
                   shape=(n, n))
    nc, comp = connected_components(m, directed=False)
    order = np.argsort(comp, kind="stable")
    bounds = np.searchsorted(comp[order], np.arange(nc + 1))
    vals = np.asarray(values, dtype=np.float64)[order]
    size = np.diff(bounds)
    means = np.empty(nc)
    # components of one or two nodes (isolated nodes, pairs: millions on R-MAT-24) without a
    # Python loop: fsum of one value is the value, fsum of two is their correctly rounded sum
    one = size == 1
    means[one] = vals[bounds[:-1][one]]
    two = size == 2
    means[two] = (vals[bounds[:-1][two]] + vals[bounds[:-1][two] + 1]) / 2
    for k in np.nonzero(size > 2)[0]:
        seg = vals[bounds[k]:bounds[k + 1]]
        means[k] = math.fsum(seg.tolist()) / len(seg)
    return means[comp], comp

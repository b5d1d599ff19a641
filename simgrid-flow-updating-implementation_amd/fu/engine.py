"""Device engines behind the C ABI.

* `CollectAll`: generation-synchronous collect-all rounds on one GPU (fu_create /
  fu_run_collectall). One round = Peer.on_receive for every directed edge + Peer.avg_and_send
  for every node (flowupdating-collectall.py:93-128), as one data-parallel kernel.
* `Trace` + `Replay`: the tick-level schedule of the reference run (Peer.loop, CA:70-85 /
  PW:69-84, and the SimGrid mailboxes), built natively on the host and replayed on the
  GPU one tick per batch. Used by the pairwise mode and by faithful small-platform runs.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L
from .graph import Graph

KERNELS = {"auto": 0, "recon": 4, "stage": 8, "pregather": 9}
LAYOUTS = {"given": 0, "degree": 1}
MODE = {"collectall": 0, "ca": 0, "pairwise": 1, "pw": 1}


def handle_info(h) -> dict:
    """Kernel in use (after autotuning), autotune state, rounds done."""
    a = np.zeros(32, dtype=np.int64)
    L.call("fu_get_info", h, L.ptr(a))
    names = {4: "recon", 8: "stage", 9: "pregather"}
    return {"kernel": names.get(int(a[0]), int(a[0])),
            "autotune": ["off", "pending", "done"][int(a[2])], "rounds": int(a[3]),
            "tile": (int(a[4]), int(a[5])), "tune_passes": int(a[6]),
            "tuned_pack_width": int(a[7]), "mega_hubs": int(a[20]),
            "stage_slices": [int(x) for x in a[27:31]],
            "tune_winner_by_width": {w: _cand_name(int(a[23 + k])) for k, w in
                                     enumerate((0, 8, 16, 32)) if a[23 + k] >= 0},
            "tune_us_per_round": {k: a[8 + i] / 1e3 for i, k in
                                  enumerate(TUNE_CANDIDATES)}}


# fu_engine.hip kCands order
TUNE_CANDIDATES = ("recon", "recon_512", "stage", "recon_1024", "pregather")


def _cand_name(code: int) -> str:
    kernel, geo = divmod(code, 10)
    if kernel == 8:
        return "stage"
    if kernel == 9:
        return "pregather"
    return "recon" + {3: "_512", 1: "_1024", 2: "_1024x256"}.get(geo, "")


class CollectAll:
    """Synchronous collect-all engine on one GPU.

    >>> g = Graph.erdos_renyi(1_000_000, 4_000_000, seed=1)
    >>> eng = CollectAll(g, uniform_values(g.n, seed=0))
    >>> eng.run(1000); est = eng.estimates()
    """

    def __init__(self, graph: Graph | None = None, values=None, *, rowptr=None, col=None,
                 rev=None, device: int = 0, kernel: str | int = "auto",
                 hub_threshold: int | None = None, layout: str = "given"):
        """layout "degree" relabels the device graph by degree (fu_create_from_graph_ex):
        the most-gathered estimates share cache lines; inputs and outputs keep the caller's
        numbering, bits per node unchanged."""
        self.values = np.ascontiguousarray(values, dtype=np.float64)
        out = L.vp()
        if graph is not None:
            if len(self.values) != graph.n:
                raise ValueError("len(values) != graph.n")
            L.call("fu_create_from_graph_ex", graph._h, L.ptr(self.values), int(device),
                   LAYOUTS[layout], ctypes.byref(out))
            self.n, self.E = graph.n, graph.E
        else:
            if layout != "given":
                raise ValueError("layout needs a Graph")
            rp = np.ascontiguousarray(rowptr, dtype=np.int64)
            c = np.ascontiguousarray(col, dtype=np.int32)
            r = None if rev is None else np.ascontiguousarray(rev, dtype=np.int32)
            n = len(rp) - 1
            if len(self.values) != n:
                raise ValueError("len(values) != n")
            L.call("fu_create", n, int(rp[-1]), L.ptr(rp), L.ptr(c), L.ptr(r),
                   L.ptr(self.values), int(device), ctypes.byref(out))
            self.n, self.E = n, int(rp[-1])
        self._h = out
        if hub_threshold is not None:
            self.set_option("hub_threshold", hub_threshold)
        k = KERNELS[kernel] if isinstance(kernel, str) else int(kernel)
        if k:
            self.set_option("kernel", k)

    def set_option(self, key: str, value: int):
        L.call("fu_set_option", self._h, key.encode(), int(value))

    def reset(self):
        L.call("fu_reset", self._h)

    def set_targets(self, target):
        self._target = np.ascontiguousarray(target, dtype=np.float64)
        L.call("fu_set_targets", self._h, L.ptr(self._target))

    def run(self, rounds: int, err_every: int = 0):
        """Run `rounds` rounds; with err_every > 0 returns the max-error trace."""
        if err_every > 0:
            trace = np.empty(max(rounds // err_every, 1))
            L.call("fu_run_collectall", self._h, int(rounds), int(err_every), L.ptr(trace))
            return trace[:rounds // err_every]
        L.call("fu_run_collectall", self._h, int(rounds), 0, None)
        return None

    def run_timed(self, rounds: int) -> float:
        """Device milliseconds for `rounds` rounds (HIP events on the handle's stream)."""
        ms = L.f32()
        L.call("fu_run_collectall_timed", self._h, int(rounds), ctypes.byref(ms))
        return float(ms.value)

    def tune(self):
        """One autotune pass now (kernel "auto"), outside any timed region: ~55 real rounds
        at the current packing width; the state advances, so reset() before a timed run."""
        L.call("fu_tune", self._h)

    def run_marked(self, rounds_at):
        """Run rounds_at[-1] rounds in one call, recording mark k once rounds_at[k] of them
        are queued (rounds_at[0] = 0: the start). Asynchronous; see elapsed()."""
        ra = rounds_at if isinstance(rounds_at, np.ndarray) and rounds_at.dtype == np.int32 \
            and rounds_at.flags["C_CONTIGUOUS"] else np.ascontiguousarray(rounds_at, dtype=np.int32)
        L.call("fu_run_collectall_marked", self._h, len(ra), ra.ctypes.data)

    def mark(self, slot: int):
        """Record HIP event `slot` (0..63) on the engine's stream (asynchronous)."""
        L.call("fu_mark", self._h, int(slot))

    def elapsed(self, a: int, b: int) -> float:
        """Device milliseconds between marks a and b (waits for b)."""
        ms = L.f32()
        L.call("fu_mark_elapsed", self._h, int(a), int(b), ctypes.byref(ms))
        return float(ms.value)

    def max_err(self) -> float:
        out = L.f64()
        L.call("fu_max_err", self._h, ctypes.byref(out))
        return float(out.value)

    def estimates(self) -> np.ndarray:
        a = np.empty(self.n)
        L.call("fu_get_estimates", self._h, L.ptr(a))
        return a

    def flows(self) -> np.ndarray:
        f = np.empty(max(self.E, 1))
        L.call("fu_get_flows", self._h, L.ptr(f))
        return f[:self.E]

    def info(self) -> dict:
        """Kernel in use (after autotuning), autotune state, rounds done."""
        return handle_info(self._h)

    def pack_widths(self) -> tuple:
        """Packed estimate table widths (0 = doubles): the last even / odd round's code
        table and the current encoding plan."""
        w = np.zeros(3, dtype=np.int32)
        L.call("fu_get_pack", self._h, L.ptr(w))
        return tuple(int(x) for x in w)

    @property
    def rounds_done(self) -> int:
        r = L.i64()
        L.call("fu_get_round", self._h, ctypes.byref(r))
        return int(r.value)

    def synchronize(self):
        L.call("fu_synchronize", self._h)

    def close(self):
        if getattr(self, "_h", None):
            L.lib.fu_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class Trace:
    """Tick-level schedule of the reference run (fu_trace_build), value-independent.

    decl_rowptr/decl_col: declared neighbour lists (actors.xml, ACT:4-27) in deployment
    order. mode: 'collectall' | 'pairwise'. order: 'fwd' | 'rev' | 'rand:<seed>'.
    """

    def __init__(self, decl_rowptr, decl_col, mode: str, ticks: int, order: str = "fwd",
                 faults: str | None = None, route_s=None, net=None):
        """route_s: optional n x n transfer times in seconds (sender row); a message matched at
        tick t is consumed from tick t + floor(T) + 1 (fu_trace_build_routes).
        net: optional link model (fu.platform.Platform.link_net): transfers share the
        links' bandwidth (max-min fair, weighted by LV08's sharing penalty when net holds
        weight_S > 0, capped by the TCP window with tcp_gamma > 0, each transfer loading its
        reverse route with crosstraffic > 0: fu_trace_build_links_cross); exclusive with
        route_s."""
        rp = np.ascontiguousarray(decl_rowptr, dtype=np.int64)
        c = np.ascontiguousarray(decl_col, dtype=np.int32)
        self.n = len(rp) - 1
        self.decl_deg = np.diff(rp)
        self.mode = mode
        self.ticks = int(ticks)
        self.order = order
        out = L.vp()
        self._route = None
        if route_s is not None:
            self._route = np.ascontiguousarray(route_s, dtype=np.float64)
            if self._route.shape != (self.n, self.n):
                raise ValueError("route_s must be n x n")
        if net is not None:
            if route_s is not None:
                raise ValueError("route_s and net are exclusive")
            self._net = {k: np.ascontiguousarray(net[k], dtype=dt) for k, dt in (
                ("bw", np.float64), ("lat", np.float64), ("shared", np.int32),
                ("route_off", np.int64), ("route_links", np.int32))}
            if len(self._net["route_off"]) != self.n * self.n + 1:
                raise ValueError("net['route_off'] must have n * n + 1 entries")
            nl = len(self._net["bw"])
            z = lambda a: L.ptr(a) if len(a) else None  # noqa: E731
            L.call("fu_trace_build_links_cross", self.n, L.ptr(rp), L.ptr(c) if len(c) else None, MODE[mode],
                   self.ticks, order.encode(), faults.encode() if faults else None, nl, z(self._net["bw"]),
                   z(self._net["lat"]), z(self._net["shared"]), L.ptr(self._net["route_off"]),
                   z(self._net["route_links"]), float(net.get("bytes", 154.0)),
                   float(net.get("lat_factor", 13.01)), float(net.get("bw_factor", 0.97)),
                   float(net.get("weight_S", 0.0)), float(net.get("tcp_gamma", 0.0)),
                   float(net.get("crosstraffic", 0.0)), ctypes.byref(out))
        else:
            L.call("fu_trace_build_routes", self.n, L.ptr(rp), L.ptr(c) if len(c) else None, MODE[mode],
                   self.ticks, order.encode(), faults.encode() if faults else None,
                   None if self._route is None else L.ptr(self._route), ctypes.byref(out))
        self._h = out
        self.faults = faults
        dr, dl = L.i64(), L.i64()
        L.call("fu_trace_fault_stats", self._h, ctypes.byref(dr), ctypes.byref(dl))
        self.dropped, self.delayed = int(dr.value), int(dl.value)
        info = np.zeros(8, dtype=np.int64)
        L.call("fu_trace_info", self._h, L.ptr(info))
        (self.n_union_edges, self.n_tasks, self.n_events, self.n_out_ids, self.n_msgs,
         _, self.dynamic_additions, self.messages_sent) = (int(x) for x in info)
        self._arrays = None

    def arrays(self) -> dict:
        if self._arrays is None:
            a = {
                "rowptr": np.empty(self.n + 1, dtype=np.int64),
                "col": np.empty(max(self.n_union_edges, 1), dtype=np.int32),
                "tick_task_off": np.empty(self.ticks + 1, dtype=np.int64),
                "tasks": np.empty((max(self.n_tasks, 1), 3), dtype=np.int32),
                "events": np.empty((max(self.n_events, 1), 4), dtype=np.int32),
                "out_ids": np.empty(max(self.n_out_ids, 1), dtype=np.int32),
                "first_avg_seq": np.empty(self.n, dtype=np.int64),
                "fires": np.empty(self.n, dtype=np.int32),
            }
            L.call("fu_trace_export", self._h, *(L.ptr(a[k]) for k in (
                "rowptr", "col", "tick_task_off", "tasks", "events", "out_ids",
                "first_avg_seq", "fires")))
            a["col"] = a["col"][:self.n_union_edges]
            a["tasks"] = a["tasks"][:self.n_tasks]
            a["events"] = a["events"][:self.n_events]
            a["out_ids"] = a["out_ids"][:self.n_out_ids]
            self._arrays = a
        return self._arrays

    def last_avg_order(self) -> list[int]:
        """Nodes in the key order of global_values['last_avg'] (order of first average)."""
        seq = self.arrays()["first_avg_seq"]
        nodes = [i for i in range(self.n) if seq[i] >= 0]
        return sorted(nodes, key=lambda i: seq[i])

    def free(self):
        if getattr(self, "_h", None):
            L.lib.fu_trace_free(self._h)
            self._h = None

    def __del__(self):
        self.free()


class Replay:
    """GPU replay of a Trace with node values."""

    def __init__(self, trace: Trace, values, device: int = 0, persistent: bool = False,
                 registers: bool = True):
        self.trace = trace
        self.values = np.ascontiguousarray(values, dtype=np.float64)
        if len(self.values) != trace.n:
            raise ValueError("len(values) != trace.n")
        out = L.vp()
        L.call("fu_replay_create_from_trace", trace._h, L.ptr(self.values), int(device),
               ctypes.byref(out))
        self._h = out
        self.n = trace.n
        self.E = trace.n_union_edges
        if persistent:
            L.call("fu_replay_set_option", self._h, b"persistent", 1)
            L.call("fu_replay_set_option", self._h, b"persistent_reg", int(registers))
        self.tick = 0

    def run(self, tick_end: int, snapshot_ticks=()):
        """Run ticks [current, tick_end); returns {tick: last_avg copy} for snapshot_ticks."""
        st = np.ascontiguousarray(sorted(snapshot_ticks), dtype=np.int32)
        snaps = np.empty((max(len(st), 1), self.n))
        L.call("fu_replay_run", self._h, int(tick_end), len(st),
               L.ptr(st) if len(st) else None, L.ptr(snaps) if len(st) else None)
        self.tick = int(tick_end)
        return {int(t): snaps[k].copy() for k, t in enumerate(st)}

    def run_timed(self, tick_end: int) -> float:
        ms = L.f32()
        L.call("fu_replay_run_timed", self._h, int(tick_end), ctypes.byref(ms))
        self.tick = int(tick_end)
        return float(ms.value)

    def state(self):
        last = np.empty(self.n)
        fl = np.empty(max(self.E, 1))
        es = np.empty(max(self.E, 1))
        L.call("fu_replay_get", self._h, L.ptr(last), L.ptr(fl), L.ptr(es))
        return last, fl[:self.E], es[:self.E]

    def close(self):
        if getattr(self, "_h", None):
            L.lib.fu_replay_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

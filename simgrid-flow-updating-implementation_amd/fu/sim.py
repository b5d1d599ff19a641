"""SimGrid-shaped host surface: the drop-in for the reference scripts' `__main__`.

The reference's entry point (flowupdating-collectall.py:151-166, PW:140-155) is

    e = Engine(sys.argv)
    e.load_platform("./platforms/small_platform.xml")
    e.register_actor("peer", Peer)
    e.load_deployment("./actors.xml")
    e.netzone_root.add_host("observer", 25e6)
    Actor.create("watcher", Host.by_name("observer"), watcher, 1000.0, 10.0)
    e.run_until(10000)

This module keeps that shape. `Peer` is one of the two algorithm classes below, and
`Engine.add_watcher(1000.0, 10.0)` replaces the watcher actor. `run_until` does not step a
discrete-event simulator. It builds the tick schedule natively (fu_trace_build), replays
it on the GPU (fu_replay_*), and prints the watcher's `value{...}` / `last_avg{...}` lines
(CA:134-142) from the GPU snapshots. Log lines use SimGrid's default layout
`[host:actor:(pid) time] [category/PRIORITY] message`; that layout is not verifiable
offline (SimGrid cannot be installed here), so it is best effort.

`Engine(..., sync=True)` runs generation-synchronous rounds on the symmetric union graph
instead (the hot-path kernel), printing one watcher snapshot per `interval` rounds.
"""
from __future__ import annotations

import sys

import numpy as np

from .engine import CollectAll, Replay, Trace
from .platform import (CROSSTRAFFIC, Platform, declared_csr, load_deployment, load_platform,
                       symmetric_union_csr)


class CollectAllPeer:
    """Marker for the collect-all algorithm (flowupdating-collectall.py:22-128)."""
    mode = "collectall"
    TICK_INTERVAL = 1.0  # CA:23
    TICK_TIMEOUT = 50  # CA:24
    not_neighbour_msg = "{sender} was not {name}'s neighbor"  # CA:96


class PairwisePeer:
    """Marker for the pairwise algorithm (flowupdating-pairwise.py:22-117)."""
    mode = "pairwise"
    TICK_INTERVAL = 1.0  # PW:23
    TICK_TIMEOUT = 50.0  # PW:24
    not_neighbour_msg = "{sender} is not {name}'s neighbor"  # PW:96


class _NetZone:
    def __init__(self, engine):
        self._e = engine

    def add_host(self, name, speed=0.0):
        if self._e.platform is None:
            self._e.platform = Platform()
        self._e.platform.add_host(name, speed)
        return name


def _fmt_time(t: float) -> str:
    return f"{t:.6f}"


class Engine:
    """Drop-in for `simgrid.Engine` as the reference scripts use it."""

    def __init__(self, argv=None, *, order: str = "fwd", device: int = 0, sync: bool = False,
                 out=None, allow_unrouted: bool = False, crosstraffic: float = 0.0):
        """allow_unrouted: neighbouring hosts the platform does not route get one-tick delivery
        instead of an error. crosstraffic: SimGrid's network/crosstraffic factor in the link
        model (0 = off, the default here; SimGrid's own default is on, at 0.05, but its effect
        cannot be pinned offline)."""
        self.argv = list(argv or [])
        # engine flags may also come through argv like SimGrid's --cfg (CA:152)
        for a in self.argv[1:]:
            if a.startswith("--fu-order="):
                order = a.split("=", 1)[1]
            elif a.startswith("--fu-device="):
                device = int(a.split("=", 1)[1])
            elif a == "--fu-sync":
                sync = True
            elif a == "--fu-allow-unrouted":
                allow_unrouted = True
            elif a.startswith("--cfg=network/crosstraffic:"):  # SimGrid's own flag
                val = a.split(":", 1)[1].strip().lower()
                crosstraffic = CROSSTRAFFIC if val in ("1", "yes", "true", "on") else 0.0
        self.order = order
        self.device = device
        self.sync = sync
        self.allow_unrouted = allow_unrouted
        self.crosstraffic = float(crosstraffic)
        self.out = out if out is not None else sys.stdout
        self.platform: Platform | None = None
        self.registry = {}
        self.deployment = None
        self.watcher = None
        self.netzone_root = _NetZone(self)
        self.global_values = {}
        self.clock = 0.0
        self.lines: list[str] = []
        self.result = None

    # -- SimGrid-shaped setup -------------------------------------------------------------
    def load_platform(self, path: str):
        self.platform = load_platform(path)

    def register_actor(self, name: str, cls):
        if cls not in (CollectAllPeer, PairwisePeer):
            raise TypeError("register_actor: use fu.CollectAllPeer or fu.PairwisePeer")
        self.registry[name] = cls

    def load_deployment(self, path: str):
        self.deployment = load_deployment(path)
        for a in self.deployment.actors:
            if a.function not in self.registry:
                raise ValueError(f"actor function {a.function!r} is not registered")
            if self.platform is not None and a.host not in self.platform.hosts:
                raise ValueError(f"actor host {a.host!r} is not in the platform")

    def add_watcher(self, run_until: float = 1000.0, interval: float = 10.0,
                    host: str = "observer"):
        """Replaces Actor.create("watcher", Host.by_name("observer"), watcher, 1000.0, 10.0)
        (CA:162): print global_values every `interval` until `run_until`, then kill all."""
        self.watcher = (float(run_until), float(interval), host)

    # -- run --------------------------------------------------------------------------------
    def _emit(self, host, actor, pid, t, prio, msg):
        line = f"[{host}:{actor}:({pid}) {_fmt_time(t)}] [python/{prio}] {msg}"
        self.lines.append(line)
        if self.out is not False:
            print(line, file=self.out)

    def _peer_setup(self):
        if self.deployment is None:
            raise RuntimeError("load_deployment first")
        fns = {a.function for a in self.deployment.actors}
        if len(fns) != 1:
            raise ValueError("exactly one registered actor function is supported")
        fn = fns.pop()
        cls = self.registry[fn]
        names, values, nbrs = self.deployment.peers(fn)
        return cls, fn, names, values, nbrs

    def run_until(self, t_end: float):
        cls, fn, names, values, nbrs = self._peer_setup()
        if self.sync:
            return self._run_sync(cls, names, values, nbrs, t_end)
        n = len(names)
        decl_rp, decl_col = declared_csr(names, nbrs)
        net = None
        if self.platform is not None and self.platform.routes:
            net = self._link_net(names, decl_rp, decl_col)
        if self.watcher is not None:
            w_end, w_int, w_host = self.watcher
            last_tick = int(min(w_end, t_end))
            ticks = last_tick + 1  # peers act at t = 0..last_tick, then the watcher kills
            snap_times = []
            tt = 0.0
            while tt < w_end:  # CA:140-142
                tt = tt + min(w_int, w_end - tt)
                snap_times.append(tt)
        else:
            ticks = int(np.ceil(t_end))
            snap_times = []
            w_host = None
        trace = Trace(decl_rp, decl_col, cls.mode, ticks, self.order, net=net)
        snap_ticks = sorted({int(t) for t in snap_times if int(t) < ticks})
        rep = Replay(trace, values, device=self.device)
        snaps = rep.run(ticks, snapshot_ticks=snap_ticks)
        last, flows, est = rep.state()
        rep.close()
        arr = trace.arrays()
        # tick of every node's first average (presence in global_values["last_avg"])
        first_tick = self._first_fire_ticks(trace, arr)
        order = trace.last_avg_order()
        pid = {nm: i + 1 for i, nm in enumerate(names)}
        # start lines at t = 0 (CA:66-67)
        for i, nm in enumerate(names):
            self._emit(nm, fn, pid[nm], 0.0, "INFO", f"Peer {nm} with value {float(values[i])!r} started.")
        events = self._dynamic_addition_lines(trace, arr, names, cls)
        ev_i = 0
        value_dict = {nm: float(values[i]) for i, nm in enumerate(names)}
        self.global_values = {"value": dict(value_dict)}
        wpid = n + 1
        for tt in snap_times:
            while ev_i < len(events) and events[ev_i][0] <= tt:
                t_e, i_e, msg = events[ev_i]
                self._emit(names[i_e], fn, pid[names[i_e]], float(t_e), "ERROR", msg)
                ev_i += 1
            t_int = int(tt)
            la = {names[i]: float(snaps[t_int][i]) for i in order if first_tick[i] <= t_int}
            gv = {"value": dict(value_dict)}
            if la:
                gv["last_avg"] = la
            for key, d in gv.items():  # CA:134-136
                self._emit(w_host, "watcher", wpid, tt, "INFO", f"{key}{d}")
            self.global_values = gv
        while ev_i < len(events):
            t_e, i_e, msg = events[ev_i]
            self._emit(names[i_e], fn, pid[names[i_e]], float(t_e), "ERROR", msg)
            ev_i += 1
        if self.watcher is not None:
            self._emit(w_host, "watcher", wpid, snap_times[-1] if snap_times else 0.0, "INFO",
                       "Killing every actor but myself.")  # CA:144
        else:
            la = {names[i]: float(last[i]) for i in order}
            self.global_values = {"value": dict(value_dict), **({"last_avg": la} if la else {})}
        self.clock = float(ticks - 1) if self.watcher is not None else float(ticks)
        self.result = {"names": names, "values": values, "last_avg": last, "flows": flows,
                       "estimates": est, "union_rowptr": arr["rowptr"], "union_col": arr["col"],
                       "fires": arr["fires"], "snapshots": snaps, "trace": trace}
        return self.result

    def _run_sync(self, cls, names, values, nbrs, rounds):
        if cls is not CollectAllPeer:
            raise ValueError("synchronous rounds are defined for the collect-all algorithm only")
        rp, col = symmetric_union_csr(names, nbrs)
        eng = CollectAll(rowptr=rp, col=col, values=values, device=self.device)
        interval = int(self.watcher[1]) if self.watcher else int(rounds)
        rounds = int(rounds)
        done = 0
        while done < rounds:
            step = min(interval, rounds - done)
            eng.run(step)
            done += step
            a = eng.estimates()
            self.global_values = {"value": {nm: float(values[i]) for i, nm in enumerate(names)},
                                  "last_avg": {nm: float(a[i]) for i, nm in enumerate(names)}}
            for key, d in self.global_values.items():
                self._emit("observer", "watcher", len(names) + 1, float(done), "INFO", f"{key}{d}")
        self.result = {"names": names, "values": values, "last_avg": eng.estimates(),
                       "flows": eng.flows(), "rowptr": rp, "col": col}
        eng.close()
        return self.result

    # -- helpers ----------------------------------------------------------------------------
    def _link_net(self, names, decl_rp, decl_col):
        """The platform's links and the routes of every pair of actors that exchange messages
        (declared neighbours, both directions: replies go back to the sender), for
        fu_trace_build_links_ex: concurrent transfers share link bandwidth (SimGrid LV08
        factors, shares weighted by the sharing penalty, the TCP window: fu/platform.py). On the reference platform every transfer ends within a tick, so the
        schedule is the plain one (CA:76)."""
        src = np.repeat(np.arange(len(names)), np.diff(decl_rp))
        pairs = set(zip(src.tolist(), np.asarray(decl_col).tolist()))
        pairs |= {(j, i) for i, j in pairs}
        return self.platform.link_net(names, pairs=pairs, allow_unrouted=self.allow_unrouted,
                                      crosstraffic=self.crosstraffic)

    def _route_matrix(self, names):
        """Transfer time (s) of every host pair's route under SimGrid's LV08 model
        (fu/platform.py), or None when every route takes under one tick: then the schedule
        is the plain one-tick delivery of the reference platform (CA:76). Longer routes
        delay consumption by whole ticks (fu_trace_build_routes)."""
        n = len(names)
        hosts = names  # an actor's name is its host (ACT:4-27)
        route = np.zeros((n, n))
        for i in range(n):
            for j in range(n):
                if i != j and (hosts[i], hosts[j]) in self.platform.routes:
                    route[i, j] = self.platform.route_time(hosts[i], hosts[j])
        return route if np.any(route >= 1.0) else None

    @staticmethod
    def _first_fire_ticks(trace, arr):
        n = trace.n
        ft = np.full(n, np.iinfo(np.int64).max, dtype=np.int64)
        tto = arr["tick_task_off"]
        tasks = arr["tasks"]
        ev = arr["events"]
        if len(tasks) == 0:
            return ft
        task_tick = np.searchsorted(tto, np.arange(len(tasks)), side="right") - 1
        fire = ev[:, 0] != 0
        ev_task = np.repeat(np.arange(len(tasks)), tasks[:, 2] - tasks[:, 1])
        nodes = tasks[ev_task, 0][fire]
        ticks = task_tick[ev_task][fire]
        np.minimum.at(ft, nodes, ticks)
        return ft

    @staticmethod
    def _dynamic_addition_lines(trace, arr, names, cls):
        """(tick, node, message) for each receive from an undeclared sender (CA:94-96)."""
        out = []
        tto = arr["tick_task_off"]
        tasks = arr["tasks"]
        ev = arr["events"]
        rp = arr["rowptr"]
        col = arr["col"]
        if len(tasks) == 0:
            return out
        # declared degree = slots that exist before any receive; the generator appends
        # undeclared senders after them in arrival order
        seen = {}
        task_tick = np.searchsorted(tto, np.arange(len(tasks)), side="right") - 1
        decl_deg = trace.decl_deg
        for q in range(len(tasks)):
            node, b, e = (int(x) for x in tasks[q])
            for p in range(b, e):
                if ev[p, 0] != 0:
                    continue
                slot = int(ev[p, 1])
                key = (node, slot)
                if key in seen:
                    continue
                seen[key] = True
                if decl_deg is not None and slot >= decl_deg[node]:
                    sender = names[int(col[rp[node] + slot])]
                    out.append((int(task_tick[q]), node,
                                cls.not_neighbour_msg.format(sender=sender, name=names[node])))
        out.sort(key=lambda x: x[0])
        return out


def run_reference_main(mode: str, platform: str = "./platforms/small_platform.xml",
                       deployment: str = "./actors.xml", run_until: float = 1000.0,
                       interval: float = 10.0, order: str = "fwd", device: int = 0, out=None):
    """The reference `__main__` (CA:151-166 / PW:140-155) on this engine."""
    e = Engine([], order=order, device=device, out=out)
    e.load_platform(platform)
    e.register_actor("peer", CollectAllPeer if mode in ("collectall", "ca") else PairwisePeer)
    e.load_deployment(deployment)
    e.netzone_root.add_host("observer", 25e6)
    e.add_watcher(run_until, interval)
    res = e.run_until(10000)
    line = f"[{_fmt_time(e.clock)}] [python/INFO] Simulation finished"
    e.lines.append(line)
    if e.out is not False:
        print(line, file=e.out)
    return e, res

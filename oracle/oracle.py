"""CPU oracle for the Flow Updating hot path. THIS IS TEST INFRASTRUCTURE.

Only `tests/`, `__graft_entry__.smoke()` and the `cpu_baseline` leg of `bench.py` may import
this module, and only as the checker. The product (`fu` package + `libfu.so`) never calls
it and has no CPU fallback.

It restates the reference's arithmetic and control flow. It does not import the reference.
Parity is PINNED: `tests/test_oracle_golden.py` checks every function here against the
fixtures in `tests/golden/`. Those fixtures were produced by `tests/golden/make_golden.py`,
which drives the reference's own `Peer` objects (flowupdating-collectall.py /
flowupdating-pairwise.py) under a stub `simgrid` module.

Contents
--------
* `ca_sync(...)`: collect-all, generation-synchronous rounds, vectorised
  over nodes by neighbour position. It keeps the reference's left-to-right summation order
  (CA:106, CA:109-111), so results are bitwise equal to the reference.
* `TickEmulator`: a pure-Python restatement of `Peer` (CA:22-128, PW:22-117) and of the
  SimGrid loop/mailbox model. It is meant for small graphs.
* `replay_trace(...)`: replays a product trace (the event format of `include/fu.h`) on the CPU.
  It is the oracle for the GPU replay kernels at sizes the tick emulator cannot reach.
"""
from __future__ import annotations

import math
from collections import deque

import numpy as np

MASK64 = (1 << 64) - 1


# --------------------------------------------------------------------------------------
# helpers
# --------------------------------------------------------------------------------------
def build_rev(rowptr: np.ndarray, col: np.ndarray) -> np.ndarray:
    """rev[e] = index of the reverse edge (col[e] -> i) for a symmetric CSR."""
    n = len(rowptr) - 1
    deg = np.diff(rowptr).astype(np.int64)
    src = np.repeat(np.arange(n, dtype=np.int64), deg)
    dst = col.astype(np.int64)
    key_fwd = src * n + dst
    key_bwd = dst * n + src
    order = np.argsort(key_fwd, kind="stable")
    pos = np.searchsorted(key_fwd[order], key_bwd)
    if np.any(pos >= len(col)) or np.any(key_fwd[order][np.minimum(pos, len(col) - 1)] != key_bwd):
        raise ValueError("graph is not symmetric")
    return order[pos].astype(np.int64)


def splitmix64(state: int):
    state = (state + 0x9E3779B97F4A7C15) & MASK64
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return state, z ^ (z >> 31)


def tick_orders(n: int, order: str, ticks: int):
    """Actor order per tick. 'fwd' = deployment order, 'rev' = reversed, 'rand:S' = a
    Fisher-Yates shuffle per tick driven by SplitMix64(S), j = r % (i+1). Same spec as
    fu_trace.cpp."""
    base = list(range(n))
    if order == "fwd":
        for _ in range(ticks):
            yield base
    elif order == "rev":
        r = base[::-1]
        for _ in range(ticks):
            yield r
    elif order.startswith("rand:"):
        st = int(order.split(":", 1)[1]) & MASK64
        for _ in range(ticks):
            perm = list(base)
            for i in range(n - 1, 0, -1):
                st, r = splitmix64(st)
                j = r % (i + 1)
                perm[i], perm[j] = perm[j], perm[i]
            yield perm
    else:
        raise ValueError(f"unknown tie order {order!r}")


# --------------------------------------------------------------------------------------
# Collect-all, generation-synchronous
# --------------------------------------------------------------------------------------
def ca_sync(rowptr, col, values, rounds: int, rev=None, snapshot_rounds=None):
    """Run `rounds` collect-all rounds from zero state.

    Round 0 is the timeout fire with zero flows/estimates (CA:33-34, CA:90-91, CA:105-128).
    Round r >= 1 is: receive (CA:98-99) f_ij <- -f_ji, e_ij <- a_j; then fire (CA:106-119):
        S = 0.0 + fr[e0] + fr[e1] + ...   (Python sum(), int 0 start, row order; CA:106)
        T = 0.0 + er[e0] + er[e1] + ...   (CA:109-111)
        a = ((v - S) + T) / (deg + 1)     (CA:107, CA:113)
        f[e] = (fr[e] + a) - er[e]        (CA:117)
    Isolated nodes (deg 0) hold a = v.
    Returns (a, f) after the last round, or a dict {r: (a, f)} if snapshot_rounds is given.
    """
    rowptr = np.asarray(rowptr, dtype=np.int64)
    col = np.asarray(col, dtype=np.int64)
    v = np.asarray(values, dtype=np.float64)
    n = len(v)
    deg = np.diff(rowptr)
    if rev is None:
        rev = build_rev(rowptr, col)
    rev = np.asarray(rev, dtype=np.int64)
    denom = (deg + 1).astype(np.float64)
    # nodes sorted by degree (descending): at position k the active rows are a prefix
    order = np.argsort(-deg, kind="stable")
    deg_sorted = deg[order]
    start_sorted = rowptr[:-1][order]
    maxdeg = int(deg.max()) if n else 0
    cnt = np.array([np.count_nonzero(deg_sorted > k) for k in range(maxdeg)], dtype=np.int64)
    src = np.repeat(np.arange(n, dtype=np.int64), deg)
    snaps = {}
    want = set(snapshot_rounds or [])

    a = ((v - 0.0) + 0.0) / denom
    f = np.zeros(len(col), dtype=np.float64)
    f[:] = (0.0 + a[src]) - 0.0
    if 0 in want:
        snaps[0] = (a.copy(), f.copy())
    for r in range(1, rounds):
        fr = -f[rev]
        er = a[col]
        S = np.zeros(n)
        T = np.zeros(n)
        for k in range(maxdeg):
            c = cnt[k]
            idx = start_sorted[:c] + k
            S[:c] = S[:c] + fr[idx]
            T[:c] = T[:c] + er[idx]
        S_full = np.empty(n)
        T_full = np.empty(n)
        S_full[order] = S
        T_full[order] = T
        a_new = ((v - S_full) + T_full) / denom
        f = (fr + a_new[src]) - er
        a = a_new
        if r in want:
            snaps[r] = (a.copy(), f.copy())
    if snapshot_rounds is not None:
        return snaps
    return a, f


def component_targets(rowptr, col, values):
    """Per-node target = exact mean of the node's connected component (math.fsum)."""
    rowptr = np.asarray(rowptr, dtype=np.int64)
    col = np.asarray(col, dtype=np.int64)
    n = len(values)
    comp = np.full(n, -1, dtype=np.int64)
    c = 0
    for s in range(n):
        if comp[s] >= 0:
            continue
        comp[s] = c
        stack = [s]
        while stack:
            u = stack.pop()
            for w in col[rowptr[u]:rowptr[u + 1]]:
                if comp[w] < 0:
                    comp[w] = c
                    stack.append(int(w))
        c += 1
    means = np.zeros(c)
    order = np.argsort(comp, kind="stable")
    bounds = np.searchsorted(comp[order], np.arange(c + 1))
    vals = np.asarray(values, dtype=np.float64)[order]
    for k in range(c):
        seg = vals[bounds[k]:bounds[k + 1]]
        means[k] = math.fsum(seg.tolist()) / len(seg)
    return means[comp], comp


# --------------------------------------------------------------------------------------
# Tick-level emulation (restated Peer + SimGrid loop model)
# --------------------------------------------------------------------------------------
class _Node:
    __slots__ = ("name", "value", "nbrs", "flows", "est", "heard", "count", "last",
                 "last_avg")

    def __init__(self, name, value_str, nbr_names):
        self.name = name
        self.value = float(value_str)  # CA:28
        self.nbrs = list(nbr_names)  # dict insertion order, CA:38-40
        self.flows = {}  # defaultdict(float), CA:33
        self.est = {}  # CA:34
        self.heard = set()  # CA:35
        self.count = 0  # CA:36
        self.last = {}  # PW:35 defaultdict(float)
        self.last_avg = 0.0


class LinkNet:
    """Link-sharing transfer model (fu_trace.cpp LinkNet), restated
    operation for operation so both give the same doubles: a transfer matched at tick t has
    a latency phase of lat_factor * sum(latency), then `bytes` at its max-min fair share of
    bw_factor * bandwidth on the shared links it crosses, capped by its FATPIPE links and,
    with tcp_gamma > 0, by the TCP window tcp_gamma / (2 * latency sum). Shares are weighted
    by 1 / the flow's sharing penalty, LV08's latency sum + weight_S / bandwidth over its
    links (weight_S = 0: penalty 1, equal shares). With crosstraffic c > 0 (SimGrid's
    network/crosstraffic) a flow also loads each shared link of its reverse route with c x
    its rate, and a FATPIPE link of the reverse route alone caps it at bw_factor * bw / c.
    Parity-unpinned against SimGrid (not installable offline)."""

    def __init__(self, net):
        self.n = int(net["n"])
        self.bw = [float(x) for x in net["bw"]]
        self.lat = [float(x) for x in net["lat"]]
        self.shared = [int(x) for x in net["shared"]]
        self.roff = [int(x) for x in net["route_off"]]
        self.rl = [int(x) for x in net["route_links"]]
        self.bytes = float(net.get("bytes", 154.0))
        self.lat_factor = float(net.get("lat_factor", 13.01))
        self.bw_factor = float(net.get("bw_factor", 0.97))
        self.weight_S = float(net.get("weight_S", 0.0))
        self.tcp_gamma = float(net.get("tcp_gamma", 0.0))
        self.cross = float(net.get("crosstraffic", 0.0))
        self.active = []  # flows (dicts) not done, in start order
        self.now = 0.0

    def links(self, f):
        return self.rl[self.roff[f["r"]]:self.roff[f["r"] + 1]]

    def start(self, src, dst, t):
        r = src * self.n + dst
        f = {"r": r, "rate": 0.0, "end": math.inf, "phase": 0, "rem": self.bytes}
        lsum, cap, sw = 0.0, math.inf, 0.0
        f["lk"] = []  # (link, coefficient): its shared route links, then its reverse route's
        for k in self.links(f):
            lsum = lsum + self.lat[k]
            sw = sw + self.weight_S / self.bw[k]
            if not self.shared[k]:
                cap = min(cap, self.bw_factor * self.bw[k])
            else:
                f["lk"].append((k, 1.0))
        if self.cross > 0.0:
            rb = dst * self.n + src
            fwd = self.links(f)
            for k in self.rl[self.roff[rb]:self.roff[rb + 1]]:
                if self.shared[k]:
                    f["lk"].append((k, self.cross))
                elif k not in fwd:
                    cap = min(cap, self.bw_factor * self.bw[k] / self.cross)
        if self.tcp_gamma > 0.0 and lsum > 0.0:
            cap = min(cap, self.tcp_gamma / (2.0 * lsum))
        f["lat_end"] = t + self.lat_factor * lsum
        f["cap"] = cap
        f["pen"] = lsum + sw if self.weight_S > 0.0 else 1.0
        if self.roff[r] == self.roff[r + 1]:  # same host: no transfer
            f["phase"], f["end"] = 2, t
            return f
        self.active.append(f)
        return f

    def _rates(self):
        nl = len(self.bw)
        crem = [self.bw_factor * self.bw[k] for k in range(nl)]
        cnt = [0] * nl
        use = [0.0] * nl
        un = [f for f in self.active if f["phase"] == 1]
        for f in un:
            for k, c in f["lk"]:
                cnt[k] += 1
                use[k] = use[k] + c / f["pen"]
        while un:
            best = math.inf
            for k in range(nl):
                if cnt[k] > 0:
                    best = min(best, max(0.0, crem[k] / use[k]))
            for f in un:
                best = min(best, f["cap"] * f["pen"])
            keep, fix = [], []
            for f in un:
                b = f["cap"] * f["pen"] == best
                for k, _c in f["lk"]:
                    if b:
                        break
                    b = cnt[k] > 0 and max(0.0, crem[k] / use[k]) == best
                (fix if b else keep).append(f)
            for f in fix:
                f["rate"] = f["cap"] if f["cap"] * f["pen"] == best else best / f["pen"]
                for k, c in f["lk"]:
                    crem[k] = crem[k] - c * f["rate"]
                    use[k] = use[k] - c / f["pen"]
                    cnt[k] -= 1
            un = keep

    def advance_to(self, T):
        while True:
            self._rates()
            nx = T
            for f in self.active:
                if f["phase"] == 0:
                    nx = min(nx, f["lat_end"])
                elif f["rate"] > 0.0:
                    nx = min(nx, self.now + f["rem"] / f["rate"])
            dt = nx - self.now
            ev = False
            keep = []
            for f in self.active:
                if f["phase"] == 1:
                    if f["rate"] > 0.0 and self.now + f["rem"] / f["rate"] <= nx:
                        f["phase"], f["end"] = 2, nx
                        ev = True
                        continue
                    f["rem"] = f["rem"] - f["rate"] * dt
                elif f["lat_end"] <= nx:
                    f["phase"] = 1
                    ev = True
                    if not f["rem"] > 0.0:
                        f["phase"], f["end"] = 2, nx
                        continue
                keep.append(f)
            self.active = keep
            self.now = nx
            if not ev:
                return


class TickEmulator:
    """Pure-Python model of the reference run for small graphs.

    actors: list of (host, value_str, "n1,n2,...") in deployment order (ACT:4-27).
    mode: "ca" (collect-all) or "pw" (pairwise).
    """

    def __init__(self, actors, mode: str, faults: str | None = None, route_s=None, net=None):
        """faults: "drop=P,delay=D:Q,seed=S" (extension, not in the reference; same spec and
        draw order as fu_trace.cpp: one U[0,1) draw per put, in put order).
        route_s: optional n x n transfer times in seconds (sender row): a message matched at
        tick t is consumed from tick t + floor(T) + 1 (the reference platform has T < 1 s on
        every route, CA:76; the rule for longer routes is the extension fu_trace_build_routes
        implements, parity unpinned against SimGrid itself)."""
        self.route_s = route_s
        # net: the link model (fu.platform.Platform.link_net; fu_trace_build_links) instead
        self.net = LinkNet(net) if net is not None else None
        if mode not in ("ca", "pw"):
            raise ValueError(mode)
        self.p_drop, self.p_delay, self.d_ticks, self.fstate = 0.0, 0.0, 0, 0
        for kv in filter(None, (faults or "").split(",")):
            k, v = kv.split("=")
            if k == "drop":
                self.p_drop = float(v)
            elif k == "delay":
                d, q = v.split(":")
                self.d_ticks, self.p_delay = int(d), float(q)
            elif k == "seed":
                self.fstate = int(v) & MASK64
            else:
                raise ValueError(kv)
        self.delayed = {}
        self.mode = mode
        self.names = [a[0] for a in actors]
        self.idx = {nm: i for i, nm in enumerate(self.names)}
        self.nodes = []
        for nm, val, neigh in actors:
            nb = neigh.split(",") if len(neigh) else []  # CA:29-31
            self.nodes.append(_Node(nm, val, nb))
        n = len(self.nodes)
        self.fifo = [deque() for _ in range(n)]
        self.comm = [None] * n
        self.t = 0
        self.gv_last_avg = {}  # global_values["last_avg"] in first-assignment order
        self.events = []
        self.fires = [0] * n
        self.errors = 0

    # -- messaging ------------------------------------------------------------------
    def _send(self, src, dst_name, flow, estimate):
        d = self.idx[dst_name]
        msg = (self.names[src], flow, estimate)
        if self.p_drop > 0.0 or self.p_delay > 0.0:
            self.fstate, r = splitmix64(self.fstate)
            u = (r >> 11) * 2.0 ** -53
            if u < self.p_drop:
                return
            if u < self.p_drop + self.p_delay:
                self.delayed.setdefault(self.t + self.d_ticks, []).append((d, msg))
                return
        self._arrive(d, msg)

    def _arrive(self, d, msg):
        c = self.comm[d]
        if c is not None and not c[0]:
            c[0], c[1], c[2] = True, msg, self.t
            if self.net is not None:
                c.append(self.net.start(self.idx[msg[0]], d, float(self.t)))
        else:
            self.fifo[d].append(msg)

    # -- collect-all (CA:87-128) ----------------------------------------------------
    def _ca_fire(self, i):
        nd = self.nodes[i]
        self.fires[i] += 1
        self.events.append((self.t, i, 1, -1))
        s = 0
        for x in nd.nbrs:
            s = s + nd.flows.get(x, 0.0)  # CA:106 (sum() starts from int 0)
        estimate = nd.value - s  # CA:107
        t = 0.0
        for x in nd.nbrs:
            t += nd.est.get(x, 0.0)  # CA:109-111
        avg = (estimate + t) / (len(nd.nbrs) + 1)  # CA:113
        self._set_last_avg(i, avg)  # CA:114
        for x in nd.nbrs:  # CA:116-125
            nf = nd.flows.get(x, 0.0) + avg - nd.est.get(x, 0.0)
            nd.flows[x] = nf
            nd.est[x] = avg
            self._send(i, x, nf, avg)
        nd.heard = set()  # CA:127
        nd.count = 0  # CA:128

    def _ca_tick(self, i):
        nd = self.nodes[i]
        nd.count += 1  # CA:88
        if nd.count >= 50:  # CA:90
            self._ca_fire(i)

    def _ca_receive(self, i, msg):
        nd = self.nodes[i]
        sender, flow, estimate = msg
        if sender not in nd.nbrs:  # CA:94-96
            nd.nbrs.append(sender)
            self.errors += 1
        nd.est[sender] = estimate  # CA:98
        nd.flows[sender] = -flow  # CA:99
        nd.heard.add(sender)  # CA:100
        if nd.heard.issuperset(nd.nbrs):  # CA:102
            self._ca_fire(i)

    # -- pairwise (PW:86-117) -------------------------------------------------------
    def _pw_fire(self, i, x):
        nd = self.nodes[i]
        self.fires[i] += 1
        self.events.append((self.t, i, 1, self.idx[x]))
        s = 0
        for y in nd.nbrs:
            s = s + nd.flows.get(y, 0.0)  # PW:103
        estimate = nd.value - s  # PW:104
        avg = (nd.est.get(x, 0.0) + estimate) / 2.0  # PW:105
        self._set_last_avg(i, avg)  # PW:107
        nd.flows[x] = nd.flows.get(x, 0.0) + avg - nd.est.get(x, 0.0)  # PW:108
        nd.est[x] = avg  # PW:109
        nd.last[x] = float(self.t)  # PW:111
        self._send(i, x, nd.flows[x], avg)  # PW:113-117

    def _pw_tick(self, i):
        nd = self.nodes[i]
        threshold = float(self.t) - 50.0  # PW:87
        for x in list(nd.nbrs):  # PW:89
            if nd.last.get(x, 0.0) < threshold:  # PW:90
                self._pw_fire(i, x)

    def _pw_receive(self, i, msg):
        nd = self.nodes[i]
        sender, flow, estimate = msg
        if sender not in nd.nbrs:  # PW:94-96
            nd.nbrs.append(sender)
            self.errors += 1
        nd.est[sender] = estimate  # PW:98
        nd.flows[sender] = -flow  # PW:99
        self._pw_fire(i, sender)  # PW:100

    def _extra(self, sender_name, i):
        """Whole ticks beyond the first that a transfer sender -> i takes."""
        if self.route_s is None:
            return 0
        T = float(self.route_s[self.idx[sender_name]][i])
        return int(math.floor(T)) if T >= 1.0 else 0

    def _set_last_avg(self, i, avg):
        self.nodes[i].last_avg = avg
        self.gv_last_avg[self.names[i]] = avg  # CA:62 / PW:61

    # -- the loop (CA:70-85 / PW:69-84) --------------------------------
    def run(self, ticks: int, order: str = "fwd", on_tick=None):
        receive = self._ca_receive if self.mode == "ca" else self._pw_receive
        tick = self._ca_tick if self.mode == "ca" else self._pw_tick
        n = len(self.nodes)
        for perm in tick_orders(n, order, ticks):
            if self.net is not None:  # transfers ending before this tick are consumable
                self.net.advance_to(float(self.t))
            for d, msg in self.delayed.pop(self.t, []):
                self._arrive(d, msg)
            for i in perm:
                c = self.comm[i]
                if c is None:  # CA:73-74
                    if self.fifo[i]:
                        c = [True, self.fifo[i].popleft(), self.t]
                        if self.net is not None:
                            c.append(self.net.start(self.idx[c[1][0]], i, float(self.t)))
                    else:
                        c = [False, None, -1]
                    self.comm[i] = c
                if self.net is not None:
                    arrived = c[0] and c[3]["phase"] == 2 and c[3]["end"] < self.t
                else:
                    arrived = c[0] and c[2] + self._extra(c[1][0], i) < self.t
                if arrived:  # CA:76
                    msg = c[1]
                    self.comm[i] = None
                    self.events.append((self.t, i, 0, self.idx[msg[0]]))
                    receive(i, msg)  # CA:82
                tick(i)  # CA:84
            if on_tick is not None:
                on_tick(self.t, self)
            self.t += 1  # CA:85 sleep_for(1.0)
        return self

    def last_avg_items(self):
        return [(self.idx[k], v) for k, v in self.gv_last_avg.items()]


# --------------------------------------------------------------------------------------
# Trace replay (product event format, include/fu.h) on the CPU
# --------------------------------------------------------------------------------------
FU_EV_RECV = 0
FU_EV_FIRE_CA = 1
FU_EV_FIRE_PW = 2


def replay_trace(rowptr, values, tick_task_off, tasks, events, out_ids, n_msgs,
                 snapshot_ticks=()):
    """Replay a product trace on the CPU, sequentially, in event order.

    rowptr: union CSR row pointer (slots per node, insertion order).
    tasks: int32 [n_tasks, 3] = (node, ev_begin, ev_end); tick t owns
        tasks[tick_task_off[t]:tick_task_off[t+1]].
    events: int32 [n_ev, 4] = (kind, slot_or_k, a, b):
        RECV:    (0, slot, msg_in, -)         est[slot] = msg.a ; flow[slot] = -msg.f
        FIRE_CA: (1, k, out_off, -)           average over slots [0, k), send k messages
        FIRE_PW: (2, slot, k, msg_out)        pairwise average with slot, sums slots [0, k)
    out_ids: message ids for FIRE_CA events (k entries from out_off).
    Returns (last_avg, flows, est, snapshots{tick: last_avg copy}).
    """
    rowptr = np.asarray(rowptr, dtype=np.int64)
    v = np.asarray(values, dtype=np.float64)
    n = len(v)
    E = int(rowptr[-1])
    flow = [0.0] * E
    est = [0.0] * E
    last = [0.0] * n
    mf = [0.0] * max(n_msgs, 1)
    ma = [0.0] * max(n_msgs, 1)
    snaps = {}
    want = set(snapshot_ticks)
    rp = rowptr.tolist()
    vv = v.tolist()
    ev = np.asarray(events).tolist()
    tk = np.asarray(tasks).tolist()
    oid = np.asarray(out_ids).tolist()
    T = len(tick_task_off) - 1
    for t in range(T):
        for ti in range(tick_task_off[t], tick_task_off[t + 1]):
            node, b, e = tk[ti]
            base = rp[node]
            for kind, s, a1, a2 in ev[b:e]:
                if kind == FU_EV_RECV:
                    est[base + s] = ma[a1]
                    flow[base + s] = -mf[a1]
                elif kind == FU_EV_FIRE_CA:
                    k = s
                    S = 0.0
                    for q in range(k):
                        S = S + flow[base + q]
                    estimate = vv[node] - S
                    Tsum = 0.0
                    for q in range(k):
                        Tsum += est[base + q]
                    avg = (estimate + Tsum) / (k + 1)
                    last[node] = avg
                    for q in range(k):
                        nf = flow[base + q] + avg - est[base + q]
                        flow[base + q] = nf
                        est[base + q] = avg
                        m = oid[a1 + q]
                        mf[m] = nf
                        ma[m] = avg
                else:
                    k = a1
                    S = 0.0
                    for q in range(k):
                        S = S + flow[base + q]
                    estimate = vv[node] - S
                    avg = (est[base + s] + estimate) / 2.0
                    last[node] = avg
                    nf = flow[base + s] + avg - est[base + s]
                    flow[base + s] = nf
                    est[base + s] = avg
                    mf[a2] = nf
                    ma[a2] = avg
        if t in want:
            snaps[t] = np.array(last)
    return np.array(last), np.array(flow), np.array(est), snaps

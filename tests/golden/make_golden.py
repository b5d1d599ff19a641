#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE's own arithmetic.

This script is test infrastructure. It runs only in the build container, where the
reference checkout exists at /root/reference (override with FU_REFERENCE). Elsewhere it
prints a message and exits 0. Nothing in `tests -m gpu`, `smoke()` or `bench.py` runs it.

How it works
------------
SimGrid 4.0 (requirements.txt:2 of the reference) cannot be installed offline. So this
script puts a small stub `simgrid` module into `sys.modules` and then loads
`flowupdating-collectall.py` / `flowupdating-pairwise.py` with
`importlib.util.spec_from_file_location`. Loading only defines classes; the scripts'
`__main__` blocks (CA:151-166, PW:140-155) do not run. `sys.dont_write_bytecode` is set
first, so no `__pycache__` is written into the reference tree. Only data is written, and
only into tests/golden/.

The script then drives the reference's own `Peer.__init__`, `on_receive`, `tick` and
`avg_and_send` (CA:26-128, PW:26-117) in two ways:

* generation-synchronous rounds (collect-all): every message of generation r is delivered
  before any message of generation r+1. Delivery inside a generation is shuffled. On a
  symmetric graph the result does not depend on that order.
* tick-level emulation of `Peer.loop` (CA:70-85 / PW:69-84) with the mailbox rendez-vous
  model of SURVEY.md Appendix B. The simulated transfer time on every route is in (0, 1) s,
  so a message matched at tick t can be consumed at tick t+1 at the earliest.

The stub stands in for SimGrid only. The arithmetic and the control flow of `on_receive`,
`tick` and `avg_and_send` are the reference's own code.
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import types
from collections import deque

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("FU_REFERENCE", "/root/reference")
CA_FILE = "flowupdating-collectall.py"
PW_FILE = "flowupdating-pairwise.py"

MASK64 = (1 << 64) - 1


# ----------------------------------------------------------------------------------------
# Tie-order RNG shared with the product's trace generator (fu_trace.cpp) and the oracle.
# SplitMix64; a per-tick Fisher-Yates shuffle with j = r % (i + 1).
# ----------------------------------------------------------------------------------------
def splitmix64(state: int) -> tuple[int, int]:
    state = (state + 0x9E3779B97F4A7C15) & MASK64
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return state, z ^ (z >> 31)


def tick_orders(n: int, order: str, ticks: int):
    """Yield the actor order for each tick (same spec as fu_trace.cpp)."""
    base = list(range(n))
    if order == "fwd":
        for _ in range(ticks):
            yield base
    elif order == "rev":
        rev = base[::-1]
        for _ in range(ticks):
            yield rev
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
        raise ValueError(order)


# ----------------------------------------------------------------------------------------
# Stub simgrid
# ----------------------------------------------------------------------------------------
class World:
    current_host = "?"
    router = None
    errors = 0


def _install_stub() -> types.ModuleType:
    sg = types.ModuleType("simgrid")

    class Host:
        def __init__(self, name):
            self.name = name

        @staticmethod
        def by_name(name):
            return Host(name)

    class _Comm:
        pass

    class Mailbox:
        def __init__(self, name):
            self.name = name

        @staticmethod
        def by_name(name):
            return Mailbox(name)

        def put_async(self, payload, size):
            World.router(self.name, payload, size)
            return _Comm()

        def get_async(self):  # the harness emulates the receive side itself
            raise RuntimeError("get_async is driven by the harness")

    class ActivitySet:
        def __init__(self):
            self.count = 0

        def push(self, comm):  # do not keep comms alive (CA:122 FIXME)
            self.count += 1

    class Engine:
        clock = 0.0

    class Actor:
        pass

    class _ThisActor:
        @staticmethod
        def get_host():
            return Host(World.current_host)

        @staticmethod
        def info(msg):
            pass

        @staticmethod
        def error(msg):
            World.errors += 1

    sg.Host = Host
    sg.Mailbox = Mailbox
    sg.ActivitySet = ActivitySet
    sg.Engine = Engine
    sg.Actor = Actor
    sg.this_actor = _ThisActor()
    sys.modules["simgrid"] = sg
    return sg


_counter = 0


def load_reference(fname: str):
    """Load one reference script as a fresh module (fresh `global_values`)."""
    global _counter
    sg = _install_stub()
    _counter += 1
    path = os.path.join(REF, fname)
    spec = importlib.util.spec_from_file_location(f"_fu_ref_{_counter}", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod, sg


# ----------------------------------------------------------------------------------------
# Generation-synchronous collect-all driver
# ----------------------------------------------------------------------------------------
def ca_sync(rowptr, col, values, rounds, seed):
    """Run the reference collect-all Peers generation-synchronously.

    Round 0 is the timeout fire on zero state (CA:87-91 -> CA:105-128). Round r >= 1 fires
    inside `on_receive` once every neighbour has been heard (CA:102-103).
    Returns {r: (last_avg[n], flows[E])} for every r in `rounds` (r = index of the last
    round run, so r = 0 means one round).
    """
    mod, sg = load_reference(CA_FILE)
    n = len(values)
    names = [f"n{i}" for i in range(n)]
    idx = {nm: i for i, nm in enumerate(names)}
    outbox = []
    World.router = lambda dst, p, size: outbox.append((dst, p))
    peers = []
    for i in range(n):
        World.current_host = names[i]
        neigh = ",".join(names[c] for c in col[rowptr[i]:rowptr[i + 1]])
        peers.append(mod.Peer(repr(float(values[i])), neigh))
    rng = np.random.default_rng(seed)
    out = {}
    want = set(rounds)
    last = max(rounds)

    def snap(r):
        la = np.array([peers[i].last_avg for i in range(n)], dtype=np.float64)
        gv = mod.global_values["last_avg"]
        assert all(gv[names[i]] == la[i] or (gv[names[i]] != gv[names[i]]) for i in range(n))
        fl = np.zeros(len(col), dtype=np.float64)
        for i in range(n):
            for e in range(rowptr[i], rowptr[i + 1]):
                fl[e] = peers[i].flows[names[col[e]]]
        out[r] = (la, fl)

    for i in rng.permutation(n):
        peers[i].avg_and_send()
    if 0 in want:
        snap(0)
    for r in range(1, last + 1):
        msgs = outbox[:]
        outbox.clear()
        order = rng.permutation(len(msgs))
        for k in order:
            dst, p = msgs[k]
            peers[idx[dst]].on_receive(p)
        # every non-isolated node fired exactly once in this generation
        assert len(outbox) == len(msgs), (len(outbox), len(msgs))
        if r in want:
            snap(r)
    return out


# ----------------------------------------------------------------------------------------
# Tick-level emulation of Peer.loop
# ----------------------------------------------------------------------------------------
def tick_emulation(mode, actors, ticks, order, track_flows=False):
    """Drive reference Peers through the emulated SimGrid loop for ticks 0..ticks-1.

    actors: list of (host_name, value_str, neighbours_str) in deployment order.
    Returns a dict with per-tick snapshots (after every actor acted at that tick) of
    global_values['last_avg'] (as ordered key/value lists), the event log, the final
    neighbour order per actor, final flows/estimates and fire counts.
    """
    mod, sg = load_reference(CA_FILE if mode == "ca" else PW_FILE)
    names = [a[0] for a in actors]
    aidx = {nm: i for i, nm in enumerate(names)}
    n = len(actors)
    peers = []
    World.errors = 0
    for nm, val, neigh in actors:
        World.current_host = nm
        peers.append(mod.Peer(val, neigh))
    fifo = [deque() for _ in range(n)]
    comm = [None] * n  # None | [matched: bool, payload, match_tick]
    events = []  # (tick, actor, kind, other): kind 0 = receive (other = sender), 1 = fire (other = neighbour or -1)
    cur = {"t": 0}

    def router(dst, payload, size):
        d = aidx[dst]
        c = comm[d]
        if c is not None and not c[0]:
            c[0] = True
            c[1] = payload
            c[2] = cur["t"]
        else:
            fifo[d].append(payload)

    World.router = router
    fires = [0] * n

    def wrap(i):
        orig = peers[i].avg_and_send

        def counted(*args):
            fires[i] += 1
            events.append((cur["t"], i, 1, aidx[args[0]] if args else -1))
            return orig(*args)

        peers[i].avg_and_send = counted

    for i in range(n):
        wrap(i)

    snaps_keys = []
    snaps_vals = []
    for t, perm in enumerate(tick_orders(n, order, ticks)):
        cur["t"] = t
        sg.Engine.clock = float(t)
        for i in perm:
            World.current_host = names[i]
            c = comm[i]
            if c is None:
                if fifo[i]:
                    c = [True, fifo[i].popleft(), t]
                else:
                    c = [False, None, -1]
                comm[i] = c
            if c[0] and c[2] < t:
                msg = c[1]
                comm[i] = None
                if type(msg) is mod.FlowUpdatingMsg:
                    events.append((t, i, 0, aidx[msg.sender]))
                    peers[i].on_receive(msg)
            peers[i].tick()
        la = mod.global_values["last_avg"]
        snaps_keys.append([aidx[k] for k in la.keys()])
        snaps_vals.append([la[k] for k in la.keys()])
    res = {
        "names": names,
        "values": [mod.global_values["value"][nm] for nm in names],
        "value_keys": [aidx[k] for k in mod.global_values["value"].keys()],
        "snap_keys": snaps_keys,
        "snap_vals": snaps_vals,
        "events": events,
        "fires": fires,
        "neighbors": [[aidx[k] for k in p.neighbors.keys()] for p in peers],
        "flows": [[p.flows[k] for k in p.neighbors.keys()] for p in peers],
        "estimates": [[p.estimates[k] for k in p.neighbors.keys()] for p in peers],
        "errors_logged": World.errors,
        "queued_at_end": [len(q) for q in fifo],
    }
    return res


# ----------------------------------------------------------------------------------------
# Graphs used for fixtures (the fixture stores the graph, so these need not match the
# product's generators)
# ----------------------------------------------------------------------------------------
def csr_from_pairs(n, pairs, rng=None, shuffle_rows=False):
    adj = [set() for _ in range(n)]
    for u, v in pairs:
        if u == v:
            continue
        adj[u].add(v)
        adj[v].add(u)
    rowptr = [0]
    col = []
    for i in range(n):
        row = sorted(adj[i])
        if shuffle_rows and rng is not None:
            row = list(rng.permutation(row)) if row else []
        col.extend(int(c) for c in row)
        rowptr.append(len(col))
    return np.array(rowptr, dtype=np.int32), np.array(col, dtype=np.int32)


def random_regular_pairs(n, d, rng):
    # configuration model with retries until simple
    while True:
        stubs = np.repeat(np.arange(n), d)
        rng.shuffle(stubs)
        pairs = stubs.reshape(-1, 2)
        if np.any(pairs[:, 0] == pairs[:, 1]):
            continue
        key = np.minimum(pairs[:, 0], pairs[:, 1]) * n + np.maximum(pairs[:, 0], pairs[:, 1])
        if len(np.unique(key)) == len(key):
            return [tuple(map(int, p)) for p in pairs]


def er_pairs(n, m, rng):
    return [(int(rng.integers(n)), int(rng.integers(n))) for _ in range(m)]


def rmat_pairs(scale, ef, rng, abcd=(0.57, 0.19, 0.19, 0.05)):
    n = 1 << scale
    a, b, c, _ = abcd
    pairs = []
    for _ in range(n * ef):
        u = v = 0
        for _lvl in range(scale):
            r = rng.random()
            u <<= 1
            v <<= 1
            if r < a:
                pass
            elif r < a + b:
                v |= 1
            elif r < a + b + c:
                u |= 1
            else:
                u |= 1
                v |= 1
        pairs.append((u, v))
    return n, pairs


def values_for(n, rng, special=False):
    v = rng.random(n) * 100.0
    if special and n >= 8:
        v[0] = -37.25
        v[1] = 1e15 + 0.5
        v[2] = 1e-300
        v[3] = 0.0
        v[4] = 123456789.123456789
    return v


def parse_actors_xml(path):
    import xml.etree.ElementTree as ET

    root = ET.parse(path).getroot()
    out = []
    for a in root.iter("actor"):
        args = [x.get("value") for x in a.findall("argument")]
        out.append((a.get("host"), args[0], args[1] if len(args) > 1 else ""))
    return out


def platform_summary():
    """Hosts / links / routes of the reference platform (PLAT:4-193) as a JSON fixture, so
    tests can rebuild an equivalent platform without the reference tree."""
    import xml.etree.ElementTree as ET

    root = ET.parse(os.path.join(REF, "platforms", "small_platform.xml")).getroot()
    zone = next(root.iter("zone"))
    out = {
        "routing": zone.get("routing"),
        "hosts": [[h.get("id"), h.get("speed")] for h in root.iter("host")],
        "links": [[ln.get("id"), ln.get("bandwidth"), ln.get("latency"), ln.get("sharing_policy")]
                  for ln in root.iter("link")],
        "routes": [[r.get("src"), r.get("dst"), [c.get("id") for c in r.findall("link_ctn")]]
                   for r in root.iter("route")],
    }
    with open(os.path.join(HERE, "small_platform_summary.json"), "w") as f:
        json.dump(out, f, indent=0)


def main():
    if not os.path.isfile(os.path.join(REF, CA_FILE)):
        print(f"make_golden: reference not found at {REF}; nothing to do")
        return 0
    platform_summary()
    if "--only-platform" in sys.argv:
        return 0
    rng = np.random.default_rng(20250629)

    # ---------------- generation-synchronous collect-all ----------------
    graphs = {}
    n = 64
    graphs["rr64_d4"] = (n, random_regular_pairs(n, 4, rng), False)
    graphs["rr256_d8_shuffled"] = (256, random_regular_pairs(256, 8, rng), True)
    graphs["er300_m450"] = (300, er_pairs(300, 450, rng), False)  # isolated nodes + small comps
    graphs["star_257"] = (258, [(0, i) for i in range(1, 258)], False)  # hub deg 257 > wave
    graphs["star_1500"] = (1501, [(0, i) for i in range(1, 1501)], False)  # hub deg 1500
    graphs["k8"] = (8, [(i, j) for i in range(8) for j in range(i + 1, 8)], False)
    graphs["path40"] = (40, [(i, i + 1) for i in range(39)], False)
    ns, rp = rmat_pairs(9, 8, rng)
    graphs["rmat9_ef8"] = (ns, rp, False)
    rounds = [0, 1, 2, 4, 9, 29, 59]
    manifest = {"ca_sync": {}, "tick": {}}
    for name, (gn, pairs, shuf) in graphs.items():
        rowptr, col = csr_from_pairs(gn, pairs, rng, shuffle_rows=shuf)
        vals = values_for(gn, rng, special=(name == "rr64_d4"))
        res = ca_sync(rowptr, col, vals, rounds, seed=int(rng.integers(1 << 31)))
        la = np.stack([res[r][0] for r in rounds])
        fl = np.stack([res[r][1] for r in rounds])
        fn = f"ca_sync_{name}.npz"
        np.savez_compressed(os.path.join(HERE, fn), rowptr=rowptr, col=col, values=vals,
                            rounds=np.array(rounds, dtype=np.int32), last_avg=la, flows=fl)
        manifest["ca_sync"][name] = {"file": fn, "n": int(gn), "E": int(len(col)),
                                     "max_deg": int(np.diff(rowptr).max())}
        print("ca_sync", name, gn, len(col))

    # ---------------- tick-level emulation ----------------
    actors = parse_actors_xml(os.path.join(REF, "actors.xml"))
    for mode in ("ca", "pw"):
        for order in ("fwd", "rev", "rand:7"):
            res = tick_emulation(mode, actors, 1001, order)
            tag = order.replace(":", "")
            fn = f"tick_small_platform_{mode}_{tag}.json"
            with open(os.path.join(HERE, fn), "w") as f:
                json.dump({"mode": mode, "order": order, "ticks": 1001, "actors": actors, **res}, f)
            manifest["tick"][f"small_platform_{mode}_{tag}"] = fn
            print("tick", mode, order, "fires", res["fires"])

    # small random-regular graph and a random asymmetric digraph, both modes
    def actors_from_csr(rowptr, col, vals, prefix="h"):
        return [(f"{prefix}{i}", repr(float(vals[i])),
                 ",".join(f"{prefix}{c}" for c in col[rowptr[i]:rowptr[i + 1]]))
                for i in range(len(vals))]

    rowptr, col = csr_from_pairs(32, random_regular_pairs(32, 4, rng), rng, shuffle_rows=True)
    rr_actors = actors_from_csr(rowptr, col, values_for(32, rng))
    # asymmetric: each node declares a random subset of out-neighbours
    na = 12
    asym = []
    avals = values_for(na, rng)
    for i in range(na):
        k = int(rng.integers(0, 4))
        outs = [int(x) for x in rng.choice([j for j in range(na) if j != i], size=k, replace=False)]
        asym.append((f"a{i}", repr(float(avals[i])), ",".join(f"a{j}" for j in outs)))
    for gname, acts, ticks in (("rr32_d4", rr_actors, 400), ("asym12", asym, 400)):
        for mode in ("ca", "pw"):
            for order in ("fwd", "rand:11"):
                res = tick_emulation(mode, acts, ticks, order)
                tag = order.replace(":", "")
                fn = f"tick_{gname}_{mode}_{tag}.json"
                with open(os.path.join(HERE, fn), "w") as f:
                    json.dump({"mode": mode, "order": order, "ticks": ticks, "actors": acts, **res}, f)
                manifest["tick"][f"{gname}_{mode}_{tag}"] = fn
                print("tick", gname, mode, order, "events", len(res["events"]))

    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""The native tick-trace generator (fu_trace_build) against the reference runs.

The fixtures hold the event log of the reference's own Peer objects driven tick by tick.
The trace must reproduce that log event for event. Replaying the trace with the oracle's
replay (C and Python) must reproduce every per-tick snapshot of global_values['last_avg']
bitwise.
"""
import numpy as np
import pytest

import coracle
import fu
import oracle
from conftest import fixture_decl_csr, load_json, tick_fixtures, trace_events_as_log


@pytest.mark.parametrize("name,fn", tick_fixtures())
def test_trace_matches_reference_event_log(name, fn):
    d = load_json(fn)
    names, vals, rp, col = fixture_decl_csr(d)
    tr = fu.Trace(rp, col, "collectall" if d["mode"] == "ca" else "pairwise", d["ticks"],
                  d["order"])
    a = tr.arrays()
    assert trace_events_as_log(a) == d["events"]
    assert list(a["fires"]) == d["fires"]
    # union rows in insertion order (declared, then first arrival: CA:94-95)
    rows = [list(a["col"][a["rowptr"][i]:a["rowptr"][i + 1]]) for i in range(tr.n)]
    assert rows == d["neighbors"]
    # key order of global_values["last_avg"] = order of first average
    assert tr.last_avg_order() == d["snap_keys"][-1]
    assert tr.dynamic_additions == d["errors_logged"]


@pytest.mark.parametrize("name,fn", tick_fixtures())
def test_trace_replay_oracle_matches_snapshots(name, fn):
    d = load_json(fn)
    names, vals, rp, col = fixture_decl_csr(d)
    tr = fu.Trace(rp, col, "collectall" if d["mode"] == "ca" else "pairwise", d["ticks"],
                  d["order"])
    a = tr.arrays()
    ticks = list(range(d["ticks"]))
    last, flow, est, snaps = coracle.replay(a["rowptr"], vals, a["tick_task_off"], a["tasks"],
                                            a["events"], a["out_ids"], tr.n_msgs, ticks)
    for t in ticks:
        keys = d["snap_keys"][t]
        assert [float(snaps[t][i]) for i in keys] == d["snap_vals"][t], (name, t)
    # final flows per neighbour slot
    for i in range(tr.n):
        assert list(flow[a["rowptr"][i]:a["rowptr"][i + 1]]) == d["flows"][i]


def test_trace_order_rand_is_deterministic():
    rp = np.array([0, 2, 4, 6], dtype=np.int64)
    col = np.array([1, 2, 0, 2, 0, 1], dtype=np.int32)
    t1 = fu.Trace(rp, col, "pairwise", 200, "rand:5").arrays()
    t2 = fu.Trace(rp, col, "pairwise", 200, "rand:5").arrays()
    assert np.array_equal(t1["events"], t2["events"])
    t3 = fu.Trace(rp, col, "pairwise", 200, "rand:6").arrays()
    assert not np.array_equal(t1["tasks"], t3["tasks"])


def test_trace_conflict_free_batches():
    """One task per node per tick, and no message slot is written and read in one tick."""
    g = fu.Graph.random_regular(512, 6, seed=3)
    tr = fu.Trace(g.rowptr, g.col, "pairwise", 150, "rand:1")
    a = tr.arrays()
    tto, tasks, ev, oids = a["tick_task_off"], a["tasks"], a["events"], a["out_ids"]
    for t in range(tr.ticks):
        tk = tasks[tto[t]:tto[t + 1]]
        assert len(np.unique(tk[:, 0])) == len(tk)
        reads, writes = set(), set()
        for node, b, e in tk:
            for p in range(b, e):
                if ev[p, 0] == 0:
                    reads.add(int(ev[p, 2]))
                elif ev[p, 0] == 2:
                    writes.add(int(ev[p, 3]))
                else:
                    writes.update(int(x) for x in oids[ev[p, 2]:ev[p, 2] + ev[p, 1]])
        assert not (reads & writes), t


def test_trace_pairwise_rr_oracles_agree():
    """C and Python replays agree on a mid-size pairwise trace (RR n=256, d=8)."""
    g = fu.Graph.random_regular(256, 8, seed=7)
    v = fu.uniform_values(g.n, seed=3)
    tr = fu.Trace(g.rowptr, g.col, "pairwise", 300, "fwd")
    a = tr.arrays()
    l1, f1, e1, _ = coracle.replay(a["rowptr"], v, a["tick_task_off"], a["tasks"], a["events"],
                                   a["out_ids"], tr.n_msgs)
    l2, f2, e2, _ = oracle.replay_trace(a["rowptr"], v, a["tick_task_off"], a["tasks"],
                                        a["events"], a["out_ids"], tr.n_msgs)
    assert np.array_equal(l1, l2) and np.array_equal(f1, f2) and np.array_equal(e1, e2)


def test_trace_bad_inputs():
    rp = np.array([0, 1, 2], dtype=np.int64)
    with pytest.raises(fu.FuError):
        fu.Trace(rp, np.array([0, 0], dtype=np.int32), "pairwise", 10)  # self-loop
    with pytest.raises(fu.FuError):
        fu.Trace(rp, np.array([1, 5], dtype=np.int32), "pairwise", 10)  # out of range
    with pytest.raises(fu.FuError):
        fu.Trace(rp, np.array([1, 0], dtype=np.int32), "pairwise", 10, "sideways")


@pytest.mark.parametrize("mode", ["collectall", "pairwise"])
@pytest.mark.parametrize("faults", ["drop=0.1,seed=5", "delay=3:0.2,seed=9", "drop=0.05,delay=7:0.1,seed=1"])
def test_fault_injection_matches_emulator(mode, faults):
    """Fault injection (§8(f)): the native trace and the oracle emulator draw the same faults
    in put order; events and per-tick estimates agree exactly, and the run still converges
    through the timeouts (CA:87-91, PW:86-91)."""
    d = load_json("tick_small_platform_ca_fwd.json")
    names, vals, rp, col = fixture_decl_csr(d)
    em = oracle.TickEmulator(d["actors"], "ca" if mode == "collectall" else "pw", faults=faults)
    snaps = {}

    def cb(t, e):
        if t % 50 == 0 or t == 1999:
            snaps[t] = dict(e.last_avg_items())

    em.run(2000, "fwd", on_tick=cb)
    tr = fu.Trace(rp, col, mode, 2000, "fwd", faults=faults)
    a = tr.arrays()
    assert trace_events_as_log(a) == [list(x) for x in em.events]
    assert tr.dropped + tr.delayed > 0
    ticks = sorted(snaps)
    last, flow, est, s2 = coracle.replay(a["rowptr"], vals, a["tick_task_off"], a["tasks"], a["events"],
                                         a["out_ids"], tr.n_msgs, ticks)
    for t in ticks:
        for i, v in snaps[t].items():
            assert s2[t][i] == v
    # self-healing: still converges to the mean despite lost messages
    mean = sum(vals) / len(vals)
    assert max(abs(x - mean) for x in snaps[1999].values()) / mean < 1e-6


def test_fault_spec_errors():
    rp = np.array([0, 1, 2], dtype=np.int64)
    col = np.array([1, 0], dtype=np.int32)
    for bad in ("drop=2", "delay=0:0.1", "junk=1", "drop=0.6,delay=1:0.6"):
        with pytest.raises(fu.FuError, match="faults"):
            fu.Trace(rp, col, "pairwise", 10, faults=bad)


@pytest.mark.parametrize("mode", ["collectall", "pairwise"])
@pytest.mark.parametrize("order", ["fwd", "rand:3"])
def test_route_times_match_emulator(mode, order):
    """Route transfer times of one tick or more (§8(f) row 3, fu_trace_build_routes): a message
    matched at tick t is consumed from tick t + floor(T) + 1. The native trace and the oracle
    emulator agree event for event and snapshot for snapshot; every route under one tick
    gives the plain schedule of the reference platform (CA:76)."""
    d = load_json("tick_small_platform_ca_fwd.json")
    names, vals, rp, col = fixture_decl_csr(d)
    n = len(names)
    rng = np.random.default_rng(11)
    route = rng.uniform(0.0, 3.7, (n, n))
    np.fill_diagonal(route, 0.0)
    em = oracle.TickEmulator(d["actors"], "ca" if mode == "collectall" else "pw", route_s=route)
    snaps = {}

    def cb(t, e):
        if t % 50 == 0 or t == 2999:
            snaps[t] = dict(e.last_avg_items())

    em.run(3000, order, on_tick=cb)
    tr = fu.Trace(rp, col, mode, 3000, order, route_s=route)
    a = tr.arrays()
    assert trace_events_as_log(a) == [list(x) for x in em.events]
    ticks = sorted(snaps)
    last, flow, est, s2 = coracle.replay(a["rowptr"], vals, a["tick_task_off"], a["tasks"], a["events"],
                                         a["out_ids"], tr.n_msgs, ticks)
    for t in ticks:
        for i, v in snaps[t].items():
            assert s2[t][i] == v
    mean = sum(vals) / len(vals)
    assert max(abs(x - mean) for x in snaps[2999].values()) / mean < 1e-9
    # all routes under one tick: the same trace as without route times
    fast = fu.Trace(rp, col, mode, 600, order, route_s=np.full((n, n), 0.9)).arrays()
    plain = fu.Trace(rp, col, mode, 600, order).arrays()
    for k in ("tick_task_off", "tasks", "events", "out_ids"):
        assert np.array_equal(fast[k], plain[k])
    with pytest.raises(ValueError):
        fu.Trace(rp, col, mode, 10, order, route_s=np.zeros((n, n + 1)))


def _random_net(n, seed, slow):
    """A random platform for the link model: 6-9 links (some FATPIPE), a route of 1-4
    links for every ordered host pair. slow: bandwidths low enough (200 B/s - 2 kB/s) that
    sharing moves deliveries by whole ticks."""
    rng = np.random.default_rng(seed)
    nl = int(rng.integers(6, 10))
    bw = rng.uniform(60.0, 400.0, nl) if slow else rng.uniform(1e6, 1e9, nl)
    lat = rng.uniform(0.0, 0.06 if slow else 0.015, nl)  # fast: 13.01 x 4 x 15 ms < 1 s
    shared = (rng.uniform(size=nl) > 0.25).astype(np.int32)
    off, lst = [0], []
    for i in range(n):
        for j in range(n):
            if i != j:
                lst.extend(rng.choice(nl, size=int(rng.integers(1, 5)), replace=False).tolist())
            off.append(len(lst))
    return {"n": n, "bw": bw, "lat": lat, "shared": shared, "route_off": np.array(off, dtype=np.int64),
            "route_links": np.array(lst, dtype=np.int32), "bytes": 154.0, "lat_factor": 13.01,
            "bw_factor": 0.97}


@pytest.mark.parametrize("lv08", [False, True, "cross"])
@pytest.mark.parametrize("mode", ["collectall", "pairwise"])
@pytest.mark.parametrize("order", ["fwd", "rand:5"])
@pytest.mark.parametrize("seed", [1, 2])
def test_link_sharing_matches_emulator(mode, order, seed, lv08):
    """Link sharing (§8(f) row 3, fu_trace_build_links): concurrent transfers split the
    shared links' bandwidth max-min fairly (FATPIPE links cap each transfer alone), so a
    message's delivery tick depends on the traffic beside it. The native builder and the
    oracle emulator (LinkNet, the same operations in the same order) agree event for event
    and snapshot for snapshot over 2000 ticks, with fault injection on the asymmetric
    12-node fixture. Parity-unpinned against SimGrid itself (not installable offline)."""
    d = load_json("tick_asym12_ca_fwd.json") if seed == 2 else load_json("tick_small_platform_ca_fwd.json")
    names, vals, rp, col = fixture_decl_csr(d)
    n = len(names)
    net = _random_net(n, seed, slow=True)
    if lv08:  # shares weighted by the sharing penalty, the TCP window (fu_trace_build_links_ex)
        net = dict(net, weight_S=fu.platform.LV08_WEIGHT_S, tcp_gamma=fu.platform.TCP_GAMMA)
    if lv08 == "cross":  # and SimGrid's crosstraffic (fu_trace_build_links_cross)
        net = dict(net, crosstraffic=fu.platform.CROSSTRAFFIC)
    faults = "drop=0.05,delay=3:0.05,seed=4" if seed == 2 else None
    em = oracle.TickEmulator(d["actors"], "ca" if mode == "collectall" else "pw", faults=faults, net=net)
    snaps = {}

    def cb(t, e):
        if t % 100 == 0 or t == 1999:
            snaps[t] = dict(e.last_avg_items())

    em.run(2000, order, on_tick=cb)
    tr = fu.Trace(rp, col, mode, 2000, order, faults=faults, net=net)
    a = tr.arrays()
    assert trace_events_as_log(a) == [list(x) for x in em.events]
    ticks = sorted(snaps)
    _, _, _, s2 = coracle.replay(a["rowptr"], vals, a["tick_task_off"], a["tasks"], a["events"], a["out_ids"],
                                 tr.n_msgs, ticks)
    for t in ticks:
        for i, v in snaps[t].items():
            assert s2[t][i] == v
    # sharing matters here: the same links without it (each transfer alone, its route time)
    # give another schedule
    rt = np.zeros((n, n))
    for i in range(n):
        for j in range(n):
            if i != j:
                ks = net["route_links"][net["route_off"][i * n + j]:net["route_off"][i * n + j + 1]]
                rt[i, j] = 13.01 * sum(net["lat"][k] for k in ks) + 154.0 / (0.97 * min(net["bw"][k] for k in ks))
    alone = fu.Trace(rp, col, mode, 2000, order, faults=faults, route_s=rt).arrays()
    assert not (np.array_equal(alone["tick_task_off"], a["tick_task_off"])
                and np.array_equal(alone["events"], a["events"]))
    if lv08:  # and the weighting matters: equal shares give another schedule
        eq = fu.Trace(rp, col, mode, 2000, order, faults=faults, net=_random_net(n, seed, slow=True)).arrays()
        assert not (np.array_equal(eq["tick_task_off"], a["tick_task_off"])
                    and np.array_equal(eq["events"], a["events"]))
    if lv08 == "cross":  # and so does the crosstraffic: without it another schedule
        nc = fu.Trace(rp, col, mode, 2000, order, faults=faults, net=dict(net, crosstraffic=0.0)).arrays()
        assert not (np.array_equal(nc["tick_task_off"], a["tick_task_off"])
                    and np.array_equal(nc["events"], a["events"]))


@pytest.mark.parametrize("mode", ["collectall", "pairwise"])
def test_link_model_fast_links_give_the_plain_schedule(mode, tmp_path):
    """Links fast enough that every transfer ends within a tick (the reference platform:
    PLAT:13-36) give exactly the plain schedule, and the reference platform itself does too."""
    from conftest import write_platform_xml

    d = load_json("tick_small_platform_ca_fwd.json")
    names, vals, rp, col = fixture_decl_csr(d)
    n = len(names)
    plain = fu.Trace(rp, col, mode, 800, "rand:2").arrays()
    for net in (_random_net(n, 9, slow=False), None):
        if net is None:
            plat = tmp_path / "small_platform.xml"
            write_platform_xml(plat)
            net = fu.platform.load_platform(str(plat)).link_net(names)
        got = fu.Trace(rp, col, mode, 800, "rand:2", net=net).arrays()
        for k in ("tick_task_off", "tasks", "events", "out_ids"):
            assert np.array_equal(got[k], plain[k])


def test_link_model_single_transfer_time_and_sharing():
    """One transfer alone takes the per-route LV08 time; two at once on one shared link take
    longer each, a FATPIPE link does not slow them down. Checked on the emulator's LinkNet
    (the native builder equals it event for event, test above)."""
    net = {"n": 3, "bw": np.array([100.0, 100.0]), "lat": np.array([0.01, 0.0]), "shared": np.array([1, 0]),
           "route_off": np.array([0, 0, 1, 2, 3, 3, 4, 5, 6, 6]), "route_links": np.array([0, 0, 0, 1, 1, 1]),
           "bytes": 154.0, "lat_factor": 13.01, "bw_factor": 0.97}
    ln = oracle.LinkNet(net)
    f = ln.start(0, 1, 0.0)
    ln.advance_to(10.0)
    assert f["end"] == pytest.approx(13.01 * 0.01 + 154.0 / 97.0)
    ln = oracle.LinkNet(net)
    f1, f2 = ln.start(0, 1, 0.0), ln.start(1, 0, 0.0)  # both on shared link 0
    ln.advance_to(10.0)
    assert f1["end"] == f2["end"] == pytest.approx(13.01 * 0.01 + 2 * 154.0 / 97.0)
    ln = oracle.LinkNet(net)
    f1, f2 = ln.start(1, 2, 0.0), ln.start(2, 1, 0.0)  # both on FATPIPE link 1
    ln.advance_to(10.0)
    assert f1["end"] == f2["end"] == pytest.approx(154.0 / 97.0)


def test_link_model_lv08_weights_and_tcp_window():
    """LV08's weighting: two transfers on one shared link split it in proportion to 1 / their
    sharing penalties (latency sum + weight_S / bandwidth of each route link), so the one
    that also crosses a slow FATPIPE link gets the smaller share; the TCP window caps a
    transfer at gamma / (2 * latency sum). Weighted schedules differ from equal shares."""
    W, G = fu.platform.LV08_WEIGHT_S, fu.platform.TCP_GAMMA
    # links: 0 shared (1000 B/s, 10 ms), 1 FATPIPE (2000 B/s, 0 s); route 0->1: [0],
    # route 1->0: [0, 1] (0 -> 2 and the rest: unused)
    net = {"n": 3, "bw": np.array([1000.0, 2000.0]), "lat": np.array([0.01, 0.0]), "shared": np.array([1, 0]),
           "route_off": np.array([0, 0, 1, 1, 3, 3, 3, 3, 3, 3]), "route_links": np.array([0, 0, 1]),
           "bytes": 1e6, "lat_factor": 13.01, "bw_factor": 0.97, "weight_S": W, "tcp_gamma": 0.0}
    ln = oracle.LinkNet(net)
    f1, f2 = ln.start(0, 1, 0.0), ln.start(1, 0, 0.0)
    ln.advance_to(0.2)  # both past their latency phase (13.01 x 10 ms)
    p1, p2 = 0.01 + W / 1000.0, 0.01 + W / 1000.0 + W / 2000.0
    assert f1["pen"] == p1 and f2["pen"] == p2
    assert f1["rate"] / f2["rate"] == pytest.approx(p2 / p1)
    assert f1["rate"] + f2["rate"] == pytest.approx(0.97 * 1000.0)
    eq = oracle.LinkNet(dict(net, weight_S=0.0))
    g1, g2 = eq.start(0, 1, 0.0), eq.start(1, 0, 0.0)
    eq.advance_to(0.2)
    assert g1["rate"] == g2["rate"] == 0.97 * 1000.0 / 2
    # the TCP window: gamma / (2 x 10 ms) = 210 MB/s caps a 1 GB/s link
    fast = dict(net, bw=np.array([1e9, 2e9]), tcp_gamma=G)
    ln = oracle.LinkNet(fast)
    f = ln.start(0, 1, 0.0)
    ln.advance_to(0.2)
    assert f["rate"] == G / (2.0 * 0.01) < 0.97 * 1e9


def test_link_model_crosstraffic_loads_the_reverse_route():
    """SimGrid's network/crosstraffic (fu_trace_build_links_cross): a transfer also loads the
    shared links of its reverse route with 0.05 of its rate. Two opposite transfers over two
    one-way links (0 -> 1 on link 0, 1 -> 0 on link 1) each see the other's acknowledgements:
    rate x + 0.05 y <= C on each link gives x = y = C / 1.05; without it each has its link
    alone. A FATPIPE link on the reverse route only caps a transfer at C / 0.05. Checked on
    the emulator's LinkNet; the native builder equals it event for event (test above)."""
    C = 0.97 * 1000.0
    net = {"n": 2, "bw": np.array([1000.0, 1000.0]), "lat": np.array([0.0, 0.0]), "shared": np.array([1, 1]),
           "route_off": np.array([0, 0, 1, 2, 2]), "route_links": np.array([0, 1]),
           "bytes": 1e4, "lat_factor": 13.01, "bw_factor": 0.97, "crosstraffic": 0.05}
    ln = oracle.LinkNet(net)
    f1, f2 = ln.start(0, 1, 0.0), ln.start(1, 0, 0.0)
    ln.advance_to(0.001)
    assert f1["rate"] == pytest.approx(C / 1.05) and f2["rate"] == pytest.approx(C / 1.05)
    off = oracle.LinkNet(dict(net, crosstraffic=0.0))
    g1, g2 = off.start(0, 1, 0.0), off.start(1, 0, 0.0)
    off.advance_to(0.001)
    assert g1["rate"] == g2["rate"] == C
    alone = oracle.LinkNet(net)  # one transfer: its acknowledgements load only link 1
    h = alone.start(0, 1, 0.0)
    alone.advance_to(0.001)
    assert h["rate"] == C
    fat = oracle.LinkNet(dict(net, shared=np.array([1, 0]), bw=np.array([1000.0, 10.0])))
    k = fat.start(0, 1, 0.0)  # reverse route: FATPIPE link 1 of 10 B/s caps it at 9.7 / 0.05
    fat.advance_to(0.001)
    assert k["rate"] == pytest.approx(0.97 * 10.0 / 0.05)
    with pytest.raises(fu.FuError, match="bad arguments"):
        names = ["a", "b"]
        fu.Trace(np.array([0, 1, 2]), np.array([1, 0]), "pairwise", 10, net=dict(net, crosstraffic=2.0))
        del names


def test_link_model_argument_checks():
    d = load_json("tick_small_platform_ca_fwd.json")
    names, vals, rp, col = fixture_decl_csr(d)
    n = len(names)
    net = _random_net(n, 3, slow=True)
    bad = dict(net, route_off=net["route_off"][:-1])
    with pytest.raises(ValueError):
        fu.Trace(rp, col, "pairwise", 10, net=bad)
    bad = dict(net, route_links=np.full_like(net["route_links"], 99))
    with pytest.raises(fu.FuError, match="out of range"):
        fu.Trace(rp, col, "pairwise", 10, net=bad)
    bad = dict(net, bw=np.zeros_like(net["bw"]))
    with pytest.raises(fu.FuError, match="bandwidths"):
        fu.Trace(rp, col, "pairwise", 10, net=bad)
    with pytest.raises(ValueError, match="exclusive"):
        fu.Trace(rp, col, "pairwise", 10, net=net, route_s=np.zeros((n, n)))


@pytest.mark.gpu
def test_engine_runs_a_slow_platform(tmp_path):
    """A platform whose routes need more than one tick (LV08: 13.01 x 100 ms + 154 B / (0.97
    x 1 kB/s) = 1.46 s alone) is simulated instead of being rejected: every route crosses the
    one shared link, so concurrent transfers split its bandwidth (link model,
    fu_trace_build_links). The drop-in Engine's replay equals the oracle emulator with the
    same link model bit for bit, and converges."""
    import io

    from conftest import write_deployment_xml

    d = load_json("tick_small_platform_ca_fwd.json")
    hosts = [a[0] for a in d["actors"]]
    lines = ["<?xml version='1.0'?>", '<platform version="4.1">', '  <zone id="z" routing="Full">']
    for h in hosts:
        lines.append(f'    <host id="{h}" speed="1Gf"/>')
    lines.append('    <link id="slow" bandwidth="1kBps" latency="100ms"/>')
    for i, s_ in enumerate(hosts):
        for t in hosts[i + 1:]:
            lines += [f'    <route src="{s_}" dst="{t}">', '      <link_ctn id="slow"/>', "    </route>"]
    lines += ["  </zone>", "</platform>"]
    plat = tmp_path / "slow_platform.xml"
    plat.write_text("\n".join(lines) + "\n")
    dep = tmp_path / "actors.xml"
    write_deployment_xml(dep, d["actors"])
    p = fu.platform.load_platform(str(plat))
    T = p.route_time(hosts[0], hosts[1])
    assert 1.0 < T < 2.0
    net = p.link_net(hosts)  # one shared link: concurrent transfers split its 1 kB/s
    for mode, m in (("collectall", "ca"), ("pairwise", "pw")):
        e, res = fu.run_reference_main(mode, str(plat), str(dep), 1000.0, 10.0, order="fwd",
                                       out=io.StringIO())
        em = oracle.TickEmulator(d["actors"], m, net=net)
        em.run(1001, "fwd")
        want = dict(em.last_avg_items())
        for i, v in want.items():
            assert res["last_avg"][i] == v, (mode, i)
        # two-tick deliveries slow the mixing: 1e-7 at t = 1000 (1e-13 on the reference platform)
        assert np.max(np.abs(res["last_avg"] - 190 / 6)) / (190 / 6) < 1e-6

"""Platform / deployment loaders (the reference's input surface, CA:154-157)."""
import numpy as np
import pytest

from conftest import load_json, write_deployment_xml, write_platform_xml
from fu.platform import (declared_csr, load_deployment, load_platform, parse_bandwidth,
                         parse_time, symmetric_union_csr)


def test_units():
    assert parse_bandwidth("41.279125MBps") == pytest.approx(41.279125e6)
    assert parse_bandwidth("8Mbps") == pytest.approx(1e6)
    assert parse_bandwidth("1GiBps") == 1024.0 ** 3
    assert parse_time("59.904us") == pytest.approx(59.904e-6)
    assert parse_time("1.461517ms") == pytest.approx(1.461517e-3)
    assert parse_time("15us") == pytest.approx(15e-6)
    assert parse_time("2") == 2.0 and parse_time("1.5h") == 5400.0
    assert parse_time("1d") == 86400.0 and parse_time("2w") == 1209600.0
    with pytest.raises(ValueError):
        parse_time("3parsecs")


def test_small_platform_routes_fit_in_one_tick(tmp_path):
    """The tick model needs every route to transfer in < 1 s."""
    p = tmp_path / "plat.xml"
    write_platform_xml(p)
    plat = load_platform(str(p))
    assert len(plat.hosts) == 7 and len(plat.links) == 24
    d = load_json("tick_small_platform_ca_fwd.json")
    names = [a[0] for a in d["actors"]]
    pairs = {(names[i], names[j]) for i, row in enumerate(d["neighbors"]) for j in row}
    times = [plat.route_time(s, t) for (s, t) in pairs]
    assert max(times) < 1.0
    assert max(times) == pytest.approx(0.892, abs=2e-3)  # Fafard <-> Jacquelin
    # a route no message takes may be slower than a tick (Jacquelin <-> Boivin)
    assert plat.route_time("Jacquelin", "Boivin") > 1.0
    assert plat.route_time("Fafard", "Jacquelin") == pytest.approx(plat.route_time("Jacquelin", "Fafard"))


def test_deployment_parse_and_csr(tmp_path):
    d = load_json("tick_small_platform_ca_fwd.json")
    p = tmp_path / "actors.xml"
    write_deployment_xml(p, d["actors"])
    dep = load_deployment(str(p))
    names, values, nbrs = dep.peers()
    assert names == ["Fafard", "Ginette", "Boivin", "Jupiter", "Jacquelin", "Bourassa"]
    assert list(values) == [15.0, 10.0, 20.0, 60.0, 80.0, 5.0]
    rp, col = declared_csr(names, nbrs)
    assert rp[-1] == 14  # 14 declared directed edges
    urp, ucol = symmetric_union_csr(names, nbrs)
    assert urp[-1] == 20  # 10 undirected pairs
    deg = np.diff(urp)
    # final neighbour counts after dynamic addition
    assert list(deg) == [5, 5, 2, 2, 3, 3]


def test_deployment_errors(tmp_path):
    with pytest.raises(ValueError, match="not a deployed peer"):
        declared_csr(["a", "b"], [["c"], []])
    with pytest.raises(ValueError, match="itself"):
        declared_csr(["a", "b"], [["a"], []])
    names, values, nbrs = None, None, None
    p = tmp_path / "dup.xml"
    write_deployment_xml(p, [("a", "1.5", "b,b"), ("b", "2", "")])
    names, values, nbrs = load_deployment(str(p)).peers()
    assert nbrs == [["b"], []]  # dict keys collapse duplicates (CA:38-40)


def test_link_net_missing_route_raises_unless_allowed(tmp_path):
    """A neighbouring pair the platform does not route is an error by default (SimGrid's Full
    routing stops with "no route"), naming every such pair. allow_unrouted=True runs it with an
    empty route (delivery within one tick, the plain schedule, CA:76) and warns; the trace then
    equals the plain one when no route is slow."""
    import fu

    d = load_json("tick_small_platform_ca_fwd.json")
    hosts = [a[0] for a in d["actors"]]
    lines = ["<?xml version='1.0'?>", '<platform version="4.1">', '  <zone id="z" routing="Full">']
    lines += [f'    <host id="{h}" speed="1Gf"/>' for h in hosts]
    lines.append('    <link id="fast" bandwidth="1GBps" latency="1us"/>')
    lines += [f'    <route src="{hosts[0]}" dst="{hosts[1]}">', '      <link_ctn id="fast"/>', "    </route>"]
    lines += ["  </zone>", "</platform>"]
    pf = tmp_path / "partial.xml"
    pf.write_text("\n".join(lines) + "\n")
    plat = load_platform(str(pf))
    names = [a[0] for a in d["actors"]]
    nbrs = [a[2].split(",") if a[2] else [] for a in d["actors"]]
    rp, col = declared_csr(names, nbrs)
    with pytest.raises(KeyError, match="no route Fafard -> Boivin.*Bourassa -> Jacquelin"):
        plat.link_net(names)
    # only the pairs that exchange messages need a route: a routed subset passes
    routed = plat.link_net(names, pairs=[(0, 1), (1, 0)])
    assert routed["route_off"][-1] == 2
    with pytest.warns(UserWarning, match="Fafard -> Jupiter"):
        net = plat.link_net(names, allow_unrouted=True)
    n = len(names)
    assert net["route_off"][-1] == 2  # only the routed pair (both directions) holds a link
    plain = fu.Trace(rp, col, "collectall", 300, "fwd").arrays()
    linked = fu.Trace(rp, col, "collectall", 300, "fwd", net=net).arrays()
    for k in ("events", "tasks", "tick_task_off"):
        assert np.array_equal(plain[k], linked[k]), k
    assert n == 6


def test_engine_refuses_unrouted_neighbours(tmp_path):
    """The drop-in Engine builds the link model for every declared neighbour pair, so a
    platform missing one of their routes stops at run_until (before any GPU work) unless
    --fu-allow-unrouted is given."""
    import fu

    d = load_json("tick_small_platform_ca_fwd.json")
    hosts = [a[0] for a in d["actors"]]
    lines = ["<?xml version='1.0'?>", '<platform version="4.1">', '  <zone id="z" routing="Full">']
    lines += [f'    <host id="{h}" speed="1Gf"/>' for h in hosts]
    lines.append('    <link id="fast" bandwidth="1GBps" latency="1us"/>')
    lines += [f'    <route src="{hosts[0]}" dst="{hosts[1]}">', '      <link_ctn id="fast"/>', "    </route>"]
    lines += ["  </zone>", "</platform>"]
    pf = tmp_path / "partial.xml"
    pf.write_text("\n".join(lines) + "\n")
    act = tmp_path / "actors.xml"
    write_deployment_xml(act, d["actors"])
    e = fu.Engine([], out=False)
    e.load_platform(str(pf))
    e.register_actor("peer", fu.CollectAllPeer)
    e.load_deployment(str(act))
    with pytest.raises(KeyError, match="no route"):
        e.run_until(100)
    e2 = fu.Engine(["prog", "--fu-allow-unrouted", "--cfg=network/crosstraffic:1"], out=False)
    assert e2.allow_unrouted and e2.crosstraffic == 0.05
    assert fu.Engine([], out=False).crosstraffic == 0.0


def test_route_time_applies_the_tcp_window():
    """A lone transfer's rate is min(0.97 * min bandwidth, gamma / (2 * latency sum)) in the
    per-route model, as in the link model (fu_trace_build_links_ex, oracle LinkNet)."""
    from fu.platform import LV08_LATENCY_FACTOR, TCP_GAMMA, Platform

    p = Platform()
    p.links = {"l": (1e12, 0.5)}  # 1 TB/s, 0.5 s of latency: the window (4 MiB / 1 s) binds
    p.routes = {("a", "b"): ["l"]}
    big = 1e9
    assert p.route_time("a", "b", size_bytes=big) == pytest.approx(LV08_LATENCY_FACTOR * 0.5 + big / TCP_GAMMA)
    p.links = {"l": (1e3, 1e-6)}  # a slow link: the bandwidth binds
    assert p.route_time("a", "b", size_bytes=154.0) == pytest.approx(LV08_LATENCY_FACTOR * 1e-6 + 154.0 / 970.0)

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


def test_link_net_missing_route_is_one_tick(tmp_path):
    """A platform that routes only some host pairs still runs: a neighbouring pair without a
    route gets an empty route (delivery within one tick, the plain schedule, CA:76), as the
    per-route model treated it; the trace equals the plain one when no route is slow."""
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
    net = plat.link_net(names)
    n = len(names)
    assert net["route_off"][-1] == 2  # only the routed pair (both directions) holds a link
    plain = fu.Trace(rp, col, "collectall", 300, "fwd").arrays()
    linked = fu.Trace(rp, col, "collectall", 300, "fwd", net=net).arrays()
    for k in ("events", "tasks", "tick_task_off"):
        assert np.array_equal(plain[k], linked[k]), k
    assert n == 6

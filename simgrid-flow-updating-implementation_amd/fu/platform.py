"""SimGrid XML inputs: platform files (platforms/*.xml) and deployment files (actors.xml).

The reference passes both files to SimGrid unchanged (flowupdating-collectall.py:154,
CA:157). Here they are parsed into:
* `Platform`: hosts, links and routes. It is used to validate host names, and to check the
  timing assumption the tick model relies on: every route a message takes must transfer in
  under one tick (Peer.TICK_INTERVAL = 1.0, CA:23).
* `Deployment`: actors in file order with their string arguments. `peer` actors carry
  (initial value, "n1,n2,...") (ACT:4-27, parsed by Peer.__init__ CA:26-31).
"""
from __future__ import annotations

import re
import warnings
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

# SimGrid's time units (a bare number is seconds)
_UNITS_T = {"": 1.0, "s": 1.0, "ms": 1e-3, "us": 1e-6, "ns": 1e-9, "ps": 1e-12,
            "m": 60.0, "h": 3600.0, "d": 86400.0, "w": 604800.0}

# LV08 network model defaults of SimGrid (latency factor, bandwidth factor).
LV08_LATENCY_FACTOR = 13.01
LV08_WEIGHT_S = 20537.0     # sharing penalty: latency sum + weight_S / bandwidth per route link
TCP_GAMMA = 4194304.0       # TCP window: a transfer's rate <= gamma / (2 * latency sum)
LV08_BANDWIDTH_FACTOR = 0.97
CROSSTRAFFIC = 0.05          # network/crosstraffic: a transfer's load on its reverse route's links


def parse_bandwidth(s: str) -> float:
    """SimGrid bandwidth string -> bytes per second. 'MBps' = 1e6 B/s, 'Mbps' = 1e6 bit/s."""
    m = re.fullmatch(r"\s*([0-9.eE+-]+)\s*([A-Za-z]*)\s*", s)
    if not m:
        raise ValueError(f"bad bandwidth {s!r}")
    val, unit = float(m.group(1)), m.group(2)
    if unit == "":
        return val
    prefix = {"": 1.0, "k": 1e3, "M": 1e6, "G": 1e9, "T": 1e12,
              "Ki": 1024.0, "Mi": 1024.0 ** 2, "Gi": 1024.0 ** 3, "Ti": 1024.0 ** 4}
    for p, mul in sorted(prefix.items(), key=lambda kv: -len(kv[0])):
        if unit.startswith(p) and unit[len(p):] in ("Bps", "bps"):
            base = 1.0 if unit[len(p):] == "Bps" else 0.125
            return val * mul * base
    raise ValueError(f"bad bandwidth unit {s!r}")


def parse_time(s: str) -> float:
    m = re.fullmatch(r"\s*([0-9.eE+-]+)\s*([A-Za-z]*)\s*", s)
    if not m or m.group(2) not in _UNITS_T:
        raise ValueError(f"bad time {s!r}")
    return float(m.group(1)) * _UNITS_T[m.group(2)]


@dataclass
class Platform:
    hosts: dict = field(default_factory=dict)   # id -> speed string
    links: dict = field(default_factory=dict)   # id -> (bandwidth B/s, latency s)
    routes: dict = field(default_factory=dict)  # (src, dst) -> [link ids]
    routing: str = "Full"
    fatpipe: set = field(default_factory=set)   # ids of sharing_policy="FATPIPE" links

    def add_host(self, name: str, speed="0f"):
        """Mirror of e.netzone_root.add_host (CA:159): hosts without routes, e.g. the observer."""
        self.hosts[name] = speed

    def route_time(self, src: str, dst: str, size_bytes: float = 154.0) -> float:
        """LV08 transfer time of a lone transfer: 13.01 * sum(latency) + size / rate, where
        rate = min(0.97 * min bandwidth, TCP window gamma / (2 * sum(latency))): the same
        bound the link model (link_net, fu_trace_build_links_ex) puts on every transfer, so a
        lone transfer takes the same time in both models."""
        links = self.routes.get((src, dst))
        if links is None:
            raise KeyError(f"no route {src} -> {dst}")
        if not links:
            return 0.0
        lat = sum(self.links[k][1] for k in links)
        rate = min(LV08_BANDWIDTH_FACTOR * self.links[k][0] for k in links)
        if lat > 0.0:
            rate = min(rate, TCP_GAMMA / (2.0 * lat))
        return LV08_LATENCY_FACTOR * lat + size_bytes / rate

    def link_net(self, hosts, size_bytes: float = 154.0, pairs=None, allow_unrouted: bool = False,
                 crosstraffic: float = 0.0) -> dict:
        """The link model of fu_trace_build_links for the actors on `hosts` (in actor order):
        every link (bandwidth, latency, shared unless FATPIPE) and the route of every host
        pair (empty for a host to itself). Concurrent transfers share the links' bandwidth
        (max-min fair, each share weighted by 1 / LV08's sharing penalty, rates capped by the
        TCP window); alone, a transfer takes route_time. pairs: the (i, j) actor pairs that
        exchange messages (None = all): only they need a route; the others stay empty.
        A needed pair the platform does not route raises KeyError listing every such pair, as
        SimGrid's Full routing stops on a missing route. allow_unrouted=True gives those pairs
        an empty route instead (delivery within one tick, the plain schedule of CA:76) and
        warns with the list. crosstraffic: SimGrid's network/crosstraffic factor (each
        transfer also loads the links of its reverse route with that share of its rate; 0.05
        in SimGrid, 0 = off, the default here: parity-unpinned, fu.h)."""
        ids = sorted(self.links)
        at = {k: q for q, k in enumerate(ids)}
        n = len(hosts)
        need = None if pairs is None else {(int(i), int(j)) for i, j in pairs}
        off, lst, missing = [0], [], []
        for i, a in enumerate(hosts):
            for j, b in enumerate(hosts):
                if a != b and (need is None or (i, j) in need):
                    if (a, b) in self.routes:
                        lst.extend(at[k] for k in self.routes[(a, b)])
                    else:
                        missing.append((a, b))
                off.append(len(lst))
        if missing:
            desc = ", ".join(f"{a} -> {b}" for a, b in missing)
            if not allow_unrouted:
                raise KeyError(f"no route {desc} in the platform (pass allow_unrouted=True, or "
                               "--fu-allow-unrouted to the Engine, to deliver them within one tick)")
            warnings.warn(f"unrouted host pairs get one-tick delivery: {desc}", stacklevel=2)
        return {"bw": np.array([self.links[k][0] for k in ids], dtype=np.float64),
                "lat": np.array([self.links[k][1] for k in ids], dtype=np.float64),
                "shared": np.array([0 if k in self.fatpipe else 1 for k in ids], dtype=np.int32),
                "route_off": np.array(off, dtype=np.int64), "route_links": np.array(lst, dtype=np.int32),
                "bytes": float(size_bytes), "lat_factor": LV08_LATENCY_FACTOR,
                "bw_factor": LV08_BANDWIDTH_FACTOR, "weight_S": LV08_WEIGHT_S, "tcp_gamma": TCP_GAMMA,
                "crosstraffic": float(crosstraffic), "n": n}


def load_platform(path: str) -> Platform:
    root = ET.parse(path).getroot()
    p = Platform()
    zones = list(root.iter("zone")) + list(root.iter("AS"))
    if zones:
        p.routing = zones[0].get("routing", "Full")
    for h in root.iter("host"):
        p.hosts[h.get("id")] = h.get("speed", "0f")
    for ln in root.iter("link"):
        p.links[ln.get("id")] = (parse_bandwidth(ln.get("bandwidth", "0")),
                                 parse_time(ln.get("latency", "0")))
        if ln.get("sharing_policy", "SHARED").upper() == "FATPIPE":
            p.fatpipe.add(ln.get("id"))
    for r in root.iter("route"):
        src, dst = r.get("src"), r.get("dst")
        ids = [c.get("id") for c in r.findall("link_ctn")]
        p.routes[(src, dst)] = ids
        if r.get("symmetrical", "YES").upper() in ("YES", "TRUE", "1") and (dst, src) not in p.routes:
            p.routes[(dst, src)] = list(reversed(ids))
    for (s, d), ids in p.routes.items():
        for k in ids:
            if k not in p.links:
                raise ValueError(f"{path}: route {s}->{d} uses unknown link {k!r}")
    return p


@dataclass
class ActorSpec:
    host: str
    function: str
    args: list


@dataclass
class Deployment:
    actors: list  # [ActorSpec] in file order

    def peers(self, function: str = "peer"):
        """(names, values, neighbour-name lists) of the `function` actors, in file order.

        value = float(arg0) (CA:28, Python's correctly rounded parse);
        neighbours = arg1.split(',') if arg1 else [] (CA:29-31), duplicates collapse like
        dict keys (CA:38-40), first occurrence kept."""
        names, values, nbrs = [], [], []
        for a in self.actors:
            if a.function != function:
                continue
            names.append(a.host)
            values.append(float(a.args[0]))
            raw = a.args[1] if len(a.args) > 1 else ""
            lst = raw.split(",") if len(raw) else []
            seen = {}
            for x in lst:
                seen.setdefault(x, None)
            nbrs.append(list(seen))
        return names, np.array(values, dtype=np.float64), nbrs


def load_deployment(path: str) -> Deployment:
    root = ET.parse(path).getroot()
    acts = []
    for a in root.iter("actor"):
        fn = a.get("function")
        args = [x.get("value") for x in a.findall("argument")]
        acts.append(ActorSpec(a.get("host"), fn, args))
    return Deployment(acts)


def declared_csr(names, nbrs):
    """Declared neighbour lists -> (rowptr int64, col int32) in declared order."""
    idx = {nm: i for i, nm in enumerate(names)}
    if len(idx) != len(names):
        raise ValueError("two peers are deployed on the same host")
    rowptr = [0]
    col = []
    for i, lst in enumerate(nbrs):
        for x in lst:
            if x not in idx:
                raise ValueError(f"{names[i]}: neighbour {x!r} is not a deployed peer "
                                 "(its messages would never be received)")
            if idx[x] == i:
                raise ValueError(f"{names[i]} lists itself as a neighbour")
            col.append(idx[x])
        rowptr.append(len(col))
    return np.array(rowptr, dtype=np.int64), np.array(col, dtype=np.int32)


def symmetric_union_csr(names, nbrs):
    """Union graph for synchronous rounds: row = declared neighbours, then the peers that
    declare this node but are not declared by it, in deployment order."""
    rp, col = declared_csr(names, nbrs)
    n = len(names)
    rows = [list(col[rp[i]:rp[i + 1]]) for i in range(n)]
    have = [set(r) for r in rows]
    for i in range(n):
        for j in list(rows[i]):
            if i not in have[j]:
                rows[j].append(i)
                have[j].add(i)
    rowptr = np.zeros(n + 1, dtype=np.int64)
    for i in range(n):
        rowptr[i + 1] = rowptr[i] + len(rows[i])
    return rowptr, np.array([c for r in rows for c in r], dtype=np.int32)

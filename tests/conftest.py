import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "simgrid-flow-updating-implementation_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs via gpurun)")


def load_manifest():
    with open(os.path.join(GOLDEN, "MANIFEST.json")) as f:
        return json.load(f)


def ca_sync_fixtures():
    return sorted(load_manifest()["ca_sync"].items())


def tick_fixtures():
    return sorted(load_manifest()["tick"].items())


def load_npz(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def write_platform_xml(path):
    """Rebuild the reference platform (hosts, links, routes) from the JSON summary fixture,
    in this repo's own layout."""
    s = load_json("small_platform_summary.json")
    lines = ["<?xml version='1.0'?>", '<platform version="4.1">',
             f'  <zone id="z" routing="{s["routing"]}">']
    for hid, speed in s["hosts"]:
        lines.append(f'    <host id="{hid}" speed="{speed}"/>')
    for lid, bw, lat, pol in s["links"]:
        extra = f' sharing_policy="{pol}"' if pol else ""
        lines.append(f'    <link id="{lid}" bandwidth="{bw}" latency="{lat}"{extra}/>')
    for src, dst, ids in s["routes"]:
        lines.append(f'    <route src="{src}" dst="{dst}">')
        lines.extend(f'      <link_ctn id="{k}"/>' for k in ids)
        lines.append("    </route>")
    lines += ["  </zone>", "</platform>"]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def write_deployment_xml(path, actors):
    lines = ["<?xml version='1.0'?>", '<platform version="4.1">']
    for host, val, neigh in actors:
        lines.append(f'  <actor host="{host}" function="peer">')
        lines.append(f'    <argument value="{val}"/>')
        lines.append(f'    <argument value="{neigh}"/>')
        lines.append("  </actor>")
    lines.append("</platform>")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def trace_events_as_log(arr):
    """Trace arrays -> [(tick, node, kind, other)] like the fixtures' event log.
    kind 0 = receive (other = sender node), 1 = fire (other = neighbour node or -1)."""
    tto, tasks, ev = arr["tick_task_off"], arr["tasks"], arr["events"]
    rp, col = arr["rowptr"], arr["col"]
    out = []
    t = 0
    for q in range(len(tasks)):
        while tto[t + 1] <= q:
            t += 1
        node, b, e = (int(x) for x in tasks[q])
        for p in range(b, e):
            k, s = int(ev[p, 0]), int(ev[p, 1])
            if k == 0:
                out.append([t, node, 0, int(col[rp[node] + s])])
            elif k == 1:
                out.append([t, node, 1, -1])
            else:
                out.append([t, node, 1, int(col[rp[node] + s])])
    return out


def fixture_decl_csr(d):
    from fu.platform import declared_csr

    names = [a[0] for a in d["actors"]]
    nbrs = [a[2].split(",") if a[2] else [] for a in d["actors"]]
    vals = np.array([float(a[1]) for a in d["actors"]])
    rp, col = declared_csr(names, nbrs)
    return names, vals, rp, col

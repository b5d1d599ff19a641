"""Command line: the two reference scripts as one CLI.

    python -m fu collectall [--platform P] [--deployment D] [--until 1000] [--interval 10]
    python -m fu pairwise   ...
    python -m fu collectall --sync --rounds 200         # synchronous rounds (hot path)
    python -m fu bench-graph er:n=1000000,m=4000000 --rounds 1000

Defaults mirror flowupdating-collectall.py:154,157 (./platforms/small_platform.xml,
./actors.xml, watcher 1000.0 / 10.0 at CA:162).
"""
from __future__ import annotations

import argparse
import sys
import time

from .engine import CollectAll
from .graph import Graph, component_means, uniform_values
from .sim import CollectAllPeer, Engine, run_reference_main


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m fu")
    ap.add_argument("mode", choices=["collectall", "pairwise", "bench-graph"])
    ap.add_argument("spec", nargs="?", help="graph spec for bench-graph (er:/rr:/rmat:/rgg:)")
    ap.add_argument("--platform", default="./platforms/small_platform.xml")
    ap.add_argument("--deployment", default="./actors.xml")
    ap.add_argument("--until", type=float, default=1000.0)
    ap.add_argument("--interval", type=float, default=10.0)
    ap.add_argument("--order", default="fwd", help="intra-tick actor order: fwd|rev|rand:<seed>")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--sync", action="store_true", help="generation-synchronous rounds")
    ap.add_argument("--rounds", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--kernel", default="auto")
    a = ap.parse_args(argv)
    if a.mode == "bench-graph":
        g = Graph.from_spec(a.spec, seed=a.seed)
        v = uniform_values(g.n, seed=0)
        eng = CollectAll(g, v, device=a.device, kernel=a.kernel)
        t0 = time.perf_counter()
        ms = eng.run_timed(a.rounds)
        wall = time.perf_counter() - t0
        tgt, _ = component_means(g.rowptr, g.col, v)
        eng.set_targets(tgt)
        print(f"graph n={g.n} E={g.E} max_deg={g.max_deg} rounds={a.rounds} "
              f"device_ms={ms:.3f} wall_s={wall:.3f} edge_updates/s={g.E * a.rounds / (ms / 1e3):.4e} "
              f"max_err={eng.max_err():.3e}")
        return 0
    if a.sync:
        e = Engine([], device=a.device, sync=True)
        e.load_platform(a.platform)
        e.register_actor("peer", CollectAllPeer)
        e.load_deployment(a.deployment)
        e.add_watcher(a.rounds, a.interval)
        e.run_until(a.rounds)
        return 0
    run_reference_main(a.mode, a.platform, a.deployment, a.until, a.interval, a.order, a.device)
    return 0


if __name__ == "__main__":
    sys.exit(main())

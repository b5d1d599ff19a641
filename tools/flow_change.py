"""How much of each flow changes from f_{r-2} to f_r, round by round (CPU, C oracle).

The engine stores a flow as three pieces (csrc/fu_engine.hip, f_idx): the high 32-bit word,
the middle and the low 16 bits of the low word, each rewritten only when it changes. This
tool counts, per round, the directed edges whose f_r equals f_{r-2} bit for bit, whose high
word is unchanged, and whose change stays inside the low 16 bits (the edges a round then
writes 2 bytes for). Follows CA:117 through the C oracle (oracle/fu_oracle.c round_ca).

    python tools/flow_change.py --n 1000000 --m 4000000 --rounds 1000 --out stats.json
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "simgrid-flow-updating-implementation_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))

import fu  # noqa: E402
from oracle import coracle  # noqa: E402


def flow_change(n, m, rounds, every=25, graph_seed=1, value_seed=0, nthreads=8):
    g = fu.Graph.erdos_renyi(n, m, seed=graph_seed)
    rp, col, rev = g.rowptr, g.col, g.rev
    v = fu.uniform_values(n, seed=value_seed)
    a, f = coracle.ca_sync(rp, col, rev, v, 1, nthreads=nthreads)  # after round 0: f_0
    prev = [f.copy(), f.copy()]  # prev[r % 2] = f_{r-2} when round r runs
    E = len(f)
    out = []
    for r in range(1, rounds):
        coracle.ca_rounds(rp, col, rev, v, 1, a, f, nthreads=nthreads)
        if r >= 2 and (r % every == 0 or r == rounds - 1):
            fb, ob = f.view(np.uint64), prev[r % 2].view(np.uint64)
            x = fb ^ ob
            out.append({"round": r,
                         "same": float(np.count_nonzero(x == 0) / E),
                         "high_word_same": float(np.count_nonzero((x >> np.uint64(32)) == 0) / E),
                         "change_in_low16": float(np.count_nonzero(x < np.uint64(1 << 16)) / E)})
        prev[r % 2] = f.copy()
    return {"graph": f"er:n={n},m={m}", "graph_seed": graph_seed, "value_seed": value_seed,
            "E_directed": int(E), "rounds": rounds, "per_round": out}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--m", type=int, default=4_000_000)
    ap.add_argument("--rounds", type=int, default=1000)
    ap.add_argument("--every", type=int, default=25)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    res = flow_change(a.n, a.m, a.rounds, a.every, nthreads=a.threads)
    for row in res["per_round"]:
        print(row["round"], "same %.4f  high word same %.4f  change in low 16 bits %.4f"
              % (row["same"], row["high_word_same"], row["change_in_low16"]))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()

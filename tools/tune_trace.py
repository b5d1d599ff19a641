"""Autotuner trace on ER-1M: which candidate wins each pass, at which packing width, and
which kernel the timed rounds after fu_reset use (bench.py's default sequence)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "simgrid-flow-updating-implementation_amd"))
import fu  # noqa: E402

WARMUP = int(os.environ.get("WARMUP", "400"))
g = fu.Graph.erdos_renyi(1_000_000, 4_000_000, seed=1)
v = fu.uniform_values(g.n, seed=0)
REPS = int(os.environ.get("REPS", "1"))


def show(tag):
    global eng
    i = eng.info()
    print(tag, "rounds", eng.rounds_done, "kernel", i["kernel"], i["tile"], "passes", i["tune_passes"],
          "us", i["tune_us_per_round"], "by_width", i["tune_winner_by_width"], "widths", eng.pack_widths(),
          flush=True)


for rep in range(REPS):
  print("== rep", rep, flush=True)
  eng = fu.CollectAll(g, v, device=0, kernel="auto")
  eng.tune()
  show("tune")
  for w0 in range(0, WARMUP, 64):
    eng.run(min(64, WARMUP - w0))
    eng.synchronize()
    show("warm")
  eng.reset()
  show("reset")
  for k in range(10):
    eng.run(100)
    eng.synchronize()
    show("timed")
  eng.close()

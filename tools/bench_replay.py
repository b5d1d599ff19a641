#!/usr/bin/env python3
"""Pairwise (and collect-all) tick-replay throughput: RR n=65,536 d=8 (BASELINE config 3).
Reports trace-build time (host C++), GPU replay time (HIP events), events/s, flow updates/s
(one flow update per FIRE_PW; k per FIRE_CA), and the C oracle's single-thread replay."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "simgrid-flow-updating-implementation_amd"), os.path.join(ROOT, "oracle")]
import coracle  # noqa: E402
import fu  # noqa: E402

ticks = int(os.environ.get("TICKS", "400"))
for mode in ("pairwise", "collectall"):
    g = fu.Graph.random_regular(65536, 8, seed=1)
    v = fu.uniform_values(g.n, seed=0)
    t0 = time.perf_counter()
    tr = fu.Trace(g.rowptr, g.col, mode, ticks, "rand:3")
    t_build = time.perf_counter() - t0
    a = tr.arrays()
    ev = a["events"]
    upd = int(np.sum(ev[:, 0] == 2) + np.sum(ev[ev[:, 0] == 1, 1]))
    res = {}
    for pers in (False, True, "noreg"):
        rep = fu.Replay(tr, v, persistent=bool(pers), registers=pers != "noreg")
        ms = rep.run_timed(ticks)
        res[pers] = (ms, rep.state())
        rep.close()
    ms, (last, flows, est) = res[False]
    ms_p, (last_p, flows_p, _) = res[True]
    ms_n, (last_n, flows_n, _) = res["noreg"]
    t0 = time.perf_counter()
    l_ref, f_ref, e_ref, _ = coracle.replay(a["rowptr"], v, a["tick_task_off"], a["tasks"], a["events"],
                                            a["out_ids"], tr.n_msgs)
    t_cpu = time.perf_counter() - t0
    print(json.dumps({"mode": mode, "ticks": ticks, "events": tr.n_events, "tasks": tr.n_tasks,
                      "flow_updates": upd, "trace_build_s": t_build, "gpu_ms": ms,
                      "gpu_us_per_tick": ms * 1e3 / ticks,
                      "gpu_flow_updates_per_s": upd / (ms / 1e3),
                      "cpu_oracle_1thread_s": t_cpu, "cpu_flow_updates_per_s": upd / t_cpu,
                      "gpu_persistent_ms": ms_p, "gpu_persistent_us_per_tick": ms_p * 1e3 / ticks,
                      "gpu_persistent_flow_updates_per_s": upd / (ms_p / 1e3),
                      "bitwise_equal": bool(np.array_equal(last, l_ref) and np.array_equal(flows, f_ref)),
                      "persistent_bitwise_equal": bool(np.array_equal(last_p, l_ref) and np.array_equal(flows_p, f_ref)),
                      "gpu_persistent_noreg_us_per_tick": ms_n * 1e3 / ticks,
                      "persistent_noreg_bitwise_equal": bool(np.array_equal(last_n, l_ref) and np.array_equal(flows_n, f_ref))}),
          flush=True)

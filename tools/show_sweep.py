import json, sys
for l in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sweep.log"):
    if not l.startswith("{"):
        continue
    d = json.loads(l)
    print(d["spec"], "E=", d["E"])
    for k, v in d.items():
        if isinstance(v, dict):
            print("   %-20s %8.1f us  %7.0f GB/s  %.3g eu/s" % (k, v["us_per_round_med"], v["alg_GBs"], v["edge_updates_per_s"]))

"""Pass time of the 9-mer sweep for different lane-group compositions (tool): how much
does a device group of n lanes cost, n = 1..5, and mixes (the CV shares of an 8-GPU job
hold groups of 1-5 lanes)?  Prints one JSON line per composition."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from kmerpapa_amd import engine  # noqa: E402

comps = [[5], [1], [2], [3], [4], [5, 1], [4, 4], [3, 3, 2], [5, 3]]
if len(sys.argv) > 1:  # e.g. "5 3,2": compositions as comma lists
    comps = [[int(x) for x in a.split(",")] for a in sys.argv[1:]]
prep = bench.prepare("NNNNMNNNN")
plan = engine.get_plan(0, "NNNNMNNNN")
plan.set_counts(prep["Mk"], prep["Uk"])
plan.reserve(max(8, max(sum(c) for c in comps)))
g = prep["groups"]
plan.run([g[0]])  # warm
for comp in comps:
    # n > 5 lanes: extra penalties 8, 9, ... (the 11-mer grid has 7)
    groups = [(g[i][0], g[i][1], g[i][2], (list(g[i][3]) + [8.0 + j for j in range(8)])[:n]) for i, n in enumerate(comp)]
    t0 = time.perf_counter()
    plan.run(groups)
    dt = time.perf_counter() - t0
    st = plan.stats()
    print(json.dumps({"groups": comp, "lanes": sum(comp), "pass_s": round(dt, 4), "dp_ms": round(st["dp_ms"], 2),
                      "ms_per_lane": round(st["dp_ms"] / sum(comp), 2)}), flush=True)

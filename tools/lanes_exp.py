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
mixed = set()
if len(sys.argv) > 1:  # e.g. "5 3,2 m2,3": compositions as comma lists; "m" = groups of ONE
    # fold with different alphas (the library cuts them together into mixed device groups)
    comps = []
    for a in sys.argv[1:]:
        if a.startswith("m"):
            mixed.add(len(comps))
            a = a[1:]
        comps.append([int(x) for x in a.split(",")])
prep = bench.prepare("NNNNMNNNN")
plan = engine.get_plan(0, "NNNNMNNNN")
plan.set_counts(prep["Mk"], prep["Uk"])
plan.reserve(max(8, max(sum(c) for c in comps)))
g = prep["groups"]
plan.run([g[0]])  # warm
same_fold = [x for x in g if x[0] == g[0][0]]  # one group per alpha
for ci, comp in enumerate(comps):
    # n > 5 lanes: extra penalties 8, 9, ... (the 11-mer grid has 7)
    src = same_fold if ci in mixed else g
    groups = [(src[i][0], src[i][1], src[i][2], (list(src[i][3]) + [8.0 + j for j in range(8)])[:n])
              for i, n in enumerate(comp)]
    t0 = time.perf_counter()
    plan.run(groups)
    dt = time.perf_counter() - t0
    st = plan.stats()
    rec = {"groups": comp, "mixed": ci in mixed, "lanes": sum(comp), "pass_s": round(dt, 4), "dp_ms": round(st["dp_ms"], 2),
           "ms_per_lane": round(st["dp_ms"] / sum(comp), 2)}
    if os.environ.get("KP_LAUNCH_TIMES") == "1":  # per-launch device times (lane classes, high levels ascending)
        rec["launch_ms"] = [round(float(x), 3) for x in plan.launch_ms()]
    print(json.dumps(rec), flush=True)

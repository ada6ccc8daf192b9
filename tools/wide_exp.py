"""Pass time of wider lane compositions (tool; 9-mer, one GPU): device groups of the
listed widths in one pass, best of two each, lanes cut from the (alpha, fold) groups of
the bench's 5x5x5 grid.  Which passes a 16-lane share (one 8-GPU rank) should run."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from kmerpapa_amd import engine  # noqa: E402

prep = bench.prepare("NNNNMNNNN")
plan = engine.get_plan(0, "NNNNMNNNN")
plan.set_counts(prep["Mk"], prep["Uk"])
comps = [[5], [4], [3], [2], [1], [3, 3], [2, 2, 2], [4, 4], [5, 3], [4, 4, 0], [3, 3, 2], [2, 2, 2, 2]]
need = max(sum(c) for c in comps)
try:
    plan.reserve(need)
except engine.KPError as e:
    print(json.dumps({"reserve": need, "error": str(e)}), flush=True)
    need = 7
    plan.reserve(need)
src = prep["groups"]


def best(groups):
    ms = []
    for _ in range(2):
        plan.run(groups)
        ms.append(plan.stats()["dp_ms"])
    return round(min(ms), 2)


plan.run([src[0]])  # warm
for comp in comps:
    comp = [n for n in comp if n]
    if sum(comp) > need:
        continue
    groups = [(src[i][0], src[i][1], src[i][2], list(src[i][3][:n])) for i, n in enumerate(comp)]
    ms = best(groups)
    print(json.dumps({"groups": comp, "lanes": sum(comp), "dp_ms": ms, "ms_per_lane": round(ms / sum(comp), 2)}),
          flush=True)

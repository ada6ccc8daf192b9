"""One warm 9-mer pass, then one pass per composition given on the command line (tool for
PMC runs: rocprofv3 --pmc ... -- python3 tools/pass_once.py 1 5).  Each argument is a
comma list of lane counts (one group per entry)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from kmerpapa_amd import engine  # noqa: E402

comps = [[int(x) for x in a.split(",")] for a in sys.argv[1:]] or [[1], [5]]
prep = bench.prepare("NNNNMNNNN")
plan = engine.get_plan(0, "NNNNMNNNN")
plan.reserve(max(sum(c) for c in comps))
plan.set_counts(prep["Mk"], prep["Uk"])
g = prep["groups"]
for comp in comps:
    groups = [(g[i][0], g[i][1], g[i][2], g[i][3][:n]) for i, n in enumerate(comp)]
    plan.run(groups)
    print(comp, round(plan.stats()["dp_ms"], 2), flush=True)

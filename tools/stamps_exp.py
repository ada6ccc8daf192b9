"""Per-phase shader-clock stamps (-DKP_STAMPS build) of one 9-mer pass for 1- and 5-lane
groups (tool).  Run with KMERPAPA_LIB=kmerpapa_amd/libkmerpapa_hip_stamps.so; the library
prints one KP_STAMPS line per pass on stderr."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from kmerpapa_amd import engine  # noqa: E402

prep = bench.prepare("NNNNMNNNN")
plan = engine.get_plan(0, "NNNNMNNNN")
plan.set_counts(prep["Mk"], prep["Uk"])
plan.reserve(5)
g = prep["groups"]
for comp in ([5], [1], [5], [1]):
    groups = [(g[i][0], g[i][1], g[i][2], g[i][3][:n]) for i, n in enumerate(comp)]
    print("pass", comp, file=sys.stderr, flush=True)
    plan.run(groups)
    print("dp_ms", plan.stats()["dp_ms"], file=sys.stderr, flush=True)

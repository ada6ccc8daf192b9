"""Per-level shader-clock stamps of one 5-lane 9-mer pass under phase ablations (tool).
Run with KMERPAPA_LIB pointing at a -DKP_ABLATION -DKP_STAMPS build; argv = KP_DEBUG_SKIP
values.  The library prints one KP_STAMPS line per pass on stderr."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from kmerpapa_amd import engine  # noqa: E402

prep = bench.prepare("NNNNMNNNN")
plan = engine.get_plan(0, "NNNNMNNNN")
plan.set_counts(prep["Mk"], prep["Uk"])
plan.reserve(5)
g = prep["groups"][0]
for skip in sys.argv[1:] or ["0"]:
    os.environ["KP_DEBUG_SKIP"] = skip
    print("skip", skip, file=sys.stderr, flush=True)
    try:
        plan.run([g])
    except engine.KPError as e:
        if e.code != -4:
            raise
    print("dp_ms", plan.stats()["dp_ms"], file=sys.stderr, flush=True)

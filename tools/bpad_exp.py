"""Pass time by lane layout (tool; 9-mer, one GPU): a 5-lane pass and 6-lane passes packed
[5, 1], [1, 5], [4, 2], [3, 3], best of three each, under the KP_BPAD_ALIGN of the
environment (the row length of one block lane, in floats, rounded up to that multiple)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from kmerpapa_amd import engine  # noqa: E402

prep = bench.prepare("NNNNMNNNN")
plan = engine.get_plan(0, "NNNNMNNNN")
plan.set_counts(prep["Mk"], prep["Uk"])
plan.reserve(6)
g = {(x[1], x[0]): x for x in prep["groups"]}  # (alpha, fold) -> group


def cut(grp, n):
    return (grp[0], grp[1], grp[2], list(grp[3][:n]))


def best(groups):
    ms = []
    for _ in range(3):
        plan.run(groups)
        ms.append(plan.stats()["dp_ms"])
    return round(min(ms), 2)


a, b = g[(0.5, 3)], g[(1.0, 4)]
plan.run([a])  # warm
out = {"bpad_align": os.environ.get("KP_BPAD_ALIGN", "16"), "block_pad": plan.info["block_pad"]}
for name, gs in [("5", [a]), ("5+1", [a, cut(b, 1)]), ("1+5", [cut(b, 1), a]), ("4+2", [cut(a, 4), cut(b, 2)]),
                 ("2+4", [cut(b, 2), cut(a, 4)]), ("3+3", [cut(a, 3), cut(b, 3)])]:
    out[name] = best(gs)
print(json.dumps(out), flush=True)

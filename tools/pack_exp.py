"""Pass time of a 5-lane (alpha, fold) group packed with one lane of another group in one
pass, by the folds and alphas of the two (tool; 9-mer, one GPU).  Prints one JSON line per
case: the packed pass and the two groups as separate passes, best of three each."""
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


def best(groups):
    ms = []
    for _ in range(3):
        plan.run(groups)
        ms.append(plan.stats()["dp_ms"])
    return round(min(ms), 2)


plan.run([g[(0.5, 1)]])  # warm
cases = [((0.5, 3), (1.0, 4), 0), ((0.5, 4), (0.5, 4), 0), ((2.0, 0), (10.0, 4), 1)]
for (a5, f5), (a1, f1), j in cases:
    five = g[(a5, f5)]
    one = g[(a1, f1)]
    one = (one[0], one[1], one[2], [one[3][j]])
    packed = best([five, one])
    packed_rev = best([one, five])
    sep = (best([five]), best([one]))
    print(json.dumps({"five": [a5, f5], "one": [a1, f1, one[3][0]], "packed_ms": packed, "packed_one_first_ms": packed_rev,
                      "separate_ms": sep, "saved_ms": round(sum(sep) - packed, 2)}), flush=True)

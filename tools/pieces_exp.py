"""Pass time of every fold piece of one fold of a grid's CV plan (tool): the passes
engine.plan_passes cuts the fold's lanes into (5-lane pieces, some spanning two alphas =
mixed device groups, and the remainder), each run twice on one GPU; prints one JSON line
per pass with its lane composition and the better of the two kernel times.
usage: python tools/pieces_exp.py [CONFIG] [FOLD]   (CONFIG = bench.py config, default 11mer)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from kmerpapa_amd import engine  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "11mer"]
fold = int(sys.argv[2]) if len(sys.argv) > 2 else 0
prep = bench.prepare(cfg["gen_pat"], alphas=cfg["alphas"], penalties=cfg["penalties"], nfolds=cfg["nfolds"])
plan = engine.get_plan(0, cfg["gen_pat"])
plan.set_counts(prep["Mk"], prep["Uk"])
width = plan.info["lanes_per_workgroup"]
passes, _ = engine.plan_passes([g for g in prep["groups"] if g[0] == fold], width, width)
plan.reserve(width)
plan.run(passes[0])  # warm
tot = 0.0
for pas in passes:
    ms = []
    for _ in range(2):
        plan.run(pas)
        ms.append(plan.stats()["dp_ms"])
    tot += min(ms)
    print(json.dumps({"lanes": [len(g[3]) for g in pas], "alphas": [g[1] for g in pas], "mixed": len(pas) > 1,
                      "dp_ms": round(min(ms), 2)}), flush=True)
print(json.dumps({"fold": fold, "passes": len(passes), "dp_ms_total": round(tot, 1),
                  "kernel_tag": engine.kernel_tag()}), flush=True)

"""A/B of launch knobs on one pass (tool): the first (alpha, fold) group of the 5x5 grid cut
to WS_LANES penalties, run under each configuration in turn (three rounds, alternating), with
the roots compared bit for bit between configurations.
usage: python tools/pass_ab.py GEN_PAT LANES "KNOB=V[,KNOB=V]" ["..." ...]   ("-" = no knob)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from kmerpapa_amd import engine  # noqa: E402

gp, nl = sys.argv[1], int(sys.argv[2])
confs = sys.argv[3:] or ["-"]
prep = bench.prepare(gp)
plan = engine.get_plan(0, gp)
plan.set_counts(prep["Mk"], prep["Uk"])
plan.reserve(nl)
g = prep["groups"][0]
grp = [(g[0], g[1], g[2], list(g[3])[:nl])]
ms = {c: [] for c in confs}
roots = {}
base = dict(os.environ)
for rep in range(3):
    for c in confs:
        os.environ.clear()
        os.environ.update(base)
        if c != "-":
            for kv in c.split(","):
                k, v = kv.split("=", 1)
                os.environ[k] = v
        rt, re, nlv = plan.run(grp)
        ms[c].append(round(plan.stats()["dp_ms"], 2))
        roots[c] = (rt.view(np.uint32).tolist(), re.view(np.uint32).tolist(), nlv.tolist())
os.environ.clear()
os.environ.update(base)
same = all(roots[c] == roots[confs[0]] for c in confs)
print(json.dumps({"gen_pat": gp, "lanes": nl, "ms": ms, "roots_equal": same}), flush=True)

"""One library build's 1-lane passes (tool, run once per build by tools/lib_pass_ab.sh):
for each lattice, the first (alpha, fold) group cut to LANES penalties, three passes, the
kernel ms of each, the roots, and a digest of 2^22 sampled cells of every lane (the same
sample for every build, so two builds' lines must agree bit for bit).
usage: KMERPAPA_LIB=... python tools/lib_pass_ab.py LANES GEN_PAT [GEN_PAT ...]"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from kmerpapa_amd import engine  # noqa: E402

nl = int(sys.argv[1])
for gp in sys.argv[2:]:
    prep = bench.prepare(gp)
    engine.release_all()
    plan = engine.get_plan(0, gp)
    plan.set_counts(prep["Mk"], prep["Uk"])
    plan.reserve(nl)
    g = prep["groups"][0]
    grp = [(g[0], g[1], g[2], list(g[3])[:nl])]
    ms = []
    for rep in range(3):
        rt, re, nlv = plan.run(grp)
        ms.append(round(plan.stats()["dp_ms"], 2))
    rng = np.random.default_rng(7)
    cells = np.unique(rng.integers(0, plan.info["npat"], 1 << 22, dtype=np.uint64))
    h = hashlib.sha256()
    for j in range(nl):
        h.update(plan.gather_cells(j, cells).view(np.uint32).tobytes())
    print(json.dumps({"lib": os.path.basename(engine.LIB_PATH), "gen_pat": gp, "lanes": nl, "ms": ms,
                      "roots": [rt.view(np.uint32).tolist(), re.view(np.uint32).tolist(), nlv.tolist()],
                      "sample_digest": h.hexdigest()[:16]}), flush=True)

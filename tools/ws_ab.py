"""A/B of the persistent wave-specialised sweep for 1-lane groups (kp_dp_ws.h) against
kp_dp_kernel (tool).  For each lattice: one 1-lane pass with KP_WS=0 and KP_WS=1, kernel ms
of each (three runs, alternating), the root train/test/leaves of both, and a random sample
of 2^22 cells of the lane compared bit for bit between the two builds.
usage: python tools/ws_ab.py [GEN_PAT ...]   (default NNNNMNNNN NNNNNNNNN)
       WS_LANES=n: a group of n penalties (default 1)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from kmerpapa_amd import engine  # noqa: E402

nl = int(os.environ.get("WS_LANES", "1"))
for gp in sys.argv[1:] or ["NNNNMNNNN", "NNNNNNNNN"]:
    prep = bench.prepare(gp)
    engine.release_all()
    plan = engine.get_plan(0, gp)
    plan.set_counts(prep["Mk"], prep["Uk"])
    plan.reserve(nl)
    g = prep["groups"][0]
    grp = [(g[0], g[1], g[2], list(g[3])[:nl])]
    rng = np.random.default_rng(7)
    cells = np.unique(rng.integers(0, plan.info["npat"], 1 << 22, dtype=np.uint64))
    out = {"gen_pat": gp, "lanes": nl, "ms": {"0": [], "1": []}}
    vals = {}
    for rep in range(3):
        for ws in ("0", "1"):
            os.environ["KP_WS"] = ws
            rt, re, nlv = plan.run(grp)
            out["ms"][ws].append(round(plan.stats()["dp_ms"], 2))
            if rep == 0:
                vals[ws] = (rt.copy(), re.copy(), nlv.copy(), [plan.gather_cells(j, cells) for j in range(nl)])
    a, b = vals["0"], vals["1"]
    out["roots_equal"] = bool(np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32)) and
                              np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32)) and np.array_equal(a[2], b[2]))
    out["sample_cells"] = int(cells.size)
    out["sample_mismatches"] = int(sum(np.sum((x.view(np.uint32) != y.view(np.uint32)) & ~(np.isnan(x) & np.isnan(y)))
                                       for x, y in zip(a[3], b[3])))
    print(json.dumps(out), flush=True)

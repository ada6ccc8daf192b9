"""Phase ablations of the 9-mer sweep (tool): kernel time of one 5-lane pass with phases
skipped.  Needs the timing-ablation build (make -C kmerpapa_amd/csrc ablation) and
KMERPAPA_LIB=kmerpapa_amd/libkmerpapa_hip_ablation.so; every ablated pass returns
KP_E_STATE (its numbers are invalid) after recording its timings.
usage: python tools/ablate.py SKIP [SKIP ...]   (KP_DEBUG_SKIP bit sets, 0 = full pass;
  ABLATE_LANES=n: a pass of the group's first n penalties, default 5; ABLATE_PATTERN=gen_pat:
  another lattice, default NNNNMNNNN)
  1 = no gather, 2 = no level phase, 4 = no float64 logs, 8 = no low split scan,
  16 = no level barriers"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from kmerpapa_amd import engine  # noqa: E402

GP = os.environ.get("ABLATE_PATTERN", "NNNNMNNNN")
prep = bench.prepare(GP)
plan = engine.get_plan(0, GP)
plan.set_counts(prep["Mk"], prep["Uk"])
plan.reserve(int(os.environ.get("ABLATE_LANES", "5")))
g = prep["groups"][0]
g = (g[0], g[1], g[2], list(g[3])[:int(os.environ.get("ABLATE_LANES", "5"))])
for skip in sys.argv[1:] or ["0"]:
    os.environ["KP_DEBUG_SKIP"] = skip
    ms = []
    for rep in range(3):
        try:
            plan.run([g])
        except engine.KPError as e:
            if e.code != -4 or skip == "0":  # KP_E_STATE: an ablated pass
                raise
        ms.append(plan.stats()["dp_ms"])
    print(json.dumps({"KP_DEBUG_SKIP": int(skip), "dp_ms": [round(x, 2) for x in ms]}), flush=True)

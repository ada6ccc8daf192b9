"""Per-launch non-temporal load masks for the 9-mer 5-lane pass (tool).

Runs one (alpha, fold) group of the headline pass with KP_LAUNCH_TIMES=1 for every uniform
KP_NT_SLOW = 0..6 (child rows along that many slowest-varying high positions loaded
non-temporally) and records each launch's time; then picks, per high level, the fastest
count and A/B-times that per-launch table (KP_NT_SLOW_H) against the global default,
alternating.  Prints JSON lines."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from kmerpapa_amd import engine  # noqa: E402

gp = sys.argv[1] if len(sys.argv) > 1 else "NNNNMNNNN"
reps = int(os.environ.get("NT_REPS", "2"))
os.environ["KP_LAUNCH_TIMES"] = "1"
cfg = bench.CONFIGS["11mer" if len(gp) == 11 else "9mer"]
prep = bench.prepare(gp, alphas=cfg["alphas"], penalties=cfg["penalties"], nfolds=cfg["nfolds"])
plan = engine.get_plan(0, gp)
plan.set_counts(prep["Mk"], prep["Uk"])
g = prep["groups"][0]
plan.reserve(len(g[3]))
plan.run([g])


def run(env):
    for k in ("KP_NT_SLOW", "KP_NT_SLOW_H"):
        os.environ.pop(k, None)
    os.environ.update(env)
    plan.run([g])
    return plan.stats()["dp_ms"], plan.launch_ms()


per = {}
for ns in range(0, 7):
    ts = [run({"KP_NT_SLOW": str(ns)}) for _ in range(reps)]
    per[ns] = np.min([t[1] for t in ts], axis=0)
    print(json.dumps({"nt_slow": ns, "dp_ms": [round(t[0], 2) for t in ts],
                      "launch_ms": [round(float(x), 3) for x in per[ns]]}), flush=True)
n = len(per[3])
best = [min(range(7), key=lambda ns: per[ns][i]) for i in range(n)]
table = ",".join(str(b) for b in best)
print(json.dumps({"per_launch_best": best, "model_ms": round(float(sum(per[b][i] for i, b in enumerate(best))), 2),
                  "default_ms": round(float(sum(per[3])), 2)}), flush=True)
a, b = [], []
for _ in range(3):
    a.append(run({})[0])
    b.append(run({"KP_NT_SLOW_H": table})[0])
print(json.dumps({"default_dp_ms": [round(x, 2) for x in a], "tuned_dp_ms": [round(x, 2) for x in b],
                  "KP_NT_SLOW_H": table}), flush=True)

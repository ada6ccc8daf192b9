"""Per-launch device time of one 9-mer 5-lane pass (KP_LAUNCH_TIMES=1) beside each high
level's block count, split pairs and compulsory bytes (two child rows read per high split
pair, one row written, 4 B per cell and lane, padded rows): where the pass runs below the
HBM roofline (tool; one GPU)."""
import itertools
import json
import os
import sys

os.environ["KP_LAUNCH_TIMES"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from kmerpapa_amd import engine  # noqa: E402

GP = "NNNNMNNNN"
# level and split pairs of every sub-code of a general code (kp_plan.h kPerm / kSplit)
PERM = {"N": "ACGTRYSWKMBDHVN", "M": "ACM"}
NUC = {"A": "A", "C": "C", "G": "G", "T": "T", "R": "AG", "Y": "CT", "S": "GC", "W": "AT", "K": "GT", "M": "AC",
       "B": "CGT", "D": "AGT", "H": "ACT", "V": "ACG", "N": "ACGT"}
NPAIRS = {1: 0, 2: 1, 3: 3, 4: 7}

prep = bench.prepare(GP)
plan = engine.get_plan(0, GP)
plan.set_counts(prep["Mk"], prep["Uk"])
t = plan.info["low_positions"]
bpad = plan.info["block_pad"]
lv, npair = [], []
for g in GP[t:]:
    lv.append(np.array([len(NUC[c]) - 1 for c in PERM[g]]))
    npair.append(np.array([NPAIRS[len(NUC[c])] for c in PERM[g]]))
L = np.zeros(1, np.int64)
Pn = np.zeros(1, np.int64)
for a, b in zip(lv, npair):
    L = (L[:, None] + a[None, :]).ravel()
    Pn = (Pn[:, None] + b[None, :]).ravel()
lanes = 5
g0 = prep["groups"][0]
best = None
for _ in range(3):
    plan.run([g0])
    ms = plan.launch_ms()
    if best is None or ms.sum() < best.sum():
        best = ms.copy()
rows = []
for H in range(L.max() + 1):
    sel = L == H
    nb = int(sel.sum())
    pairs = int(Pn[sel].sum())
    byts = (2 * pairs + 1) * lanes * bpad * 4.0
    ms = float(best[H])
    rows.append({"H": H, "blocks": nb, "pairs_per_block": round(pairs / nb, 2), "ms": round(ms, 3),
                 "GB": round(byts / 1e9, 1), "TBps": round(byts / ms / 1e9, 2)})
    print(json.dumps(rows[-1]), flush=True)
print(json.dumps({"total_ms": round(float(best.sum()), 2)}), flush=True)

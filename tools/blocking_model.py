"""Model (tool, host only) of blockings with fewer compulsory bytes per unit than the product's
(VERDICT r05 item 3): for each candidate, its compulsory bytes per unit, the LDS one workgroup
needs, the workgroups a CU then holds, and a predicted pass time from the measured parts of
the product's pass.

Predicted time = base (prologue, count tables, store; per block, from the ablation with
neither gather nor level phase) x (blocks ratio) + gather (ablation "no level phase" minus
base) x (compulsory bytes ratio) + level phase (ablation "no gather" minus base) x the
occupancy penalty of running fewer workgroups per CU, all overlapped as much as the product
overlaps them now (its measured full pass / the sum of its parts).  The occupancy penalty is
measured too: the 5-lane level phase alone at one workgroup per CU took 327 ms against 199 at
two (profiles/r02/experiments/ablate_occ*.txt), and the 1-lane consumer of the persistent
sweep at 16 waves per CU 107 ms against 62 at 24 (profiles/r06/experiments/ws_1lane.txt):
x1.64 per halving, taken as x(1.64 ** log2(wg_now / wg_new)).

Candidates:
  product   the low t positions of the general pattern in LDS (B = 3,375 cells at 9-mers)
  (a) M in the block: the centre M moved into the block for <= 3-lane builds (B = 10,125)
  (b) fiber: a workgroup walks the 15 blocks along one high N axis in level order and keeps
      the axis's level-0/1 rows (10 of 15) in LDS; N's B/D/H/V children still come from HBM
  (c) L2 super-block: two high positions' 225 blocks resident in one XCD's 4 MB L2
usage: python tools/blocking_model.py"""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kmerpapa_amd import engine  # noqa: E402

LDS_CU = 160 * 1024
# measured parts of 1-lane passes (ms): full, no gather, no level phase, neither
# (profiles/r06/experiments/ablate_1lane.txt, ablate_NNNNNNNNN_1lane.txt)
MEAS = {"NNNNMNNNN": (107.6, 81.3, 65.1, 18.9), "NNNNNNNNN": (592.1, 435.0, 386.5, 95.0)}
OCC = 1.64  # level phase slow-down per halving of resident workgroups (see docstring)


def lds_1lane(B, ptab_entries, scratch_entries, ct=4, kh=6, rows=1):
    """LDS of a 1-lane workgroup: `rows` score rows, the count table and its build buffers
    (the intermediate tables only, as kp_dp_ws.h sizes them), high pairs, masks."""
    return rows * 4 * (B + 32) + 2 * ct * ptab_entries + 2 * 2 * ct * scratch_entries + (kh * 7 + 1) * 24 + 64


def fits(lds, wg):
    return "yes" if lds * wg <= LDS_CU else "no"


def predict(gp, B_ratio, bytes_ratio, wg_now, wg_new):
    full, nog, nol, base = MEAS[gp]
    gather, level = nol - base, nog - base
    overlap = full / (base + gather + level)
    pen = OCC ** math.log2(wg_now / wg_new) if wg_new < wg_now else 1.0
    return overlap * (base / B_ratio + gather * bytes_ratio + level * pen)


out = []
for gp in ("NNNNMNNNN", "NNNNNNNNN"):
    info = engine.plan_info(gp)
    B = info["block"]
    ph = info["pairs_high"] / info["npat"]
    now = 8 * ph + 4
    ct = 8 if gp == "NNNNNNNNN" else 4
    lds_now = lds_1lane(B, 15 * 15 * 4, 15 * 4 * 4, ct)
    wg_now = 3  # 1-lane builds: 6 waves per SIMD, 8-wave workgroups
    rows = [{"candidate": "product", "B": B, "bytes_per_unit": round(now, 2), "lds_per_wg": lds_now,
             "wg_per_cu": wg_now, "predicted_ms": round(predict(gp, 1, 1, wg_now, wg_now), 1),
             "measured_ms": MEAS[gp][0]}]
    if "M" in gp:  # (a)
        Bm = B * 3
        bpu = 8 * (ph - 1.0 / 3.0) + 4
        lds = lds_1lane(Bm, 15 ** 3 * 2, 15 ** 2 * 4 * 2, ct, kh=5)
        wg = max(1, min(wg_now, LDS_CU // lds))
        rows.append({"candidate": "(a) M in the block", "B": Bm, "bytes_per_unit": round(bpu, 2), "lds_per_wg": lds,
                     "wg_per_cu": wg, "fits_lds": fits(lds, wg),
                     "predicted_ms": round(predict(gp, 3, bpu / now, wg_now, wg), 1)})
    # (b) fiber along one high N axis: 10 rows of the axis kept (levels 0-1), a working row
    n_axis_pairs = 25.0 / 15.0  # split pairs of one N position per cell (averaged over its digits)
    kept = 2 * n_axis_pairs - (4.0 / 15.0)  # child rows per cell along the axis minus N's B/D/H/V children
    bpu = now - 4 * kept
    lds = lds_1lane(B, 15 * 15 * 4, 15 * 4 * 4, ct, rows=11)
    wg = max(1, min(wg_now, LDS_CU // lds))
    rows.append({"candidate": "(b) fiber along one high N", "B": B, "bytes_per_unit": round(bpu, 2), "lds_per_wg": lds,
                 "wg_per_cu": wg, "fits_lds": fits(lds, wg),
                 "predicted_ms": round(predict(gp, 1, bpu / now, wg_now, wg), 1)})
    # (c) two high N positions' 225 blocks in one XCD's L2 (1 lane): 225 x row bytes
    sb = 225 * 4 * (B + 32)
    stream = 32 * wg_now * (2 * ph) * 4 * (B + 32)  # the child rows the XCD's resident workgroups stream meanwhile
    rows.append({"candidate": "(c) L2 super-block of two high N", "B": B, "bytes_per_unit": round(now, 2),
                 "lds_per_wg": lds_now, "wg_per_cu": wg_now, "super_block_bytes": sb, "l2_per_xcd": 4 << 20,
                 "streamed_meanwhile_bytes": int(stream),
                 "predicted_ms": "no byte saving: the super-block (3.1 MB) and the resident workgroups' child rows "
                                 "(~%.0f MB) do not fit a 4 MB L2 together" % (stream / 1e6)})
    out.append({"gen_pat": gp, "lanes": 1, "rows": rows})
for o in out:
    print(json.dumps(o))

"""Experiment: do two DP passes on two HIP streams of one GPU overlap usefully?

The low high-level launches of a pass are bound by per-block work (~100 ns per block,
DESIGN.md 5), the high ones by the gather's bandwidth.  Two independent passes running at
once on two streams (two kp_ctx on the same device) can mix the two kinds of workgroups.
This times N passes run one after the other on one stream against the same N passes split
over two streams (two host threads), and prints units/s for both.

usage: python tools/concurrency_exp.py GEN_PAT LANES NPASSES
"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from kmerpapa_amd import engine  # noqa: E402


def main():
    gp = sys.argv[1] if len(sys.argv) > 1 else "NNNNMNNN"
    lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    prep = bench.prepare(gp)
    groups = [(f, a, b, pens[:lanes]) for f, a, b, pens in prep["groups"]][:n]
    devs = [engine.Device(0), engine.Device(0)]
    plans = [engine.Plan(d, gp) for d in devs]
    for p in plans:
        p.reserve(lanes)
        p.set_counts(prep["Mk"], prep["Uk"])
        p.run([groups[0]])  # warm-up
    units = plans[0].info["npat"] * lanes * len(groups)

    t0 = time.perf_counter()
    single = [plans[0].run([g]) for g in groups]
    t_single = time.perf_counter() - t0

    out = [None, None]

    def work(i):
        out[i] = [plans[i].run([g]) for g in groups[i::2]]
    t0 = time.perf_counter()
    ths = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    t_dual = time.perf_counter() - t0
    same = all(single[2 * j + i][0].tobytes() == out[i][j][0].tobytes()
               for i in range(2) for j in range(len(out[i])))
    print({"gen_pat": gp, "lanes": lanes, "passes": len(groups), "single_s": round(t_single, 4),
           "dual_s": round(t_dual, 4), "single_ms_per_pass": round(t_single / len(groups) * 1e3, 2),
           "dual_ms_per_pass": round(t_dual / len(groups) * 1e3, 2), "speedup": round(t_single / t_dual, 4),
           "units_per_s_single": units / t_single, "units_per_s_dual": units / t_dual, "roots_equal": same},
          flush=True)
    for p in plans:
        p.close()
    for d in devs:
        d.close()


if __name__ == "__main__":
    main()

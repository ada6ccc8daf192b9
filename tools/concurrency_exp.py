"""Experiment: do two DP passes on two HIP streams of one GPU overlap usefully?

The low high-level launches of a pass are bound by per-block work (~100 ns per block,
DESIGN.md 5), the high ones by the gather's bandwidth.  Two independent passes running at
once on two streams (two kp_ctx on the same device) can mix the two kinds of workgroups.
This times N passes run one after the other on one stream, then two streams running N
passes each, the second starting OFFSET_MS later (so that its low levels meet the first
one's high levels), and reports the steady-state period per pass of each stream.

usage: python tools/concurrency_exp.py GEN_PAT LANES NPASSES [OFFSET_MS ...]
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
    offsets = [float(x) for x in sys.argv[4:]] or [0.0]
    prep = bench.prepare(gp)
    groups = [(f, a, b, pens[:lanes]) for f, a, b, pens in prep["groups"]]
    groups = (groups * (1 + 2 * n // len(groups)))[:2 * n]
    devs = [engine.Device(0), engine.Device(0)]
    plans = [engine.Plan(d, gp) for d in devs]
    for p in plans:
        p.reserve(lanes)
        p.set_counts(prep["Mk"], prep["Uk"])
        p.run([groups[0]])  # warm-up
    per_pass_units = plans[0].info["npat"] * lanes

    t0 = time.perf_counter()
    ref = [plans[0].run([g]) for g in groups[:n]]
    t_single = (time.perf_counter() - t0) / n
    print({"gen_pat": gp, "lanes": lanes, "single_ms_per_pass": round(t_single * 1e3, 2),
           "units_per_s": per_pass_units / t_single}, flush=True)

    for off in offsets:
        stamps = [[], []]
        out = [[], []]

        def work(i):
            if i == 1 and off > 0:
                time.sleep(off / 1e3)
            for g in groups[i * n:(i + 1) * n]:
                out[i].append(plans[i].run([g]))
                stamps[i].append(time.perf_counter())
        ths = [threading.Thread(target=work, args=(i,)) for i in range(2)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        # steady state: the passes both streams ran side by side (the first and last pass
        # of each stream overlap the other stream only partly)
        per = [(s[-2] - s[0]) / (len(s) - 2) for s in stamps]
        both = 2 * per_pass_units / max(per)
        same = out[0][0][0].tobytes() == ref[0][0].tobytes()
        print({"offset_ms": off, "stream_ms_per_pass": [round(x * 1e3, 2) for x in per],
               "pair_ms": round(max(per) * 1e3, 2), "units_per_s": both, "vs_single": round(both * t_single /
                                                                                           per_pass_units, 4),
               "wall_s": round(time.perf_counter() - t0, 3), "roots_equal": same}, flush=True)
    for p in plans:
        p.close()
    for d in devs:
        d.close()


if __name__ == "__main__":
    main()

"""Randomised GPU-vs-oracle parity sweep (not part of the test suite: a longer run of
tests/test_gpu_parity.py's random cases).  Random IUPAC general patterns (k = 3..6, at
most two N), random counts (zeros included), folds, pseudo counts, 1-8 penalties, block
sizes and lanes per workgroup; every cell's float32 score and every root test value must
equal the oracle's bit for bit.  usage: python tools/parity_sweep.py N_CASES SEED  (SWEEP_MAX_CELLS bounds the lattice, SWEEP_K lists the pattern lengths;
SWEEP_U64=1 scales the counts past 2^32 so that every case takes the uint64 itype).  Half the
cases run two alphas per fold, so that the library cuts their lanes into mixed device groups
(two (alpha, beta) sets in one workgroup, the MIX builds)"""
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kmerpapa_amd import engine as eng  # noqa: E402
from kmerpapa_amd.CV_tools import fold_tables  # noqa: E402
from kmerpapa_amd.pattern_utils import generality, matches, perm_code  # noqa: E402
from oracle import oracle as O  # noqa: E402


MAX_CELLS = int(os.environ.get("SWEEP_MAX_CELLS", "300000"))
U64 = os.environ.get("SWEEP_U64") == "1"
KS = [int(x) for x in os.environ.get("SWEEP_K", "3,4,5,6,7").split(",")]  # pattern lengths drawn from


def case(rng):
    k = rng.choice(KS)
    while True:
        gp = "".join(rng.choice("MRSWKYACGTBDHVNNN") for _ in range(k))
        if np.prod([len(perm_code[c]) for c in gp]) <= MAX_CELLS:
            break
    ctx = {}
    for kmer in matches(gp):
        bg = rng.randrange(0, 30000) if rng.random() > 0.1 else 0
        pos = rng.randrange(0, bg + 1) // rng.choice([1, 5, 50, 500])
        ctx[kmer] = (pos, bg - pos)
    if sum(v[0] for v in ctx.values()) == 0:
        ctx[next(iter(ctx))] = (5, 100)
    if U64:  # totals past 2^32 - 1: the reference's uint64 itype (CV :94-97)
        scale = (2 ** 33) // max(1, sum(m + u for m, u in ctx.values())) + 1
        ctx = {k: (m * scale, u * scale) for k, (m, u) in ctx.items()}
    return gp, ctx


def main():
    n, seed = int(sys.argv[1]), int(sys.argv[2])
    rng = random.Random(seed)
    dev = eng.get_device(0)
    bad = 0
    t0 = time.time()
    for i in range(n):
        gp, ctx = case(rng)
        nf = rng.choice([2, 3, 5])
        os.environ["KP_LANES_PER_WG"] = str(rng.choice([1, 2, 3, 4, 5, 5, 5, 6, 8]))
        itype = np.uint64 if U64 else np.uint32
        contexts, Mf, Uf = fold_tables(ctx, nf, np.random.RandomState(i), itype)
        Mk, Uk = eng.counts_in_kmer_order(gp, contexts, Mf, Uf, generality(gp), itype)
        alphas = rng.sample([0.0, 0.1, 1.0, 7.0], rng.choice([1, 2]))
        tot_m = Mf.sum(axis=0).astype(np.uint64)
        tot_u = Uf.sum(axis=0).astype(np.uint64)
        mtr, utr = tot_m.sum() - tot_m, tot_u.sum() - tot_u
        with np.errstate(divide="ignore", invalid="ignore"):
            betas = {a: (a * (1.0 - mtr / (mtr + utr))) / (mtr / (mtr + utr)) for a in alphas}
        pens = sorted(rng.sample([0.0, 0.7, 2.0, 3.3, 5.0, 8.0, 13.0, 21.0], rng.randint(1, 8)))
        plan = eng.Plan(dev, gp, rng.choice([0, 0, 16, 64, 512, 2048]))
        plan.set_counts(Mk, Uk)
        try:
            groups = [(f, a, float(betas[a][f]), pens) for f in range(nf) for a in alphas]
            _, re, _ = plan.run(groups)
            for ai, alpha in enumerate(alphas):
                for pi, c in enumerate(pens):
                    ref = O.cv_pass(gp, contexts, Mf, Uf, alpha, betas[alpha], c, 64 if U64 else 32)
                    for f in range(nf):
                        lane = (f * len(alphas) + ai) * len(pens) + pi
                        score, _ = plan.dump_lane(lane)
                        ok = np.array_equal(np.asarray(score).view(np.uint32), ref["score"][:, f].view(np.uint32)) and \
                            np.float32(re[lane]).tobytes() == np.float32(ref["root_test"][f]).tobytes()
                        if not ok:
                            bad += 1
                            print("MISMATCH", i, gp, nf, alpha, c, f, flush=True)
        except eng.KPError as e:
            print("error", i, gp, alphas, e, flush=True)
            bad += 1
        plan.close()
        if i % 20 == 0:
            print(f"case {i} {gp} ({generality(gp)} k-mers) {bad} bad so far, {time.time() - t0:.0f} s", flush=True)
    print(f"done: {n} cases, {bad} mismatches", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

"""Pure-Python restatement of the reference's CV pass: the "reference-equivalent pure-Python
path" of SURVEY.md 8(d), timed by bench.py's cpu_baseline beside the C oracle.

TEST INFRASTRUCTURE ONLY (like the rest of oracle/): imported by tests/ and by the
cpu_baseline leg of bench.py (as a child process), never by the product package.

What the reference runs per (alpha, penalty) -- src/kmerpapa/algorithms/
bottum_up_array_penalty_plus_pseudo_CV.py, executed as plain Python when numba's njit
is an identity (how SURVEY.md 6 timed it, ~1e5 units/s):
  * level 0, score_test_folds :15-20 with get_train :22-24: every k-mer row gets
    train = f32(-2 (xlogy(M_tr, p) + xlog1py(U_tr, -p)) + c), test likewise on the fold;
  * levels >= 1, handle_pattern :26-78: splits at every ambiguous position in position
    order, pairs in table order; f32 sums of the children's train and test values, taken
    on a strict "<" per fold; the first split's counts are the cell's counts (:52-55,
    wrapping at itype width); then the float64 single-pattern term c + (-2 M) log p +
    (-2 U) log(1-p), compared in float64 against the float32 store (:56-78).
Cells are visited in ascending index order, which is topological: a split child has a
strictly smaller digit at the split position, so a smaller index (the reference walks
level by level; the order inside a level changes no value).  Fold vectors are numpy
float32 (exact float32 adds and compares), the single term is Python float64 with
math.log / math.log1p (the C library's, as numba and the C oracle call).  Pinned against
the C oracle bit for bit in tests/test_pyref.py.
"""
import math
import sys
import time

import numpy as np

_PERM = {"A": "A", "C": "C", "G": "G", "T": "T", "R": "AGR", "Y": "CTY", "S": "GCS",
         "W": "ATW", "K": "GTK", "M": "ACM", "B": "CGTSYKB", "D": "AGTRWKD",
         "H": "ACTMWYH", "V": "ACGMRSV", "N": "ACGTRYSWKMBDHVN"}
_PAIRS = {"R": "AG", "Y": "CT", "S": "GC", "W": "AT", "K": "GT", "M": "AC",
          "V": "AS CR GM", "H": "AY CW TM", "D": "AK GW TR", "B": "CK GY TS",
          "N": "SW KM RY AB CD GH TV"}


def _lattice(gen_pat):
    """Per position: radix, place value, and for every digit whether it is a nucleotide
    and its split pairs as (child1 - cell, child2 - cell) index offsets."""
    pos = []
    w = 1
    for g in gen_pat:
        perm = _PERM[g]
        digits = []
        for d, x in enumerate(perm):
            pairs = [((perm.index(p[0]) - d) * w, (perm.index(p[1]) - d) * w) for p in _PAIRS.get(x, "").split()]
            digits.append((x in "ACGT", pairs))
        pos.append((len(perm), digits))
        w *= len(perm)
    return pos, w


# IEEE-754 semantics where Python would raise (0/0 -> NaN, log 0 -> -inf, log of a
# negative or NaN -> NaN), as numba and C compute them; positive finite arguments go to
# the C library's log / log1p
def _div(a, b):
    try:
        return a / b
    except ZeroDivisionError:
        return math.nan if (a != a or a == 0.0) else math.copysign(math.inf, a) * math.copysign(1.0, b)


def _log(x):
    return math.log(x) if x > 0.0 else (-math.inf if x == 0.0 else math.nan)


def _log1p(x):
    return math.log1p(x) if x > -1.0 else (-math.inf if x == -1.0 else math.nan)


def _xlogy(x, y):
    return 0.0 if (x == 0 and y == y) else x * _log(y)


def _xlog1py(x, y):
    return 0.0 if (x == 0 and y == y) else x * _log1p(y)


def cv_pass(gen_pat, M, U, alpha, betas, penalty, itype_bits=32):
    """One CV pass over all folds for one (alpha, penalty).  ``M``/``U``: ``[npat, nf]``
    uint64 with the k-mer rows filled (cell index order, position 0 fastest); the other rows
    are overwritten with the aggregated counts.  Returns float32 ``(score, test)``
    ``[npat, nf]``."""
    pos, npat = _lattice(gen_pat)
    nf = M.shape[1]
    mask = np.uint64((1 << itype_bits) - 1) if itype_bits < 64 else np.uint64(0xFFFFFFFFFFFFFFFF)
    score = np.full((npat, nf), np.inf, np.float32)
    test = np.zeros((npat, nf), np.float32)
    betas = [float(b) for b in betas]
    alpha = float(alpha)
    penalty = float(penalty)
    for n in range(npat):
        rest = n
        kmer = True
        splits = []
        for r, digits in pos:
            nuc, pairs = digits[rest % r]
            rest //= r
            kmer = kmer and nuc
            splits.extend(pairs)
        m_row = [int(v) for v in M[n]]
        u_row = [int(v) for v in U[n]]
        if kmer:
            sm, su = sum(m_row), sum(u_row)
            for f in range(nf):
                mtr, utr = sm - m_row[f], su - u_row[f]
                p = _div(float(mtr) + alpha, (float(mtr + utr) + alpha) + betas[f])
                score[n, f] = -2.0 * (_xlogy(float(mtr), p) + _xlog1py(float(utr), -p)) + penalty
                test[n, f] = -2.0 * (_xlogy(float(m_row[f]), p) + _xlog1py(float(u_row[f]), -p))
            continue
        best, best_t = score[n], test[n]  # views: updated in place
        for i, (o1, o2) in enumerate(splits):
            c1, c2 = n + o1, n + o2
            cand = score[c1] + score[c2]
            take = cand < best
            if take.any():
                cand_t = test[c1] + test[c2]
                best[take] = cand[take]
                best_t[take] = cand_t[take]
            if i == 0:
                M[n] = (M[c1] + M[c2]) & mask
                U[n] = (U[c1] + U[c2]) & mask
                m_row = [int(v) for v in M[n]]
                u_row = [int(v) for v in U[n]]
        sm, su = sum(m_row), sum(u_row)
        for f in range(nf):
            mtr, utr = sm - m_row[f], su - u_row[f]
            p = _div(float(mtr) + alpha, (float(mtr + utr) + alpha) + betas[f])
            logp, log1mp = _log(p), _log(1.0 - p)
            s = penalty
            if mtr > 0:
                s += (-2.0 * float(mtr)) * logp
            if utr > 0:
                s += (-2.0 * float(utr)) * log1mp
            if s < float(best[f]):
                best[f] = s
                t = 0.0
                if m_row[f] > 0:
                    t += (-2.0 * float(m_row[f])) * logp
                if u_row[f] > 0:
                    t += (-2.0 * float(u_row[f])) * log1mp
                best_t[f] = t
    return score, test


def _task(path):
    """Child-process entry of bench.py's timing: one (alpha, penalty) pass on the sample in
    ``path`` (npz: gen_pat, M, U, alpha, betas, penalty, itype_bits); prints seconds."""
    d = np.load(path)
    M, U = d["M"].copy(), d["U"].copy()
    t0 = time.perf_counter()
    cv_pass(str(d["gen_pat"]), M, U, float(d["alpha"]), d["betas"], float(d["penalty"]), int(d["itype_bits"]))
    print(time.perf_counter() - t0, flush=True)


if __name__ == "__main__":
    _task(sys.argv[1])

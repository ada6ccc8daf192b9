"""Brute force on tiny lattices (SURVEY.md §4 test plan item 4): enumerate EVERY split tree
of the general pattern (every partition the reference's recursion can express: keep a
pattern whole, or split it at one ambiguous position into one of its complement pairs,
pattern_utils.py:48-84, and recurse), score each partition in float64 as the sum of its
patterns' terms (Fit :26-29 for single k-mers, :56-61 for wider patterns), and check that
the DP finds the minimum: its float32 root score equals the brute-force minimum to float32
accuracy, and the partition it returns scores that minimum (ties allowed).

The CPU test checks the oracle (pinned to the reference by test_oracle_golden.py) this way;
the GPU test checks the HIP fit through the drop-in driver.
"""
import math
import random

import pytest

from oracle.oracle import _PERM, _SPLIT

CASES = ["NM", "RN", "NS", "MMM", "RYS", "SWK", "N", "NMA"]


def _matches(pat):
    out = [""]
    for x in pat:
        out = [o + n for o in out for n in _PERM[x] if n in "ACGT"]
    return out


def _ctx(pat, seed):
    rng = random.Random(seed)
    ctx = {}
    for kmer in _matches(pat):
        bg = rng.randrange(0, 4000) if rng.random() > 0.15 else 0
        ctx[kmer] = (rng.randrange(0, bg + 1) // rng.choice([1, 5, 40]), bg)
    for k, (m, b) in ctx.items():
        ctx[k] = (m, b - m)
    if sum(v[0] for v in ctx.values()) == 0:
        ctx[next(iter(ctx))] = (5, 900)
    return ctx


def _term(pat, ctx, alpha, beta, pen):
    ks = _matches(pat)
    m = sum(ctx[k][0] for k in ks)
    u = sum(ctx[k][1] for k in ks)
    p = (m + alpha) / (((m + u) + alpha) + beta)
    if len(pat) == sum(1 for x in pat if x in "ACGT"):  # one k-mer: xlogy / xlog1py form
        a = 0.0 if m == 0 else m * math.log(p)
        b = 0.0 if u == 0 else u * math.log1p(-p)
        return -2.0 * (a + b) + pen
    s = pen
    if m > 0:
        s += (-2.0 * m) * math.log(p)
    if u > 0:
        s += (-2.0 * u) * math.log(1.0 - p)
    return s


def _all_partitions(pat):
    """Every split tree's leaf list (the same partition can come from several trees)."""
    out = [[pat]]
    for i, x in enumerate(pat):
        if x not in _SPLIT:
            continue
        for pr in _SPLIT[x].split():
            left = _all_partitions(pat[:i] + pr[0] + pat[i + 1:])
            right = _all_partitions(pat[:i] + pr[1] + pat[i + 1:])
            out.extend(a + b for a in left for b in right)
    return out


def _brute(pat, ctx, alpha, beta, pen):
    cache = {}

    def t(p):
        if p not in cache:
            cache[p] = _term(p, ctx, alpha, beta, pen)
        return cache[p]
    parts = _all_partitions(pat)
    scores = [math.fsum(t(p) for p in part) for part in parts]
    return min(scores), {tuple(sorted(p)): s for p, s in zip(parts, scores)}, t


def _params(ctx, alpha):
    nm = sum(v[0] for v in ctx.values())
    nu = sum(v[1] for v in ctx.values())
    my = nm / (nm + nu)
    return nm, nu, (alpha * (1.0 - my)) / my


def _check(pat, ctx, alpha, beta, pen, score, names):
    best, by_part, t = _brute(pat, ctx, alpha, beta, pen)
    # every k-mer covered exactly once
    cover = sorted(k for n in names for k in _matches(n))
    assert cover == sorted(ctx)
    got = math.fsum(t(n) for n in names)
    tol = 4e-7 * max(1.0, abs(best))
    assert abs(float(score) - best) <= tol, (pat, float(score), best)
    assert got <= best + tol, (pat, got, best)  # the returned partition attains the minimum
    assert tuple(sorted(names)) in by_part  # and is one the split recursion can express


@pytest.mark.parametrize("pat", CASES)
@pytest.mark.parametrize("pen", [0.0, 3.0, 25.0])
def test_oracle_fit_is_bruteforce_optimal(pat, pen):
    import numpy as np

    from oracle import oracle as O
    ctx = _ctx(pat, 31 * sum(map(ord, pat)) + int(pen))
    alpha = 0.7
    nm, nu, beta = _params(ctx, alpha)
    ks = list(ctx)
    M = np.array([ctx[k][0] for k in ks], np.int64)
    U = np.array([ctx[k][1] for k in ks], np.int64)
    score, _, _, names, _ = O.fit(pat, ks, M, U, alpha, beta, pen, 32)
    _check(pat, ctx, alpha, beta, pen, score, names)


@pytest.mark.gpu
@pytest.mark.parametrize("pat", CASES)
@pytest.mark.parametrize("pen", [0.0, 3.0, 25.0])
def test_gpu_fit_is_bruteforce_optimal(pat, pen):
    from kmerpapa_amd import engine
    from kmerpapa_amd.algorithms import bottum_up_array_w_numba as fitm
    engine.load()
    ctx = _ctx(pat, 31 * sum(map(ord, pat)) + int(pen))
    alpha = 0.7
    nm, nu, beta = _params(ctx, alpha)

    class A:
        verbosity = 0
    score, _, _, names = fitm.pattern_partition_bottom_up(pat, ctx, alpha, beta, pen, A, nm, nu)
    _check(pat, ctx, alpha, beta, pen, score, names)

"""Score helpers of the penalized likelihood (host side).

Same names and arithmetic as the reference's ``kmerpapa.score_utils``
(src/kmerpapa/score_utils.py:3-35).  The reference's ``scipy.special.xlogy`` / ``xlog1py``
are x times the C library's log / log1p (tests/test_libm.py
test_scipy_xlogy_xlog1py_are_libm), with x == 0 -> 0 unless y is NaN; they are restated
here on Python's math module (the same libm calls) -- importing scipy took 0.3 s of the
CLI's run (its LL line), and the values are bit-identical (tests/test_score_utils.py).
"""
import math

_NAN, _NEG_INF = float("nan"), float("-inf")


def xlogy(x, y):
    """scipy.special.xlogy for Python floats: 0 if x == 0 and y is not NaN, else x * log(y)."""
    if y != y:
        return _NAN
    if x == 0:
        return 0.0
    return x * (math.log(y) if y > 0 else (_NEG_INF if y == 0 else _NAN))


def xlog1py(x, y):
    """scipy.special.xlog1py for Python floats: 0 if x == 0 and y is not NaN, else x * log1p(y)."""
    if y != y:
        return _NAN
    if x == 0:
        return 0.0
    return x * (math.log1p(y) if y > -1 else (_NEG_INF if y == -1 else _NAN))


def get_loss(L, alpha, beta, penalty=0):
    """-2 * log-likelihood of (n_pos, n_neg) pairs plus ``len(L) * penalty`` (ref :3-19)."""
    acc = 0.0
    for nm, nu in L:
        p = (nm + alpha) / (nm + nu + alpha + beta)
        acc += xlogy(nm, p) + xlog1py(nu, -p)
    return -2 * acc + len(L) * penalty


def get_betas(alpha, M, U):
    """Per-fold beta such that the prior mean alpha/(alpha+beta) is the fold's rate (ref :22-35)."""
    rate = M / (M + U)
    return (alpha * (1.0 - rate)) / rate

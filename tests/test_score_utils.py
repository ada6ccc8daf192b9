"""score_utils.get_loss / xlogy / xlog1py (reference score_utils.py:3-19): the math-module
restatement equals scipy.special's functions bit for bit, edge cases included."""
import math

import numpy as np

from kmerpapa_amd import score_utils as S


def _bits(a, b):
    a, b = float(a), float(b)
    return (math.isnan(a) and math.isnan(b)) or np.float64(a).tobytes() == np.float64(b).tobytes()


def test_xlogy_xlog1py_match_scipy():
    import scipy.special as sp
    rng = np.random.RandomState(3)
    xs = np.concatenate([rng.randint(0, 10 ** 7, 20000).astype(float), [0.0, 0.0, 1.0, 5.0]])
    ys = np.concatenate([rng.uniform(0, 1, 20000), [0.0, float("nan"), 0.0, 1.0]])
    for x, y in zip(xs, ys):
        assert _bits(S.xlogy(x, y), sp.xlogy(x, y)), (x, y)
        assert _bits(S.xlog1py(x, -y), sp.xlog1py(x, -y)), (x, -y)
    for x, y in [(1.0, -1.0), (2.0, -2.0), (0.0, -3.0), (3.0, -0.5)]:
        assert _bits(S.xlogy(x, y), sp.xlogy(x, y)), (x, y)
        assert _bits(S.xlog1py(x, y), sp.xlog1py(x, y)), (x, y)


def test_get_loss_matches_scipy_formula():
    import scipy.special as sp
    rng = np.random.RandomState(4)
    L = [(int(m), int(u)) for m, u in zip(rng.randint(0, 500, 3000), rng.randint(0, 10 ** 6, 3000))]
    alpha, beta = 2.0, 7.3e4
    acc = 0.0
    for nm, nu in L:
        p = (nm + alpha) / (nm + nu + alpha + beta)
        acc += sp.xlogy(nm, p) + sp.xlog1py(nu, -p)
    assert _bits(S.get_loss(L, alpha, beta), -2 * acc)
    assert _bits(S.get_loss(L, alpha, beta, 3.0), -2 * acc + len(L) * 3.0)

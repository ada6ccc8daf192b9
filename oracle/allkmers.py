"""CPU restatement of ``--score all_kmers``'s loss sums (numpy).

TEST INFRASTRUCTURE ONLY (the checker of ``kp_allkmers_cv``): imported by tests/, never by
the product package ``kmerpapa_amd``.

Restates src/kmerpapa/algorithms/all_kmers_CV.py (v0.2.4):
  * test_folds :8-13   p = (trM + a) / (trM + trU + a + b); -2 (xlogy(teM, p) + xlog1py(teU, -p))
  * k-mer loop :36-44  trM = row total - fold (uint64); sum_train / sum_test accumulated
                       row by row in float64 from numpy.zeros(nf), in matches() order
scipy's xlogy / xlog1py call the C library's log / log1p (tests/test_libm.py checks that).
Pinned by the reference's own CLI runs (tests/golden/allk5.json, tests/test_all_kmers.py).
"""
import numpy as np


def test_folds(trainM, trainU, testM, testU, alpha, betas):
    """-2 LL of test counts under the training rate (all_kmers_CV.py :8-13)."""
    from scipy.special import xlog1py, xlogy
    p = (trainM + alpha) / (trainM + trainU + alpha + betas)
    return -2 * (xlogy(testM, p) + xlog1py(testU, -p))


def _seq_sum_rows(terms):
    """Row-by-row float64 sum from 0.0, in order (``s += row`` in a loop)."""
    s = np.zeros(terms.shape[1])
    for row in terms:
        s += row
    return s


def allkmers_sums(M, U, alphas, betas, per_row=False):
    """``(sum_train, sum_test)`` ``[na, nf]`` for fold counts ``M``/``U`` ``[n, nf]``
    (uint64, matches() order) and ``betas`` ``[na, nf]`` -- the quantities kp_allkmers_cv
    returns.  ``per_row=True`` evaluates test_folds one k-mer row ([nf] arrays) at a time
    as the reference's loop does (:38-44): numpy's vectorised division over a whole
    [n, nf] table returns 0/0 as a NaN of the other sign than its [nf]-row path and the C
    library (measured), so NaN encodings are compared per row; the values are the same."""
    M = np.asarray(M, np.uint64)
    U = np.asarray(U, np.uint64)
    trM = M.sum(axis=1, keepdims=True) - M
    trU = U.sum(axis=1, keepdims=True) - U
    tr, te = [], []
    with np.errstate(divide="ignore", invalid="ignore"):
        for a, b in zip(alphas, np.asarray(betas, np.float64)):
            if per_row:
                s_tr, s_te = np.zeros(M.shape[1]), np.zeros(M.shape[1])
                for i in range(M.shape[0]):
                    s_tr += test_folds(trM[i], trU[i], trM[i], trU[i], a, b)
                    s_te += test_folds(trM[i], trU[i], M[i], U[i], a, b)
                tr.append(s_tr)
                te.append(s_te)
                continue
            tr.append(_seq_sum_rows(test_folds(trM, trU, trM, trU, a, b)))
            te.append(_seq_sum_rows(test_folds(trM, trU, M, U, a, b)))
    return np.array(tr).reshape(len(alphas), M.shape[1]), np.array(te).reshape(len(alphas), M.shape[1])

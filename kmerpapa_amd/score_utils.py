"""Score helpers of the penalized likelihood (host side).

Same names and arithmetic as the reference's ``kmerpapa.score_utils``
(src/kmerpapa/score_utils.py:3-35).  ``xlogy``/``xlog1py`` are scipy's
(x == 0 -> 0 unless y is NaN), the same third-party functions the reference calls
(imported on use: the CLI calls get_loss only when verbose, and starts 0.3 s faster).
"""


def get_loss(L, alpha, beta, penalty=0):
    """-2 * log-likelihood of (n_pos, n_neg) pairs plus ``len(L) * penalty`` (ref :3-19)."""
    from scipy.special import xlog1py, xlogy
    acc = 0.0
    for nm, nu in L:
        p = (nm + alpha) / (nm + nu + alpha + beta)
        acc += xlogy(nm, p) + xlog1py(nu, -p)
    return -2 * acc + len(L) * penalty


def get_betas(alpha, M, U):
    """Per-fold beta such that the prior mean alpha/(alpha+beta) is the fold's rate (ref :22-35)."""
    rate = M / (M + U)
    return (alpha * (1.0 - rate)) / rate

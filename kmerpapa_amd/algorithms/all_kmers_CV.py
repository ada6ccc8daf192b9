"""One rate per k-mer, cross-validated over the pseudo count -- drop-in for the
reference's ``kmerpapa.algorithms.all_kmers_CV`` (src/kmerpapa/algorithms/all_kmers_CV.py,
v0.2.4; ``--score all_kmers``).

There is no lattice DP here: every k-mer is its own pattern, so the per-k-mer -2LL is a
closed form.  The fold split is the shared one (CV_tools, native ``kp_fold_split``); the
losses of all (k-mer, fold) pairs of every pseudo count are evaluated on the GPU
(``kp_allkmers_cv``, csrc/kp_allk.h) with the reference's operation order and the C
library's logs, and summed k-mer by k-mer in float64 in ``matches`` order as the
reference's ``sum_test += ...`` loop does (:36-44), so results are bit-identical.
"""
import sys

import numpy as np

from .. import engine
from ..CV_tools import make_all_folds_contextD_kmers
from ..pattern_utils import generality
from ..score_utils import get_betas


def test_folds(trainM, trainU, testM, testU, alphas, betas):
    """-2 LL of test counts under the training rate (ref :8-13; host helper kept for the
    reference's API -- the CV below evaluates it on the GPU)."""
    from scipy.special import xlog1py, xlogy  # (imported on use: the CLI starts 0.2 s faster without it)
    p = (trainM + alphas) / (trainM + trainU + alphas + betas)
    return -2 * (xlogy(testM, p) + xlog1py(testU, -p))


def all_kmers(gen_pat, contextD, alphas, args, nmut, nunmut, index_mut=0):
    """Best pseudo count for one-rate-per-k-mer (ref :15-63).  Returns ``(best_alpha, best_test_loss)``."""
    nf = args.nfolds
    nit = args.iterations
    npat = generality(gen_pat)
    U_mem = np.zeros((npat, nf), dtype=np.uint64)
    M_mem = np.zeros((npat, nf), dtype=np.uint64)
    test_loss = {a_i: [] for a_i in range(len(alphas))}
    train_loss = {a_i: [] for a_i in range(len(alphas))}
    if index_mut != 0:
        contextD = {k: (v[index_mut], v[-1]) for k, v in contextD.items()}
    devices = engine.visible_devices()  # no CPU path: raises without the library / a GPU
    if not devices:
        raise engine.KPError(-3, "--score all_kmers runs on the GPU: no GPU is visible to the HIP runtime "
                                 f"({engine.LIB_PATH})")
    dev = engine.get_device(devices[0])
    prng = np.random.RandomState(args.seed)
    for _ in range(nit):
        make_all_folds_contextD_kmers(contextD, U_mem, M_mem, gen_pat, prng)
        M_sum_test = M_mem.sum(axis=0)  # n_mut for each fold
        U_sum_test = U_mem.sum(axis=0)
        M_sum_train = sum(M_sum_test) - M_sum_test
        U_sum_train = sum(U_sum_test) - U_sum_test
        betas = np.array([get_betas(alpha, M_sum_train, U_sum_train) for alpha in alphas], np.float64)
        sum_train, sum_test = dev.allkmers_cv(M_mem, U_mem, alphas, betas.reshape(len(alphas), nf))
        for a_i in range(len(alphas)):
            train_loss[a_i].extend(list(sum_train[a_i]))
            test_loss[a_i].extend(list(sum_test[a_i]))
    best_test_loss = 1e100
    best_alpha = None
    for a_i, alpha in enumerate(alphas):
        test = sum(test_loss[a_i]) / nit
        if args.verbosity > 0:
            print(f'alpha={alpha} test_loss={test}', file=sys.stderr)
        if test < best_test_loss:
            best_alpha = alpha
            best_test_loss = test
    return best_alpha, best_test_loss

"""CV_tools.fold_feed, the CV driver's pipelined fold split (host code, no GPU): the folds it
hands over in k-mer order are fold_tables' folds scattered by kmer_order, its all-data
counts are their sum, and a failure on the caller's side ends the producer thread."""
import numpy as np
import pytest

from kmerpapa_amd import engine
from kmerpapa_amd.CV_tools import fold_feed, fold_tables
from kmerpapa_amd.pattern_utils import generality, matches


def _ctx(gen_pat, seed):
    rng = np.random.RandomState(seed)
    return {c: (int(rng.randint(0, 40)), int(rng.randint(40, 900))) for c in matches(gen_pat)}


@pytest.mark.parametrize("gen_pat,nf", [("NMN", 3), ("NNRNN", 5)])
def test_fold_feed_equals_fold_tables(gen_pat, nf):
    ctx = _ctx(gen_pat, 7)
    feed, th = fold_feed(ctx, gen_pat, nf, np.random.RandomState(3), np.uint64)
    got = [feed.get(f) for f in range(nf)]
    th.join()
    contexts, M, U = fold_tables(ctx, nf, np.random.RandomState(3), np.uint64)
    idx = engine.kmer_order(gen_pat, list(contexts))
    nk = generality(gen_pat)
    for f in range(nf):
        m = np.zeros(nk, np.uint64)
        u = np.zeros(nk, np.uint64)
        m[idx] = M[:, f]
        u[idx] = U[:, f]
        assert np.array_equal(got[f][0], m) and np.array_equal(got[f][1], u)
    assert np.array_equal(feed.M_all, sum(g[0] for g in got))
    assert np.array_equal(feed.U_all, sum(g[1] for g in got))
    assert all(t is not None for t in feed.t_put)


def test_fold_feed_caller_failure_ends_producer():
    ctx = _ctx("NMN", 1)
    with pytest.raises(ValueError):
        fold_feed(ctx, "ANN", 3, np.random.RandomState(0), np.uint64)  # k-mers outside the pattern

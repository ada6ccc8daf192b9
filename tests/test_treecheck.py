"""The host tree re-derivation (oracle/treecheck.py) against the pinned oracle's full
arrays: fed the oracle's stored train scores, it must re-derive every tree node, the
root's test -2LL bit for bit and, in fit mode, the reference's partition in order.  This
is what makes it a checker for the GPU's full-size lanes (tests/test_gpu_fullsize.py)."""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import treecheck as T
from tests.fixtures import context_table, golden_json


def _kmer_index(lat, contexts):
    idx = np.zeros(len(contexts), np.int64)
    for j, ctx in enumerate(contexts):
        idx[j] = sum(T.IUPAC[g].index(ch) * w for g, ch, w in zip(lat.gp, ctx, lat.kw))
    return idx


@pytest.fixture(scope="module")
def grid5():
    from kmerpapa_amd.CV_tools import fold_tables
    ctx, gp, nm, nu = context_table(5)
    contexts, Mf, Uf = fold_tables(ctx, 5, np.random.RandomState(1), np.uint32)
    return gp, contexts, Mf.astype(np.int64), Uf.astype(np.int64)


@pytest.mark.parametrize("alpha,penalty", [(0.5, 3.0), (1.0, 5.0), (10.0, 7.0), (0.0, 2.0)])
def test_treecheck_cv_lanes_vs_oracle(grid5, alpha, penalty):
    from kmerpapa_amd.score_utils import get_betas
    gp, contexts, Mf, Uf = grid5
    lat = T.Lattice(gp)
    idx = _kmer_index(lat, contexts)
    Mk = np.zeros((lat.n_kmers, 5), np.int64)
    Uk = np.zeros((lat.n_kmers, 5), np.int64)
    Mk[idx], Uk[idx] = Mf, Uf
    ms, us = Mf.sum(axis=0), Uf.sum(axis=0)
    betas = get_betas(alpha, ms.sum() - ms, us.sum() - us)
    ref = O.cv_pass(gp, contexts, Mf, Uf, alpha, betas, penalty, 32)
    nodes = 0
    for f in range(5):
        r = T.rederive(lat, lambda cells: ref["score"][cells.astype(np.int64), f],
                       Mk.sum(axis=1) - Mk[:, f], Uk.sum(axis=1) - Uk[:, f], Mk[:, f], Uk[:, f],
                       alpha, float(betas[f]), penalty)
        assert r["root_train"].view(np.uint32) == ref["root_train"][f].view(np.uint32)
        assert r["root_test"].view(np.uint32) == ref["root_test"][f].view(np.uint32)
        nodes += r["nodes"]
        assert r["nodes"] == 2 * r["leaves"].size - 1
    assert nodes > 5


def test_treecheck_fit_partitions_vs_reference():
    """Fit mode (test counts zero): the leaves in backtrack order are the reference's own
    5-mer partitions (tests/golden/fit5.json: the reference's names)."""
    g = golden_json("fit5.json")
    ctx, gp, nm, nu = context_table(5)
    lat = T.Lattice(gp)
    ks = sorted(ctx)
    idx = _kmer_index(lat, ks)
    M = np.zeros(lat.n_kmers, np.int64)
    U = np.zeros(lat.n_kmers, np.int64)
    M[idx] = [ctx[k][0] for k in ks]
    U[idx] = [ctx[k][1] for k in ks]
    z = np.zeros_like(M)
    for fo in g["fits"]:
        sc, _, _, names, arrs = O.fit(gp, ks, M[idx], U[idx], fo["alpha"], fo["beta"], fo["penalty"], 32)
        r = T.rederive(lat, lambda cells: arrs["score"][cells.astype(np.int64)], M, U, z, z,
                       fo["alpha"], fo["beta"], fo["penalty"])
        assert float(r["root_train"]) == fo["score"]
        assert [lat.pattern(c) for c in r["leaves"]] == fo["names"]


def test_treecheck_catches_a_changed_child(grid5):
    """One ulp changed in a split child of the root: the walk names the root."""
    from kmerpapa_amd.score_utils import get_betas
    gp, contexts, Mf, Uf = grid5
    lat = T.Lattice(gp)
    idx = _kmer_index(lat, contexts)
    Mk = np.zeros((lat.n_kmers, 5), np.int64)
    Uk = np.zeros((lat.n_kmers, 5), np.int64)
    Mk[idx], Uk[idx] = Mf, Uf
    ms, us = Mf.sum(axis=0), Uf.sum(axis=0)
    betas = get_betas(1.0, ms.sum() - ms, us.sum() - us)
    ref = O.cv_pass(gp, contexts, Mf, Uf, 1.0, betas, 5.0, 32)
    s = ref["score"][:, 0].copy()
    r = T.rederive(lat, lambda cells: s[cells.astype(np.int64)], Mk.sum(axis=1) - Mk[:, 0],
                   Uk.sum(axis=1) - Uk[:, 0], Mk[:, 0], Uk[:, 0], 1.0, float(betas[0]), 5.0)
    assert r["leaves"].size > 1
    # a leaf one ulp lower: either its parent's best split sum drops (the parent's stored
    # value no longer re-derives) or it is absorbed by rounding and the leaf's own stored
    # value no longer matches its single-pattern term
    for cell in (int(r["leaves"][0]), int(r["leaves"][-1]), lat.root):
        t = s.copy()
        t[cell] = np.nextafter(t[cell], np.float32(-np.inf))
        with pytest.raises(T.TreeMismatch):
            T.rederive(lat, lambda cells: t[cells.astype(np.int64)], Mk.sum(axis=1) - Mk[:, 0],
                       Uk.sum(axis=1) - Uk[:, 0], Mk[:, 0], Uk[:, 0], 1.0, float(betas[0]), 5.0)


def _lane0(grid5, alpha=1.0, penalty=5.0):
    from kmerpapa_amd.score_utils import get_betas
    gp, contexts, Mf, Uf = grid5
    lat = T.Lattice(gp)
    idx = _kmer_index(lat, contexts)
    Mk = np.zeros((lat.n_kmers, 5), np.int64)
    Uk = np.zeros((lat.n_kmers, 5), np.int64)
    Mk[idx], Uk[idx] = Mf, Uf
    ms, us = Mf.sum(axis=0), Uf.sum(axis=0)
    betas = get_betas(alpha, ms.sum() - ms, us.sum() - us)
    ref = O.cv_pass(gp, contexts, Mf, Uf, alpha, betas, penalty, 32)
    args = (Mk.sum(axis=1) - Mk[:, 0], Uk.sum(axis=1) - Uk[:, 0], Mk[:, 0], Uk[:, 0], alpha, float(betas[0]), penalty)
    mtr = (ref["M"].sum(axis=1) - ref["M"][:, 0]).astype(np.int64)  # every cell's train counts
    utr = (ref["U"].sum(axis=1) - ref["U"][:, 0]).astype(np.int64)
    return lat, ref["score"][:, 0].copy(), args, mtr, utr


def _root_candidates(lat):
    dig = lat.digits(lat.root)
    out = []
    for i, d in enumerate(dig):
        base = lat.root - d * lat.cw[i]
        for pa, pb in lat.pairs[i][d]:
            out.append((base + pa * lat.cw[i], base + pb * lat.cw[i]))
    return out


@pytest.mark.parametrize("alpha,penalty", [(1.0, 5.0), (0.0, 2.0)])
def test_local_values_reproduce_every_cell(grid5, alpha, penalty):
    """The one-level re-derivation (local_values) of EVERY cell of the lattice from the
    oracle's stored scores and train counts gives the oracle's own value bit for bit
    (alpha = 0: empty k-mers give p = 0/0, NaN encodings included)."""
    from tests.fixtures import bits_equal
    lat, s, (mtr_k, utr_k, _, _, a, b, c), mtr, utr = _lane0(grid5, alpha, penalty)
    cells = np.arange(s.size)
    got = T.local_values(lat, cells, mtr, utr, lambda x: s[x.astype(np.int64)], a, b, c)
    assert bits_equal(got, s)


def test_offtree_too_high_candidate_caught(grid5):
    """A split candidate of the root that does NOT win, stored one ulp too high: the root's
    first minimum is unchanged, so the on-tree walk alone passes; the candidate's own
    re-derivation (offtree) fails."""
    lat, s, args, _, _ = _lane0(grid5)
    r = T.rederive(lat, lambda x: s[x.astype(np.int64)], *args)
    assert r["candidates"] > 2 * r["nodes"]
    left = set(int(x) for x in np.asarray(r["leaves"]))
    best = min(np.float32(s[c1] + s[c2]) for c1, c2 in _root_candidates(lat))
    loser = next(c1 for c1, c2 in _root_candidates(lat)
                 if np.float32(s[c1] + s[c2]) > best and c1 not in left)
    t = s.copy()
    t[loser] = np.nextafter(t[loser], np.float32(np.inf))
    g = lambda x: t[x.astype(np.int64)]  # noqa: E731
    T.rederive(lat, g, *args, offtree=False)
    with pytest.raises(T.TreeMismatch, match="split candidate"):
        T.rederive(lat, g, *args)


def test_offtree_flipped_argmin_caught(grid5):
    """The verdict's case: the root's WINNING child stored too high, and every cell above it
    recomputed consistently from that value (as a sweep that read the wrong value would
    have): the root's argmin flips to a worse split and the on-tree walk reproduces the
    flipped tree bit for bit; the off-tree re-derivation of the too-high child fails."""
    lat, s, args, mtr, utr = _lane0(grid5)
    r0 = T.rederive(lat, lambda x: s[x.astype(np.int64)], *args)
    sums = [(np.float32(s[c1] + s[c2]), c1) for c1, c2 in _root_candidates(lat)]
    best = min(v for v, _ in sums)
    win = next(c1 for v, c1 in sums if v == best)
    t = s.copy()
    t[win] = t[win] + np.float32(1e4)
    lev = lat.digit_array(np.arange(s.size))
    lvl = np.zeros(s.size, np.int64)
    for i, g in enumerate(lat.gp):
        lv = np.array([len(T.IUPAC[x]) - 1 for x in O._PERM[g]])
        lvl += lv[lev[:, i]]
    a, b, c = args[4:]
    for L in range(int(lvl[win]) + 1, int(lvl.max()) + 1):
        cells = np.nonzero(lvl == L)[0]
        t[cells] = T.local_values(lat, cells, mtr[cells], utr[cells], lambda x: t[x.astype(np.int64)], a, b, c)
    g = lambda x: t[x.astype(np.int64)]  # noqa: E731
    r1 = T.rederive(lat, g, *args, offtree=False)  # consistent above the bad cell: passes
    assert not np.array_equal(r1["leaves"], r0["leaves"])  # ... with a different tree
    with pytest.raises(T.TreeMismatch, match="split candidate"):
        T.rederive(lat, g, *args)

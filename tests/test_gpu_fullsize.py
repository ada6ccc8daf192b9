"""Parity at the benchmark's full size (BASELINE configs[3]: synthetic 9-mer counts,
NNNNMNNNN = 7.69e9 cells), where the oracle would need days: size-independent
properties of the optimal partition and of the CV roots, checked on the GPU result.

* the partition covers every k-mer exactly once and its counts sum to the totals
  (the reference CLI's own sanity checks, cli.py:289-292);
* the root score equals the sum of the leaves' terms (penalty + -2LL per leaf, float64
  here; float32 sums along the tree on the GPU) -- the value the DP minimised;
* optimality sanity: it is no worse than the one-pattern and the all-k-mers partitions;
* the CV root train value is non-decreasing in the penalty (min over partitions of
  LL + c |P|).
The backtrack itself re-derives every node's decision from the stored scores and
fails with KP_E_PARITY unless each one reproduces its float32 score bit for bit.
Independently of it, the HOST re-derives every optimal tree (oracle/treecheck.py: the
reference's recurrence with the C library's logs) from the GPU's stored scores and pins,
bit for bit, the fit's root and partition and the root train / test values of every lane
of the 9-mer grid (125) and of two folds of the 11-mer grid (98): the numbers that reach
the CVfile.  Every cell of embedded sub-lattices is compared with the oracle as well.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GEN_PAT = "NNNNMNNNN"


@pytest.fixture(scope="module")
def counts():
    import bench
    kmers, M, U = bench.synthetic_counts(GEN_PAT, seed=9)
    return kmers, M, U


def _leaf_term(m, u, alpha, beta, pen):
    """The reference's per-pattern score: level 0 (one k-mer) uses xlogy/xlog1py and the
    -2(a+b)+c order (Fit :26-29); wider patterns c + (-2M)log p + (-2U)log(1-p) (Fit :56-61)."""
    p = (m + alpha) / (((m + u) + alpha) + beta)
    a = 0.0 if m == 0 else m * math.log(p)
    b = 0.0 if u == 0 else u * math.log1p(-p)
    return -2.0 * (a + b) + pen


def _wide_term(m, u, alpha, beta, pen):
    p = (m + alpha) / (((m + u) + alpha) + beta)
    s = pen
    if m > 0:
        s += (-2.0 * m) * math.log(p)
    if u > 0:
        s += (-2.0 * u) * math.log(1.0 - p)
    return s


def _fit_tree_rederived(gen_pat, kmers, M, U, alpha, beta, pen, score, names):
    """The fit's root score and its partition in backtrack order (Fit :17-24, :121), bit for
    bit: the host re-derives the whole optimal tree from the GPU's stored scores of the fit
    lane (oracle/treecheck.py: the reference's scan order, first minimum, the C library's
    logs; test counts zero)."""
    from kmerpapa_amd import engine
    from oracle import treecheck as T
    plan = engine.get_plan(engine.visible_devices()[0], gen_pat, 0)  # the plan the fit ran on
    lat = T.Lattice(gen_pat)
    assert np.array_equal(engine.kmer_order(gen_pat, kmers), np.arange(lat.n_kmers))  # k-mer index order
    z = np.zeros(lat.n_kmers, np.int64)
    r = T.rederive(lat, lambda cells: plan.gather_cells(0, cells), np.asarray(M, np.int64), np.asarray(U, np.int64),
                   z, z, alpha, beta, pen)
    assert r["root_train"].view(np.uint32) == np.float32(score).view(np.uint32)
    assert [lat.pattern(c) for c in r["leaves"]] == list(names)
    return r


def test_9mer_full_fit_properties(counts):
    from kmerpapa_amd import engine
    from kmerpapa_amd.algorithms import bottum_up_array_w_numba as fitm
    from kmerpapa_amd.pattern_utils import generality, matches
    kmers, M, U = counts
    ctx = {k: (int(m), int(u)) for k, m, u in zip(kmers, M, U)}
    nm, nu = int(M.sum()), int(U.sum())
    my = nm / (nm + nu)
    alpha, pen = 2.0, 5.0
    beta = (alpha * (1.0 - my)) / my

    class A:
        verbosity = 0
    score, Mr, Ur, names = fitm.pattern_partition_bottom_up(GEN_PAT, ctx, alpha, beta, pen, A, nm, nu)
    assert (int(Mr), int(Ur)) == (nm, nu)
    n_kmers = generality(GEN_PAT)
    assert sum(generality(x) for x in names) == n_kmers
    cover = np.zeros(n_kmers, np.int64)
    total = 0.0
    for name in names:
        ks = list(matches(name))
        idx = engine.kmer_order(GEN_PAT, ks)
        cover[idx] += 1
        m, u = int(M[idx].sum()), int(U[idx].sum())
        total += _leaf_term(m, u, alpha, beta, pen) if len(ks) == 1 else _wide_term(m, u, alpha, beta, pen)
    assert (cover == 1).all()
    assert 50 < len(names) < n_kmers
    assert abs(float(score) - total) <= 2e-6 * abs(total)
    _fit_tree_rederived(GEN_PAT, kmers, M, U, alpha, beta, pen, score, names)
    one = _wide_term(nm, nu, alpha, beta, pen)
    every = sum(_leaf_term(int(m), int(u), alpha, beta, pen) for m, u in zip(M, U))
    assert float(score) <= one * (1 + 1e-6) and float(score) <= every * (1 + 1e-6)


def test_9mer_full_cv_roots_monotone_in_penalty(counts):
    from kmerpapa_amd import engine
    from kmerpapa_amd.CV_tools import fold_tables
    from kmerpapa_amd.pattern_utils import generality
    from kmerpapa_amd.score_utils import get_betas
    kmers, M, U = counts
    ctx = {k: (int(m), int(u)) for k, m, u in zip(kmers, M, U)}
    contexts, Mf, Uf = fold_tables(ctx, 5, np.random.RandomState(1), np.uint32)
    assert (Mf.sum(axis=1) == np.array([ctx[c][0] for c in contexts])).all()  # fold split conserves counts
    Mk, Uk = engine.counts_in_kmer_order(GEN_PAT, contexts, Mf, Uf, generality(GEN_PAT), np.uint32)
    M_sum, U_sum = Mk.sum(axis=0, dtype=np.uint64), Uk.sum(axis=0, dtype=np.uint64)
    betas = get_betas(1.0, M_sum.sum() - M_sum, U_sum.sum() - U_sum)
    pens = [3.0, 4.0, 5.0, 6.0, 7.0]
    plan = engine.get_plan(engine.visible_devices()[0], GEN_PAT, 0)
    plan.set_counts(Mk, Uk)
    rt, re, nl = plan.run([(2, 1.0, float(betas[2]), pens)])
    rt = np.asarray(rt, np.float64)
    assert np.isfinite(rt).all() and (np.diff(rt) >= -1e-6 * np.abs(rt[1:])).all()
    assert (np.diff(np.asarray(nl, np.int64)) <= 0).all()  # fewer (or equal) patterns as c grows
    assert np.isfinite(np.asarray(re)).all()


# ---------------------------------------------------------------------------------------
# Full-size CV lanes pinned cell by cell: a cell's DP value depends only on its own
# sub-lattice (the k-mers it matches, their fold counts, alpha, beta_f and c: CV :26-78),
# so every cell of a sub-pattern S embedded in NNNNMNNNN must equal the oracle's value of
# the same pattern in a run on the lattice of S alone, given the FULL run's fold counts
# and betas.  The oracle runs one fold as a 2-column table [fold f, all other folds]:
# train = sum of columns - column 0 = all data - fold f (CV :22-24, :56-59), exactly the
# full run's train counts of fold f, at a fifth of the work of all five folds.
# ---------------------------------------------------------------------------------------

@pytest.fixture(scope="module")
def cv_split(counts):
    from kmerpapa_amd import engine
    from kmerpapa_amd.CV_tools import fold_tables
    from kmerpapa_amd.pattern_utils import generality
    kmers, M, U = counts
    ctx = {k: (int(m), int(u)) for k, m, u in zip(kmers, M, U)}
    contexts, Mf, Uf = fold_tables(ctx, 5, np.random.RandomState(1), np.uint32)
    Mk, Uk = engine.counts_in_kmer_order(GEN_PAT, contexts, Mf, Uf, generality(GEN_PAT), np.uint32)
    msum, usum = Mk.sum(axis=0, dtype=np.uint64), Uk.sum(axis=0, dtype=np.uint64)
    return {"contexts": contexts, "Mf": Mf, "Uf": Uf, "Mk": Mk, "Uk": Uk,
            "mtr": msum.sum() - msum, "utr": usum.sum() - usum}


def _embedded_cells(full, sub):
    """Full-lattice index of every cell of the sub-lattice ``sub`` (in the sub-lattice's own
    index order), from the oracle's IUPAC tables (mixed radix, position 0 fastest)."""
    from oracle.oracle import _PERM
    n = 1
    for g in sub:
        n *= len(_PERM[g])
    x = np.arange(n, dtype=np.int64)
    out = np.zeros(n, np.uint64)
    w = 1
    for g, s in zip(full, sub):
        r = len(_PERM[s])
        lut = np.array([_PERM[g].index(ch) for ch in _PERM[s]], np.uint64)
        out += lut[x % r] * np.uint64(w)
        x //= r
        w *= len(_PERM[g])
    return out


IUPAC = {"A": "A", "C": "C", "G": "G", "T": "T", "R": "AG", "Y": "CT", "S": "CG", "W": "AT", "K": "GT",
         "M": "AC", "B": "CGT", "D": "AGT", "H": "ACT", "V": "ACG", "N": "ACGT"}

SUBS = ["ANNNMNNNA",   # low in the index space
        "AANNMNNNV"]   # last position V: cells at index >= 13/15 * npat > 2^32


@pytest.mark.timeout(1200)
def test_9mer_full_cv_lane_embedded_sublattices_vs_oracle(cv_split):
    """One 5-lane (alpha, fold) group of the headline CV pass over the whole 9-mer lattice
    (7.69e9 cells, default block: 6 high positions, 17 launches): every cell of two
    embedded sub-lattices (ANNNMNNNA: 3.4e7 cells; AANNMNNNV: 1.6e7 cells at cell indices
    and score-buffer offsets past 2^32) equals the oracle bit for bit in all 5 lanes."""
    from kmerpapa_amd import engine
    from kmerpapa_amd.score_utils import get_betas
    from oracle import oracle as O
    from tests.fixtures import bits_equal
    sp = cv_split
    alpha, fold, pens = 2.0, 3, [3.0, 4.0, 5.0, 6.0, 7.0]
    betas = get_betas(alpha, sp["mtr"], sp["utr"])
    plan = engine.get_plan(engine.visible_devices()[0], GEN_PAT, 0)
    assert plan.info["npat"] == 7688671875 and plan.info["high_levels"] > 1
    plan.set_counts(sp["Mk"], sp["Uk"])
    plan.run([(fold, alpha, float(betas[fold]), pens)])
    assert plan.stats()["dp_launches"] == 17
    bf = float(betas[fold])
    for sub in SUBS:
        keep = [i for i, c in enumerate(sp["contexts"]) if all(c[j] in IUPAC[ch] for j, ch in enumerate(sub))]
        ctxs = [sp["contexts"][i] for i in keep]
        mf, uf = sp["Mf"][keep], sp["Uf"][keep]
        m2 = np.stack([mf[:, fold], mf.sum(axis=1) - mf[:, fold]], axis=1)
        u2 = np.stack([uf[:, fold], uf.sum(axis=1) - uf[:, fold]], axis=1)
        cells = _embedded_cells(GEN_PAT, sub)
        assert cells.size == O.npat(sub)
        if sub == "AANNMNNNV":
            assert (cells > 2 ** 32).sum() > cells.size // 4  # last digit M or V: index > 2^32
        for j, c in enumerate(pens):
            ref = O.cv_pass(sub, ctxs, m2, u2, alpha, [bf, bf], c, 32, threads=_threads())
            got = plan.gather_cells(j, cells)
            assert bits_equal(got, ref["score"][:, 0]), (sub, c, int(np.sum(got.view(np.uint32) !=
                                                                             ref["score"][:, 0].view(np.uint32))))
            del ref


def _threads():
    import os
    n = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except AttributeError:
        pass
    return max(1, min(n, 16))


def _leaf_kmers(gen_pat, leaves):
    """(leaf number, k-mer index) of every k-mer every leaf cell matches, vectorised: the
    leaf cells are decoded to IUPAC letters (oracle tables) and expanded position by
    position; k-mer index = KmerEnumeration order (position 0 fastest, digit = rank of the
    nucleotide among the general code's nucleotides, alphabetical)."""
    from oracle.oracle import _PERM
    x = np.asarray(leaves, np.int64).copy()
    codes = []
    for g in gen_pat:
        r = len(_PERM[g])
        codes.append(x % r)
        x //= r
    leaf = np.arange(len(leaves), dtype=np.int64)
    kidx = np.zeros(len(leaves), np.int64)
    w = 1
    for i, g in enumerate(gen_pat):
        nucs = IUPAC[g]
        # per sub-code of g: its nucleotides' digits (padded with -1)
        tab = np.full((len(_PERM[g]), 4), -1, np.int64)
        size = np.zeros(len(_PERM[g]), np.int64)
        for d, ch in enumerate(_PERM[g]):
            ds = [nucs.index(n) for n in IUPAC[ch]]
            tab[d, :len(ds)] = ds
            size[d] = len(ds)
        code_i = codes[i][leaf]
        rep = size[code_i]
        start = np.cumsum(rep) - rep
        leaf = np.repeat(leaf, rep)
        kidx = np.repeat(kidx, rep)
        j = np.arange(leaf.size) - np.repeat(start, rep)
        kidx = kidx + tab[codes[i][leaf], j] * w
        w *= len(nucs)
    return leaf, kidx


def _tree_check_pass(plan, lat, groups, Mk, Uk, rt, re, nl):
    """Every lane of the pass just run (``groups``, lanes group-major): the host walks the
    lane's optimal tree top-down from the GPU's stored train scores (oracle/treecheck.py:
    split candidates in the reference's scan order with the first minimum winning, the
    single-pattern term from the host C library's log in CV :56-78's operation order, the
    k-mer terms of CV :15-20) and requires every node's stored score to be the re-derived
    one bit for bit; the root's train and test values returned by the pass must equal the
    re-derived root (test = the float32 sums test[c1] + test[c2] along the tree, CV :47,
    :158-163) and kp_fit_leaves the re-derived leaves in backtrack order.  The leaves
    must also cover every k-mer exactly once.  Returns the number of tree nodes checked."""
    from oracle import treecheck as T
    Mall, Uall = Mk.sum(axis=1), Uk.sum(axis=1)
    lane, nodes = 0, 0
    for fold, a, b, pens in groups:
        mte, ute = Mk[:, fold], Uk[:, fold]
        for c in pens:
            r = T.rederive(lat, lambda cells, j=lane: plan.gather_cells(j, cells), Mall - mte, Uall - ute,
                           mte, ute, a, float(b), c)
            where = (fold, a, c)
            assert r["root_train"].view(np.uint32) == np.float32(rt[lane]).view(np.uint32), where
            assert r["root_test"].view(np.uint32) == np.float32(re[lane]).view(np.uint32), where
            leaves = plan.leaves(lane)
            assert leaves.size == int(nl[lane]) and np.array_equal(leaves, r["leaves"]), where
            _, kidx = _leaf_kmers(lat.gp, leaves)
            assert kidx.size == lat.n_kmers and (np.bincount(kidx, minlength=lat.n_kmers) == 1).all(), where
            nodes += r["nodes"]
            lane += 1
    return nodes


@pytest.mark.timeout(1200)
def test_9mer_full_cv_all_125_lanes_tree_rederived(cv_split):
    """The whole 5x5x5 headline grid (25 passes of 5 lanes over 7.69e9 cells): every lane's
    root train and root test -- the numbers that reach the CVfile -- pinned bit for bit by
    re-deriving the lane's whole optimal tree on the host from the GPU's stored scores
    (_tree_check_pass)."""
    from kmerpapa_amd import engine
    from kmerpapa_amd.score_utils import get_betas
    from oracle import treecheck as T
    sp = cv_split
    alphas, pens, nf = [0.5, 1.0, 2.0, 5.0, 10.0], [3.0, 4.0, 5.0, 6.0, 7.0], 5
    plan = engine.get_plan(engine.visible_devices()[0], GEN_PAT, 0)
    plan.set_counts(sp["Mk"], sp["Uk"])
    lat = T.Lattice(GEN_PAT)
    assert lat.n_kmers == plan.info["n_kmers"]
    Mk = sp["Mk"].astype(np.int64)
    Uk = sp["Uk"].astype(np.int64)
    lanes = nodes = 0
    for a in alphas:
        betas = get_betas(a, sp["mtr"], sp["utr"])
        for f in range(nf):
            grp = [(f, a, float(betas[f]), pens)]
            rt, re, nl = plan.run(grp)
            nodes += _tree_check_pass(plan, lat, grp, Mk, Uk, rt, re, nl)
            lanes += len(pens)
    assert lanes == 125
    print(f"9-mer grid: {lanes} lanes, {nodes} tree nodes re-derived")


@pytest.mark.timeout(1500)
def test_11mer_full_two_folds_all_lanes_tree_rederived():
    """BASELINE configs[4] at full size (ANNNNMNNNNA, 7.69e9 cells, 10 folds, 7x7 grid):
    folds 0 and 6, all 49 lanes each, run as the passes engine.plan_passes cuts the grid
    into (5-lane fold pieces, five mixed two-alpha pieces and one 4-lane piece per fold):
    every lane's root train, root test and partition pinned by the host tree re-derivation."""
    from kmerpapa_amd import engine
    from kmerpapa_amd.CV_tools import fold_tables
    from kmerpapa_amd.pattern_utils import generality
    from kmerpapa_amd.score_utils import get_betas
    from oracle import treecheck as T
    import bench
    gp, nf = "ANNNNMNNNNA", 10
    kmers, M, U = bench.synthetic_counts(gp, seed=9)
    ctx = {k: (int(m), int(u)) for k, m, u in zip(kmers, M, U)}
    contexts, Mf, Uf = fold_tables(ctx, nf, np.random.RandomState(1), np.uint32)
    Mk, Uk = engine.counts_in_kmer_order(gp, contexts, Mf, Uf, generality(gp), np.uint32)
    ms, us = Mf.sum(axis=0, dtype=np.uint64), Uf.sum(axis=0, dtype=np.uint64)
    grid = []
    for a in ALPHAS11:
        betas = get_betas(a, ms.sum() - ms, us.sum() - us)
        grid += [(f, a, float(betas[f]), PENS11) for f in range(nf)]
    engine.release_all()
    plan = engine.get_plan(engine.visible_devices()[0], gp, 0)
    plan.set_counts(Mk, Uk)
    width = plan.info["lanes_per_workgroup"]
    passes, _ = engine.plan_passes([g for g in grid if g[0] in (0, 6)], width, width)
    assert sum(1 for p in passes if len({g[1] for g in p}) == 2) == 10  # mixed pieces
    lat = T.Lattice(gp)
    Mk, Uk = Mk.astype(np.int64), Uk.astype(np.int64)
    lanes = nodes = 0
    for pas in passes:
        rt, re, nl = plan.run(pas)
        nodes += _tree_check_pass(plan, lat, pas, Mk, Uk, rt, re, nl)
        lanes += sum(len(g[3]) for g in pas)
    assert lanes == 98
    print(f"11-mer folds 0, 6: {lanes} lanes, {nodes} tree nodes re-derived")
    engine.release_all()


@pytest.mark.timeout(900)
def test_9mer_full_lane_buffer_grow_sequence(cv_split):
    """The product's allocation sequence at full size: a fresh plan reserves 2 lanes
    (61 GB of score rows), runs a 2-lane pass, grows to 5 lanes (154 GB: the 2-lane buffer
    is freed and a larger one allocated -- the sequence that made the stream-ordered pool
    return memory not holding what was written), runs a 5-lane pass; after
    each pass every cell of the embedded sub-lattice AANNMNNNV (offsets past 2^32) equals
    the oracle in the first and last lane."""
    from kmerpapa_amd import engine
    from kmerpapa_amd.score_utils import get_betas
    from oracle import oracle as O
    from tests.fixtures import bits_equal
    sp = cv_split
    engine.release_all()
    alpha, fold = 5.0, 1
    bf = float(get_betas(alpha, sp["mtr"], sp["utr"])[fold])
    sub = "AANNMNNNV"
    keep = [i for i, c in enumerate(sp["contexts"]) if all(c[j] in IUPAC[ch] for j, ch in enumerate(sub))]
    ctxs = [sp["contexts"][i] for i in keep]
    mf, uf = sp["Mf"][keep], sp["Uf"][keep]
    m2 = np.stack([mf[:, fold], mf.sum(axis=1) - mf[:, fold]], axis=1)
    u2 = np.stack([uf[:, fold], uf.sum(axis=1) - uf[:, fold]], axis=1)
    cells = _embedded_cells(GEN_PAT, sub)
    ref = {}
    plan = engine.Plan(engine.get_device(engine.visible_devices()[0]), GEN_PAT, 0)
    try:
        plan.set_counts(sp["Mk"], sp["Uk"])
        for pens in ([3.5, 6.5], [3.0, 4.0, 5.0, 6.0, 7.0]):
            plan.reserve(len(pens))
            plan.run([(fold, alpha, bf, pens)])
            for j in (0, len(pens) - 1):
                c = pens[j]
                if c not in ref:
                    ref[c] = O.cv_pass(sub, ctxs, m2, u2, alpha, [bf, bf], c, 32, threads=_threads())["score"][:, 0]
                assert bits_equal(plan.gather_cells(j, cells), ref[c]), (len(pens), c)
    finally:
        plan.close()


# ---------------------------------------------------------------------------------------
# The same embedded-sub-lattice check through the product's own asynchronous count path:
# the fold split drawn fold by fold on a host thread (CV_tools.fold_feed -> engine.FoldFeed),
# the all-data counts uploaded first and the fold's table filled on the plan's count stream
# (kp_counts_begin / kp_counts_fold), the pass run by engine.run_groups -- exactly as the
# CV driver runs it (bottum_up_array_penalty_plus_pseudo_CV.cv_roots).
# ---------------------------------------------------------------------------------------

def _fed_pass_vs_oracle(gen_pat, ctx, nf, groups, subs):
    """Run ``groups`` (one fold, at most one workgroup of lanes) over the whole lattice of
    ``gen_pat`` through the fold feed; then every cell of each embedded sub-lattice in
    ``subs`` equals the oracle's run on that sub-lattice with the full run's fold counts and
    each lane's own (alpha, beta, c), bit for bit."""
    from kmerpapa_amd import engine
    from kmerpapa_amd.CV_tools import fold_feed, fold_tables
    from oracle import oracle as O
    from tests.fixtures import bits_equal
    fold = groups[0][0]
    assert all(g[0] == fold for g in groups)
    dev = engine.visible_devices()[0]
    engine.release_all()
    feed, pr = fold_feed(ctx, gen_pat, nf, np.random.RandomState(1), np.uint32)
    try:
        engine.run_groups(gen_pat, feed, None, groups, devices=[dev])
    finally:
        pr.join()
    plan = engine.get_plan(dev, gen_pat, 0)
    assert plan.stats()["units"] == plan.info["npat"] * sum(len(g[3]) for g in groups)  # one pass, every lane
    # the oracle's inputs: the same seeded split drawn at once (sorted-context order); the
    # feed's fold-f table (k-mer order) must hold exactly these counts
    contexts, Mf, Uf = fold_tables(ctx, nf, np.random.RandomState(1), np.uint32)
    idx = engine.kmer_order(gen_pat, contexts)
    mk, uk = feed.get(fold)
    assert np.array_equal(mk[idx], Mf[:, fold]) and np.array_equal(uk[idx], Uf[:, fold])
    lanes = [(g[1], g[2], c) for g in groups for c in g[3]]
    for sub in subs:
        keep = [i for i, c in enumerate(contexts) if all(c[j] in IUPAC[ch] for j, ch in enumerate(sub))]
        ctxs = [contexts[i] for i in keep]
        mf, uf = Mf[keep], Uf[keep]
        m2 = np.stack([mf[:, fold], mf.sum(axis=1) - mf[:, fold]], axis=1)
        u2 = np.stack([uf[:, fold], uf.sum(axis=1) - uf[:, fold]], axis=1)
        cells = _embedded_cells(gen_pat, sub)
        assert cells.size == O.npat(sub)
        for lane, (a, b, c) in enumerate(lanes):
            ref = O.cv_pass(sub, ctxs, m2, u2, a, [b, b], c, 32, threads=_threads())
            got = plan.gather_cells(lane, cells)
            assert bits_equal(got, ref["score"][:, 0]), (sub, lane, a, c, int(np.sum(
                got.view(np.uint32) != ref["score"][:, 0].view(np.uint32))))
            del ref
    return plan


@pytest.mark.timeout(1200)
def test_9mer_full_fold0_group_fold_feed_vs_oracle(counts):
    """A second (alpha, fold) group of the headline pass, fold 0 (the first drawn, which
    every share's first pass waits for), through the fold feed: every cell of ANNNMNNNA and
    AANNMNNNV in all 5 lanes equals the oracle."""
    from kmerpapa_amd.score_utils import get_betas
    kmers, M, U = counts
    ctx = {k: (int(m), int(u)) for k, m, u in zip(kmers, M, U)}
    from kmerpapa_amd.CV_tools import fold_tables
    _, Mf, Uf = fold_tables(ctx, 5, np.random.RandomState(1), np.uint32)
    ms, us = Mf.sum(axis=0, dtype=np.uint64), Uf.sum(axis=0, dtype=np.uint64)
    alpha = 0.5
    b0 = float(get_betas(alpha, ms.sum() - ms, us.sum() - us)[0])
    plan = _fed_pass_vs_oracle(GEN_PAT, ctx, 5, [(0, alpha, b0, [3.0, 4.0, 5.0, 6.0, 7.0])], SUBS)
    assert plan.stats()["dp_launches"] == 17
    from kmerpapa_amd import engine
    engine.release_all()


SUBS11 = ["AANNNMNNNAA",   # low in the index space (3.4e7 cells)
          "AAANNMNNNVA"]   # V at the last ambiguous position: cells past 2^32 (1.6e7 cells)
ALPHAS11 = [0.5, 1.0, 2.0, 3.0, 5.0, 7.0, 10.0]
PENS11 = [2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 8.0]


@pytest.mark.timeout(1500)
def test_11mer_full_mixed_fold_piece_fold_feed_vs_oracle():
    """BASELINE configs[4] at full size (ANNNNMNNNNA, 7.69e9 cells, 10 folds): one MIXED
    5-lane fold piece of the 7x7 grid exactly as engine.plan_passes cuts it (fold 6: alpha
    3.0 with c = 6, 7, 8 and alpha 5.0 with c = 2, 3 in one workgroup, a second rate and
    pair of logs per cell for the last two lanes), fed fold by fold as the CV driver does:
    every cell of AANNNMNNNAA and AAANNMNNNVA (offsets past 2^32) in all 5 lanes equals the
    oracle run with that lane's own alpha and beta."""
    from kmerpapa_amd import engine
    from kmerpapa_amd.CV_tools import fold_tables
    from kmerpapa_amd.score_utils import get_betas
    import bench
    gp, nf, fold = "ANNNNMNNNNA", 10, 6
    kmers, M, U = bench.synthetic_counts(gp, seed=9)
    ctx = {k: (int(m), int(u)) for k, m, u in zip(kmers, M, U)}
    _, Mf, Uf = fold_tables(ctx, nf, np.random.RandomState(1), np.uint32)
    ms, us = Mf.sum(axis=0, dtype=np.uint64), Uf.sum(axis=0, dtype=np.uint64)
    betas = {a: get_betas(a, ms.sum() - ms, us.sum() - us) for a in ALPHAS11}
    grid = [(f, a, float(betas[a][f]), PENS11) for a in ALPHAS11 for f in range(nf)]
    piece = [(fold, 3.0, float(betas[3.0][fold]), [6.0, 7.0, 8.0]), (fold, 5.0, float(betas[5.0][fold]), [2.0, 3.0])]
    passes, _ = engine.plan_passes(grid, 7, 5)
    assert [tuple((g[0], g[1], g[2], list(g[3])) for g in p) for p in passes].count(
        tuple((g[0], g[1], g[2], list(g[3])) for g in piece)) == 1  # a pass of the grid's own plan
    assert engine.device_groups(piece, 5) == [(0, 5, 2)]  # one workgroup, last 2 lanes on the second alpha
    _fed_pass_vs_oracle(gp, ctx, nf, piece, SUBS11)
    engine.release_all()

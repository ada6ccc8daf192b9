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


def _tree_check_pass(plan, lat, groups, Mk, Uk, rt, re, nl, offtree=(), stats=None):
    """Every lane of the pass just run (``groups``, lanes group-major): the host walks the
    lane's optimal tree top-down from the GPU's stored train scores (oracle/treecheck.py:
    split candidates in the reference's scan order with the first minimum winning, the
    single-pattern term from the host C library's log in CV :56-78's operation order, the
    k-mer terms of CV :15-20) and requires every node's stored score to be the re-derived
    one bit for bit; the root's train and test values returned by the pass must equal the
    re-derived root (test = the float32 sums test[c1] + test[c2] along the tree, CV :47,
    :158-163) and kp_fit_leaves the re-derived leaves in backtrack order.  The leaves
    must also cover every k-mer exactly once.  Lanes in ``offtree`` also re-derive every
    split candidate of every tree node one level down (treecheck ``offtree``: the cells the
    tree's first minima were taken against).  Returns the number of tree nodes checked;
    ``stats`` (a dict) accumulates nodes, candidates and lanes."""
    from oracle import treecheck as T
    Mall, Uall = Mk.sum(axis=1), Uk.sum(axis=1)
    lane, nodes = 0, 0
    for fold, a, b, pens in groups:
        mte, ute = Mk[:, fold], Uk[:, fold]
        for c in pens:
            r = T.rederive(lat, lambda cells, j=lane: plan.gather_cells(j, cells), Mall - mte, Uall - ute,
                           mte, ute, a, float(b), c, offtree=lane in offtree)
            if stats is not None:
                stats["nodes"] = stats.get("nodes", 0) + r["nodes"]
                stats["candidates"] = stats.get("candidates", 0) + r["candidates"]
                stats["lanes"] = stats.get("lanes", 0) + 1
                stats["offtree_lanes"] = stats.get("offtree_lanes", 0) + (lane in offtree)
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


_GRID9 = {}  # (fold, alpha, c) -> (root train, root test, leaves) of the one-GPU 5x5x5 run
ALPHAS9, PENS9 = [0.5, 1.0, 2.0, 5.0, 10.0], [3.0, 4.0, 5.0, 6.0, 7.0]


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
            for j, c in enumerate(pens):  # the one-GPU job's roots, for the 8-rank shares below
                _GRID9[(f, a, c)] = (rt[j], re[j], nl[j])
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


# ---------------------------------------------------------------------------------------
# The 8-GPU job's own passes at full size.  An 8-rank CV job (torchrun, one process per GPU;
# the in-job replacement for the reference's README fan-out, README.md:39-51) gives every
# rank a lane-granular share of the grid (shard.rank_groups) and runs it as
# engine.plan_passes cuts it with pass_cap = one workgroup + 1 lane: at 9-mers every
# 16-lane share is [5], [5], [5 + 1], the last a packed pass of two folds whose odd lane
# reads another fold's count-table row in the same launches.  Here one GPU runs exactly
# those passes, rank after rank; every lane of ranks 0 and 7 is tree-checked with the
# off-tree candidates, one packed odd lane is compared cell by cell over the WHOLE lattice
# with the oracle, and shard.unshard of the eight ranks' roots must equal the one-GPU
# job's roots bit for bit.
# ---------------------------------------------------------------------------------------

def _kmer_cells(lat):
    """Cell index of every k-mer (k-mer index order): digit = position of the k-mer's
    nucleotide in perm_code of the general code (oracle tables)."""
    from oracle.oracle import _PERM
    cells = np.zeros(lat.n_kmers, np.uint64)
    for i, g in enumerate(lat.gp):
        lut = np.array([_PERM[g].index(n) for n in IUPAC[g]], np.uint64)
        cells += lut[lat.kdig[i]] * np.uint64(lat.cw[i])
    return cells


def _full_lane_vs_oracle(plan, lane, lat, mtr, utr, alpha, beta, c):
    """Every cell of ``lane`` of the plan's last pass against the oracle's memory-lean run
    of that one lane over the whole lattice (oracle.cv_lane: the kpo_cv recurrence, train
    counts only, 12 B/cell; the k-mers' train counts = all data - the lane's fold), read
    back in chunks of 2^27 cells.  Returns the number of cells compared."""
    from oracle import oracle as O
    from tests.fixtures import bits_equal
    ref = O.cv_lane(lat.gp, _kmer_cells(lat), mtr, utr, alpha, beta, c, 32, threads=_threads())
    n = ref.size
    assert n == plan.info["npat"]
    step = 1 << 27
    for i0 in range(0, n, step):
        i1 = min(n, i0 + step)
        got = plan.gather_cells(lane, np.arange(i0, i1, dtype=np.uint64))
        if not bits_equal(got, ref[i0:i1]):
            bad = np.nonzero((got.view(np.uint32) != ref[i0:i1].view(np.uint32)) &
                             ~(np.isnan(got) & np.isnan(ref[i0:i1])))[0]
            raise AssertionError(f"lane {lane}: {bad.size} cells of [{i0}, {i1}) differ, first {i0 + int(bad[0])} "
                                 f"({lat.pattern(i0 + int(bad[0]))}): {got[bad[0]]!r} vs {ref[i0 + bad[0]]!r}")
    del ref
    return n


def _grid_cv_order(mtr, utr, alphas, pens, nf):
    """The CV driver's groups (alpha-major, folds in shard.fold_order, CV :138-145 of the
    drop-in), with float betas."""
    from kmerpapa_amd.score_utils import get_betas
    from kmerpapa_amd.shard import fold_order
    grid = []
    for a in alphas:
        betas = get_betas(a, mtr, utr)
        grid += [(f, a, float(betas[f]), list(pens)) for f in fold_order(nf)]
    return grid


@pytest.mark.timeout(1500)
def test_9mer_8rank_shares_pinned_full_size(cv_split):
    """BASELINE configs[3] as the 8-GPU job runs it: each rank's share of the 5x5x5 grid as
    its own passes ([5], [5], [5 + 1] or [5], [5], [5]), one rank after the other on this
    GPU.  Ranks 0, 4 and 7 (a [5 + 1] pass of two folds, one of two alphas of the same fold,
    a 15-lane share): every lane's root train / test and partition re-derived on the host
    with every split candidate of every tree node re-derived one level down (47 lanes); rank 0's packed odd
    lane (another fold's single lane beside a 5-lane group) equal to the oracle in all
    7.69e9 cells; the eight ranks' roots unsharded equal the one-GPU job's bit for bit."""
    from kmerpapa_amd import engine, shard
    from oracle import treecheck as T
    sp = cv_split
    grid = _grid_cv_order(sp["mtr"], sp["utr"], ALPHAS9, PENS9, 5)
    dev = engine.visible_devices()[0]
    plan = engine.get_plan(dev, GEN_PAT, 0)
    plan.set_counts(sp["Mk"], sp["Uk"])
    width = plan.info["lanes_per_workgroup"]
    assert width == 5
    if len(_GRID9) < 125:  # (the 125-lane test did not run first) the one-GPU job's passes
        rt, re, nl = engine.run_groups(GEN_PAT, sp["Mk"], sp["Uk"], grid, devices=[dev])
        lane = 0
        for f, a, b, pens in grid:
            for c in pens:
                _GRID9[(f, a, c)] = (rt[lane], re[lane], nl[lane])
                lane += 1
    lat = T.Lattice(GEN_PAT)
    Mk, Uk = sp["Mk"].astype(np.int64), sp["Uk"].astype(np.int64)
    Mall, Uall = Mk.sum(axis=1), Uk.sum(axis=1)
    stats, parts, full_cells = {}, [], 0
    for r in range(8):
        mine = shard.rank_groups(grid, r, 8)
        passes, order = engine.plan_passes(mine, engine.pass_cap(mine, plan.require_lanes(), width), width)
        shape = [[len(g[3]) for g in pas] for pas in passes]
        if r == 0:
            assert shape == [[5], [5], [5, 1]] and len({g[0] for g in passes[-1]}) == 2, shape
        if r == 4:
            assert shape == [[5], [5], [5, 1]] and len({g[0] for g in passes[-1]}) == 1, shape
        if r == 7:
            assert shape == [[5], [5], [5]], shape
        outs = []
        for pas in passes:
            rt, re, nl = plan.run(pas)
            outs.append((rt, re, nl))
            if r in (0, 4, 7):
                nlanes = sum(len(g[3]) for g in pas)
                _tree_check_pass(plan, lat, pas, Mk, Uk, rt, re, nl, offtree=range(nlanes), stats=stats)
            if r == 0 and len(pas) == 2:  # the packed two-fold pass: its odd lane over the whole lattice
                f, a, b, pens = pas[1]
                full_cells += _full_lane_vs_oracle(plan, 5, lat, Mall - Mk[:, f], Uall - Uk[:, f], a, b, pens[0])
        parts.append(tuple(engine.unpermute_lanes(order, np.concatenate([o[i] for o in outs])) for i in range(3)))
    got = [shard.unshard(grid, 8, [p[i] for p in parts]) for i in range(3)]
    want = [np.array([_GRID9[(f, a, c)][i] for f, a, b, pens in grid for c in pens]) for i in range(3)]
    for g, w in zip(got[:2], want[:2]):
        assert np.array_equal(np.asarray(g, np.float32).view(np.uint32), np.asarray(w, np.float32).view(np.uint32))
    assert np.array_equal(np.asarray(got[2], np.uint64), np.asarray(want[2], np.uint64))
    assert stats["lanes"] == 47 and stats["offtree_lanes"] == 47 and full_cells == plan.info["npat"]
    print(f"9-mer 8 ranks: 125 lanes unsharded = one-GPU roots; ranks 0, 4, 7: {stats['lanes']} lanes, "
          f"{stats['nodes']} tree nodes, {stats['candidates']} split candidates re-derived; "
          f"{full_cells} cells of the packed odd lane = oracle")


@pytest.mark.timeout(1500)
def test_11mer_8rank_share_mid_fold_pinned_full_size():
    """BASELINE configs[4] (ANNNNMNNNNA, 10 folds, 7x7 grid = 490 lanes) as the 8-GPU job
    cuts it: rank 1's share starts in the middle of a (alpha, fold) group and spans two
    alphas, so its passes pack pieces of different folds.  Every lane's root and partition
    is re-derived on the host (with every split candidate one level down on every fourth
    lane), a packed lane is compared with the oracle over the whole lattice, and the share's
    roots equal the same lanes run as the one-GPU job runs their groups."""
    from kmerpapa_amd import engine, shard
    from kmerpapa_amd.CV_tools import fold_tables
    from kmerpapa_amd.pattern_utils import generality
    from oracle import treecheck as T
    import bench
    gp, nf = "ANNNNMNNNNA", 10
    kmers, M, U = bench.synthetic_counts(gp, seed=9)
    ctx = {k: (int(m), int(u)) for k, m, u in zip(kmers, M, U)}
    contexts, Mf, Uf = fold_tables(ctx, nf, np.random.RandomState(1), np.uint32)
    Mk, Uk = engine.counts_in_kmer_order(gp, contexts, Mf, Uf, generality(gp), np.uint32)
    ms, us = Mf.sum(axis=0, dtype=np.uint64), Uf.sum(axis=0, dtype=np.uint64)
    grid = _grid_cv_order(ms.sum() - ms, us.sum() - us, ALPHAS11, PENS11, nf)
    rank = 1
    ids = shard.assign_lanes(grid, 8)[rank]
    assert ids[0] % len(PENS11) != 0  # starts mid-group
    mine = shard.rank_groups(grid, rank, 8)
    assert len({g[1] for g in mine}) == 2
    engine.release_all()
    dev = engine.visible_devices()[0]
    plan = engine.get_plan(dev, gp, 0)
    plan.set_counts(Mk, Uk)
    width = plan.info["lanes_per_workgroup"]
    passes, order = engine.plan_passes(mine, engine.pass_cap(mine, plan.require_lanes(), width), width)
    assert any(len({g[0] for g in pas}) == 2 for pas in passes)  # packed pieces of two folds
    lat = T.Lattice(gp)
    Mk64, Uk64 = Mk.astype(np.int64), Uk.astype(np.int64)
    Mall, Uall = Mk64.sum(axis=1), Uk64.sum(axis=1)
    stats, outs, full_cells, k = {}, [], 0, 0
    for pas in passes:
        rt, re, nl = plan.run(pas)
        outs.append((rt, re, nl))
        nlanes = sum(len(g[3]) for g in pas)
        _tree_check_pass(plan, lat, pas, Mk64, Uk64, rt, re, nl,
                         offtree=[j for j in range(nlanes) if (k + j) % 4 == 0], stats=stats)
        if not full_cells and len({g[0] for g in pas}) == 2:  # first packed pass: its last lane
            f, a, b, pens = pas[-1]
            full_cells = _full_lane_vs_oracle(plan, nlanes - 1, lat, Mall - Mk64[:, f], Uall - Uk64[:, f], a, b,
                                              pens[-1])
        k += nlanes
    share = [np.concatenate([o[i] for o in outs]) for i in range(3)]
    share = [engine.unpermute_lanes(order, x) for x in share]
    # the one-GPU job's passes over the groups this share touches
    touched = sorted({(g[0], g[1]) for g in mine})
    groups1 = [g for g in grid if (g[0], g[1]) in touched]
    p1, o1 = engine.plan_passes(groups1, engine.pass_cap(groups1, plan.require_lanes(), width), width)
    res1 = [plan.run(pas) for pas in p1]
    one = [engine.unpermute_lanes(o1, np.concatenate([x[i] for x in res1])) for i in range(3)]
    key1 = {(f, a, c): j for j, (f, a, c) in enumerate((f, a, c) for f, a, b, pens in groups1 for c in pens)}
    sel = [key1[(f, a, c)] for f, a, b, pens in mine for c in pens]
    for i in range(2):
        assert np.array_equal(np.asarray(share[i], np.float32).view(np.uint32),
                              np.asarray(one[i], np.float32)[sel].view(np.uint32))
    assert np.array_equal(np.asarray(share[2], np.uint64), np.asarray(one[2], np.uint64)[sel])
    assert stats["lanes"] == len(ids) and stats["offtree_lanes"] >= 10 and full_cells == plan.info["npat"]
    print(f"11-mer rank 1 of 8: {stats['lanes']} lanes in {len(passes)} passes = one-GPU roots; "
          f"{stats['nodes']} tree nodes, {stats['candidates']} split candidates ({stats['offtree_lanes']} lanes) "
          f"re-derived; {full_cells} cells of a packed lane = oracle")
    engine.release_all()

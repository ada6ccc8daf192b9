"""GPU parity on BASELINE.json's configs 3-5, through the C-ABI.

* config 4 (the headline, synthetic 9-mer counts, NNNNMNNNN): the benchmark's own counts
  restricted to sub-lattices the CPU oracle finishes in seconds --
    - ANNNMNNNA (34M cells), CV mode, 5 folds x 5 penalties x 2 pseudo counts: every
      lane's root train/test value and every lane's full float32 score array, bit for bit;
    - NNNNMNNNA (5.1e8 cells, 5 high positions), fit mode: score, root counts, the
      partition in backtrack order and the full score array;
* config 3 (the reference's 7-mer test data, NNNMNNN): the whole 3x3 grid x 5 folds
  against the oracle (every root) and against the reference itself (tests/golden/cv7.json:
  the reference's per-fold roots and CVfile rows, produced by make_golden.py);
* config 5 (synthetic 11-mers, 7x7 grid, 10 folds; run restricted by the super pattern
  ANNNNMNNNNA as SURVEY.md 8(d) prescribes): the full 7.69e9-cell lattice with 10 folds and
  7 penalties (size-independent properties, as test_gpu_fullsize.py), and the sub-lattice
  AANNNMNNNAA (34M cells x 10 folds x 7 penalties) bit for bit against the oracle.

Oracle passes run with OpenMP over each level's cells (same values as one thread).
"""
import functools
import io
import math
import os

import numpy as np
import pytest

from tests.fixtures import bits_equal, context_table, golden_json

pytestmark = pytest.mark.gpu


def _threads():
    n = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except AttributeError:
        pass
    return max(1, min(n, 16))


@pytest.fixture(scope="module")
def eng():
    from kmerpapa_amd import engine
    engine.load()
    assert engine.device_count() >= 1, "no GPU visible to the HIP runtime"
    return engine


@functools.lru_cache(maxsize=2)
def _synthetic(full_pat):
    import bench
    return bench.synthetic_counts(full_pat, seed=9)


def _restricted(full_pat, sub_pat):
    """The benchmark's synthetic counts of ``full_pat`` (bench.synthetic_counts), keeping the
    k-mers that match ``sub_pat`` (what ``--super_pattern sub_pat`` keeps)."""
    kmers, M, U = _synthetic(full_pat)
    fixed = [(i, c) for i, c in enumerate(sub_pat) if c != full_pat[i]]
    ctx = {}
    for k, m, u in zip(kmers, M, U):
        if all(k[i] == c for i, c in fixed):
            ctx[k] = (int(m), int(u))
    return ctx


def _folds(ctx, gen_pat, nf, seed=1):
    from kmerpapa_amd import engine
    from kmerpapa_amd.CV_tools import fold_tables
    from kmerpapa_amd.pattern_utils import generality
    contexts, Mf, Uf = fold_tables(ctx, nf, np.random.RandomState(seed), np.uint32)
    Mk, Uk = engine.counts_in_kmer_order(gen_pat, contexts, Mf, Uf, generality(gen_pat), np.uint32)
    msum, usum = Mk.sum(axis=0, dtype=np.uint64), Uk.sum(axis=0, dtype=np.uint64)
    return contexts, Mf, Uf, Mk, Uk, msum.sum() - msum, usum.sum() - usum


def _cv_vs_oracle(eng, gen_pat, ctx, nf, alphas, pens, full_lanes):
    """One GPU pass over every (alpha, fold) group; then one oracle pass per (alpha, c):
    roots of every lane bit for bit, full score arrays of the lanes in ``full_lanes``
    (None = all)."""
    from kmerpapa_amd.score_utils import get_betas
    from oracle import oracle as O
    contexts, Mf, Uf, Mk, Uk, mtr, utr = _folds(ctx, gen_pat, nf)
    betas = {a: get_betas(a, mtr, utr) for a in alphas}
    plan = eng.Plan(eng.get_device(0), gen_pat, 0)
    plan.set_counts(Mk, Uk)
    groups = [(f, a, float(betas[a][f]), pens) for a in alphas for f in range(nf)]
    rt, re, _ = plan.run(groups)
    checked = 0
    for a_i, a in enumerate(alphas):
        for p_i, c in enumerate(pens):
            ref = O.cv_pass(gen_pat, contexts, Mf, Uf, a, betas[a], c, 32, threads=_threads())
            for f in range(nf):
                lane = (a_i * nf + f) * len(pens) + p_i
                assert bits_equal(rt[lane], ref["root_train"][f]), (gen_pat, a, c, f, "root train")
                assert bits_equal(re[lane], ref["root_test"][f]), (gen_pat, a, c, f, "root test")
                if full_lanes is None or lane in full_lanes:
                    score, _ = plan.dump_lane(lane)
                    assert bits_equal(score, ref["score"][:, f]), (gen_pat, a, c, f, "score array")
                    checked += 1
            del ref
    plan.close()
    return len(rt), checked


def test_9mer_sublattice_cv_vs_oracle(eng):
    """Config 4's counts on ANNNMNNNA (34,171,875 cells): 2 alphas x 5 folds x 5 penalties
    = 50 lanes, every root and every full score array equal the oracle's."""
    ctx = _restricted("NNNNMNNNN", "ANNNMNNNA")
    assert len(ctx) == 8192
    lanes, checked = _cv_vs_oracle(eng, "ANNNMNNNA", ctx, 5, [0.5, 10.0], [3.0, 4.0, 5.0, 6.0, 7.0], None)
    assert lanes == 50 and checked == 50


@pytest.mark.timeout(900)
def test_9mer_5high_fit_vs_oracle(eng):
    """Config 4's counts on NNNNMNNNA (512,578,125 cells; 5 high positions at the default
    block of 3 low positions): score, root counts, partition in backtrack order and every
    cell's float32 score equal the oracle's."""
    from kmerpapa_amd.algorithms import bottum_up_array_w_numba as fitm
    from kmerpapa_amd.pattern_utils import PatternEnumeration
    from oracle import oracle as O
    gp = "NNNNMNNNA"
    ctx = _restricted("NNNNMNNNN", gp)
    nm = sum(v[0] for v in ctx.values())
    nu = sum(v[1] for v in ctx.values())
    my = nm / (nm + nu)
    alpha, pen = 1.0, 4.0
    beta = (alpha * (1.0 - my)) / my
    sc, Mr, Ur, leaves = fitm.fit_partition(gp, ctx, alpha, beta, pen, np.uint32)
    plan = eng.get_plan(eng.visible_devices()[0], gp, 0)
    assert plan.info["npat"] == 512578125
    score_gpu, _ = plan.dump_lane(0)
    kmers = list(ctx)
    M = np.array([ctx[k][0] for k in kmers], np.int64)
    U = np.array([ctx[k][1] for k in kmers], np.int64)
    rs, rm, ru, rnames, arrs = O.fit(gp, kmers, M, U, alpha, beta, pen, 32, threads=_threads())
    assert np.float32(sc).tobytes() == np.float32(rs).tobytes()
    assert (int(Mr), int(Ur)) == (rm, ru)
    PE = PatternEnumeration(gp)
    assert [PE.num2pattern(int(x)) for x in leaves] == rnames
    assert len(rnames) > 50
    assert bits_equal(score_gpu, arrs["score"])
    eng.release_all()


def test_7mer_grid_vs_oracle_and_reference(eng):
    """Config 3: the reference's 7-mer test data (NNNMNNN, 34,171,875 cells), the 3x3 grid
    c in {3,5,7} x alpha in {0.5,1,10}, 5 folds, seed 1, through the drop-in CV driver:
    every (alpha, c, fold) root equals the oracle's, and the per-fold roots, CVfile text and
    best point equal the reference's own (tests/golden/cv7.json)."""
    from kmerpapa_amd.algorithms import bottum_up_array_penalty_plus_pseudo_CV as cvm
    from kmerpapa_amd.CV_tools import fold_tables
    from oracle import oracle as O
    ctx, gp, nm, nu = context_table(7)
    alphas, pens = [0.5, 1.0, 10.0], [3.0, 5.0, 7.0]
    res = cvm.cv_roots(gp, ctx, alphas, pens, 5, 1, 1, np.uint32, devices=[0])
    contexts, Mf, Uf = fold_tables(ctx, 5, np.random.RandomState(1), np.uint32)
    for a_i, a in enumerate(alphas):
        for p_i, c in enumerate(pens):
            ref = O.cv_pass(gp, contexts, Mf, Uf, a, res["betas"][0, a_i], c, 32, threads=_threads())
            assert bits_equal(res["train"][0, a_i, p_i], ref["root_train"]), (a, c)
            assert bits_equal(res["test"][0, a_i, p_i], ref["root_test"]), (a, c)
            del ref
    buf = io.StringIO()

    class A:
        nfolds = 5
        iterations = 1
        seed = 1
        verbosity = 0
        CVfile = buf
    best = cvm.pattern_partition_bottom_up(gp, ctx, alphas, A, nm, nu, pens)
    g = golden_json("cv7.json")
    if g is None:
        pytest.skip("reference cv7 golden not generated (make_golden.py cv7p_* + cv7merge)")
    assert g["gen_pat"] == gp and g["alphas"] == alphas and g["penalties"] == pens
    for ps in g["passes"]:
        a_i, p_i = alphas.index(ps["alpha"]), pens.index(ps["penalty"])
        assert np.array_equal(res["betas"][0, a_i], np.array(ps["betas"]))
        assert bits_equal(res["train"][0, a_i, p_i], np.array(ps["root_train"], np.float32))
        assert bits_equal(res["test"][0, a_i, p_i], np.array(ps["root_test"], np.float32))
    assert buf.getvalue() == g["cvfile"]
    assert [best[0], best[1], best[2]] == g["best"]


PENS11 = [2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 8.0]


def test_11mer_sublattice_cv_vs_oracle(eng):
    """Config 5's counts (synthetic 11-mers, ANNNNMNNNNA) on AANNNMNNNAA (34M cells),
    10 folds x 7 penalties = 70 lanes: every root equals the oracle's; the full score
    arrays of one lane per fold too."""
    ctx = _restricted("ANNNNMNNNNA", "AANNNMNNNAA")
    assert len(ctx) == 8192
    full = {f * len(PENS11) + (f % len(PENS11)) for f in range(10)}
    lanes, checked = _cv_vs_oracle(eng, "AANNNMNNNAA", ctx, 10, [1.0], PENS11, full)
    assert lanes == 70 and checked == 10


def test_11mer_grid_fold_pieces_vs_oracle(eng):
    """Config 5's 7x7 grid as the CV driver runs it (engine.run_groups: each fold's lanes cut
    into 5-lane pieces, four of every seven spanning two alphas -> mixed device groups) on
    config 5's counts restricted to AANNNMNNAAA (2.3M cells), 10 folds: the root train and
    root test of every one of the 490 lanes equal the oracle's run with that lane's alpha
    (the backtrack re-derives each lane's optimal tree with its own alpha)."""
    from kmerpapa_amd.score_utils import get_betas
    from oracle import oracle as O
    gp = "AANNNMNNAAA"
    ctx = _restricted("ANNNNMNNNNA", gp)
    nf = 10
    alphas = [0.5, 1.0, 2.0, 3.0, 5.0, 7.0, 10.0]
    contexts, Mf, Uf, Mk, Uk, mtr, utr = _folds(ctx, gp, nf)
    betas = {a: get_betas(a, mtr, utr) for a in alphas}
    groups = [(f, a, float(betas[a][f]), PENS11) for a in alphas for f in range(nf)]
    passes, _ = eng.plan_passes(groups, 7, 5)
    assert sum(1 for p in passes if len({g[1] for g in p}) == 2) == 5 * nf  # mixed pieces
    rt, re, _ = eng.run_groups(gp, Mk, Uk, groups, devices=eng.visible_devices()[:1])
    for a_i, a in enumerate(alphas):
        for p_i, c in enumerate(PENS11):
            ref = O.cv_pass(gp, contexts, Mf, Uf, a, betas[a], c, 32, threads=_threads())
            for f in range(nf):
                lane = (a_i * nf + f) * len(PENS11) + p_i
                assert bits_equal(rt[lane], ref["root_train"][f]), (a, c, f, "root train")
                assert bits_equal(re[lane], ref["root_test"][f]), (a, c, f, "root test")
    eng.release_all()


def _wide_term(m, u, alpha, beta, pen):
    p = (m + alpha) / (((m + u) + alpha) + beta)
    s = pen
    if m > 0:
        s += (-2.0 * m) * math.log(p)
    if u > 0:
        s += (-2.0 * u) * math.log(1.0 - p)
    return s


def _kmer_term(m, u, alpha, beta, pen):
    p = (m + alpha) / (((m + u) + alpha) + beta)
    a = 0.0 if m == 0 else m * math.log(p)
    b = 0.0 if u == 0 else u * math.log1p(-p)
    return -2.0 * (a + b) + pen


@pytest.mark.timeout(900)
def test_11mer_full_lattice_properties(eng):
    """Config 5 at full size: ANNNNMNNNNA (7,688,671,875 cells), 10-fold split of the
    synthetic 11-mer counts, one (alpha, fold) group with the grid's 7 penalties: roots
    finite, train non-decreasing and pattern count non-increasing in c; then the fit on all
    data: the partition covers every k-mer once, its counts are the totals and its root
    score is the float64 sum of its leaves' terms."""
    from kmerpapa_amd.algorithms import bottum_up_array_w_numba as fitm
    from kmerpapa_amd.pattern_utils import generality, matches
    from kmerpapa_amd.score_utils import get_betas
    gp = "ANNNNMNNNNA"
    kmers, M, U = _synthetic(gp)
    ctx = {k: (int(m), int(u)) for k, m, u in zip(kmers, M, U)}
    contexts, Mf, Uf, Mk, Uk, mtr, utr = _folds(ctx, gp, 10)
    assert (Mf.sum(axis=1) == np.array([ctx[c][0] for c in contexts])).all()
    betas = get_betas(2.0, mtr, utr)
    plan = eng.get_plan(eng.visible_devices()[0], gp, 0)
    assert plan.info["npat"] == 7688671875
    plan.set_counts(Mk, Uk)
    rt, re, nl = plan.run([(7, 2.0, float(betas[7]), PENS11)])
    rt = np.asarray(rt, np.float64)
    assert np.isfinite(rt).all() and (np.diff(rt) >= -1e-6 * np.abs(rt[1:])).all()
    assert (np.diff(np.asarray(nl, np.int64)) <= 0).all()
    assert np.isfinite(np.asarray(re)).all()
    nm, nu = int(M.sum()), int(U.sum())
    my = nm / (nm + nu)
    alpha, pen = 2.0, 5.0
    beta = (alpha * (1.0 - my)) / my

    class A:
        verbosity = 0
    score, Mr, Ur, names = fitm.pattern_partition_bottom_up(gp, ctx, alpha, beta, pen, A, nm, nu)
    assert (int(Mr), int(Ur)) == (nm, nu)
    n_kmers = generality(gp)
    cover = np.zeros(n_kmers, np.int64)
    total = 0.0
    for name in names:
        ks = list(matches(name))
        idx = eng.kmer_order(gp, ks)
        cover[idx] += 1
        m, u = int(M[idx].sum()), int(U[idx].sum())
        total += _kmer_term(m, u, alpha, beta, pen) if len(ks) == 1 else _wide_term(m, u, alpha, beta, pen)
    assert (cover == 1).all()
    assert 50 < len(names) < n_kmers
    assert abs(float(score) - total) <= 2e-6 * abs(total)
    from tests.test_gpu_fullsize import _fit_tree_rederived
    _fit_tree_rederived(gp, kmers, M, U, alpha, beta, pen, score, names)  # root + partition bit for bit
    eng.release_all()

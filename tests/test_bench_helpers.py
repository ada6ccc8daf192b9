"""bench.py's host-side helpers (no GPU): the synthetic count table is the CLI's sorted
array table, the 8-rank CV shares cover every (alpha, fold, penalty) lane exactly once in
lane order, and passes never exceed the pass cap."""
import numpy as np

import bench
from kmerpapa_amd import engine
from kmerpapa_amd.io_utils import KmerCounts


def test_kmer_table_is_sorted_and_complete():
    kmers, M, U = bench.synthetic_counts("NMN", seed=3)
    t = bench.kmer_table(kmers, M, U)
    assert isinstance(t, KmerCounts)
    assert list(t) == sorted(kmers)
    for k, m, u in zip(kmers, M, U):
        assert t[k] == (int(m), int(u))


def _prep(nfolds=5, alphas=(0.5, 1.0, 2.0, 5.0, 10.0), pens=(3.0, 4.0, 5.0, 6.0, 7.0)):
    groups = [(f, a, 0.1 * (f + 1) * a, list(pens)) for a in alphas for f in range(nfolds)]
    return {"groups": groups}


def test_cv_shares_cover_every_lane_once():
    prep = _prep()
    want = [(g[0], g[1], c) for g in prep["groups"] for c in g[3]]
    for world in (1, 2, 3, 8):
        cap = engine.pass_cap(prep["groups"], 9)
        shares = bench.cv_shares(prep, world, cap)
        got = [(g[0], g[1], c) for passes in shares for p in passes for g in p for c in g[3]]
        assert sorted(got) == sorted(want) and len(got) == len(want)
        for passes in shares:  # passes in fold order (by the highest fold a pass needs)
            folds = [max(g[0] for g in p) for p in passes]
            assert folds == sorted(folds)
        assert all(sum(len(g[3]) for g in p) <= cap for passes in shares for p in passes)
        lanes = [sum(len(g[3]) for p in passes for g in p) for passes in shares]
        assert max(lanes) - min(lanes) <= 1


def test_pass_cap_is_one_workgroup_plus_one_lane_by_default():
    """Passes hold one workgroup's lanes plus one (a small piece of a split group packs
    beside a full one: 5 + 1, 4 + 2, 3 + 3 lanes each save ~11 ms); a wider user
    group keeps its width; KMERPAPA_PASS_LANES overrides."""
    groups = [(0, 1.0, 1.0, [1.0] * 5), (1, 1.0, 1.0, [1.0] * 3)]
    assert engine.PASS_LANES == 0
    assert engine.pass_cap(groups, 9, 5) == 6
    assert engine.pass_cap(groups, 9) == 7  # (no width known: the old 7-lane packing)
    assert engine.pass_cap(groups, 4, 5) == 4
    assert engine.pass_cap([(0, 1.0, 1.0, [1.0] * 8)], 9, 5) == 8
    # an 8-rank share of the 5x5x5 grid: [5, 5, 5, 1] -> passes [5], [5], [5, 1]
    share = [(f, 1.0, 1.0, [1.0] * n) for f, n in enumerate([5, 5, 5, 1])]
    assert [[len(g[3]) for g in p] for p in engine.pack_passes(share, engine.pass_cap(share, 9, 5))] == \
        [[5], [5], [5, 1]]
    # two full groups never share a pass; 4 + 2 and 3 + 3 do
    assert [[len(g[3]) for g in p] for p in engine.pack_passes(
        [(f, 1.0, 1.0, [1.0] * n) for f, n in enumerate([5, 5, 4, 2, 3, 3])], 6)] == [[5], [5], [4, 2], [3, 3]]
    # the 5x5x5 grid on one GPU: 25 passes of one group each
    p9, _ = engine.plan_passes(_prep()["groups"], engine.pass_cap(_prep()["groups"], 9, 5), 5)
    assert len(p9) == 25 and all(len(p) == 1 for p in p9)


def test_plan_passes_fold_order_and_lane_mapping():
    """8-rank shares of the 5x5x5 grid: [f4: 2 lanes, f0: 5, f1: 5, f2: 4] runs as passes
    [f0], [f1], [f2 + f4] and [f2: 1, f3: 5, f4: 5, f0: 5] as [f0], [f3 + f2], [f4]: the first
    pass needs only fold 0 (drawn first), a small piece never delays a lower fold's pass,
    the fold with the most lanes of a pass is laid out first, and results map back to the
    share's lane order."""
    share = [(4, 1.0, 1.0, [1.0, 2.0]), (0, 2.0, 1.0, [1.0] * 5), (1, 2.0, 1.0, [1.0] * 5), (2, 2.0, 1.0, [1.0] * 4)]
    for width in (None, 5):  # 5-lane fold pieces leave this share's groups whole
        passes, order = engine.plan_passes(share, engine.pass_cap(share, 9), width)
        assert [[(g[0], len(g[3])) for g in p] for p in passes] == [[(0, 5)], [(1, 5)], [(2, 4), (4, 2)]]
        lane_ids = np.arange(16)  # lane ids in the share's own order
        run = lane_ids[order]  # what the passes return
        assert (engine.unpermute_lanes(order, run) == lane_ids).all()
    share2 = [(2, 1.0, 1.0, [1.0]), (3, 1.0, 1.0, [1.0] * 5), (4, 1.0, 1.0, [1.0] * 5), (0, 1.0, 1.0, [1.0] * 5)]
    passes2, _ = engine.plan_passes(share2, engine.pass_cap(share2, 9))
    assert [[(g[0], len(g[3])) for g in p] for p in passes2] == [[(0, 5)], [(3, 5), (2, 1)], [(4, 5)]]
    # a share whose lowest fold is a 1-lane piece: that piece runs alone first rather than
    # wait (packed beside the 4-lane fold-2 piece) for fold 2 to be drawn
    share3 = [(2, 1.0, 1.0, [1.0] * 4), (3, 1.0, 1.0, [1.0] * 5), (4, 1.0, 1.0, [1.0] * 5), (0, 2.0, 1.0, [1.0])]
    passes3, order3 = engine.plan_passes(share3, engine.pass_cap(share3, 9), 5)
    assert [[(g[0], len(g[3])) for g in p] for p in passes3] == [[(0, 1)], [(2, 4)], [(3, 5)], [(4, 5)]]
    assert sorted(order3.tolist()) == list(range(15)) and order3[0] == 14
    # a 1-lane fold-4 piece packed with a 5-lane fold-3 group is laid out after it
    share4 = [(0, 1.0, 1.0, [1.0] * 5), (3, 1.0, 1.0, [1.0] * 5), (4, 2.0, 1.0, [1.0])]
    passes4, order4 = engine.plan_passes(share4, engine.pass_cap(share4, 9, 5), 5)
    assert [[(g[0], len(g[3])) for g in p] for p in passes4] == [[(0, 5)], [(3, 5), (4, 1)]]
    assert order4.tolist() == list(range(11))


def test_fold_pieces_cut_wide_grids_into_workgroup_widths():
    """The 11-mer grid (7 alphas x 7 penalties x 10 folds): each fold's 49 lanes become nine
    5-lane pieces and one 4-lane piece, a piece holding at most two alphas of one fold (the
    library runs it as one mixed device group), every lane exactly once and in order."""
    alphas, pens = [0.5, 1.0, 2.0, 3.0, 5.0, 7.0, 10.0], [2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 8.0]
    groups = [(f, a, 0.01 * a * (f + 1), list(pens)) for a in alphas for f in range(10)]
    passes, order = engine.plan_passes(groups, engine.pass_cap(groups, 9), 5)
    assert len(passes) == 100
    assert sorted(order.tolist()) == list(range(490))
    for p in passes:
        assert len({g[0] for g in p}) == 1 and 1 <= len(p) <= 2
        assert sum(len(g[3]) for g in p) in (4, 5)
    folds = [p[0][0] for p in passes]
    assert folds == sorted(folds)
    # every lane of the passes is the (fold, alpha, penalty) its lane id names
    lanes = [(g[0], g[1], c) for g in groups for c in g[3]]
    got = [(g[0], g[1], c) for p in passes for g in p for c in g[3]]
    assert got == [lanes[i] for i in order]
    # the 5x5x5 grid: pieces are the (alpha, fold) groups themselves
    p9, o9 = engine.plan_passes(_prep()["groups"], 7, 5)
    assert all(len(p) == 1 and len(p[0][3]) == 5 for p in p9) and len(p9) == 25


def test_scaling_table_entries():
    """bench.scaling_table: the measured entry is N = world (1 under the plain bench, the
    job's own N under torchrun); modelled worlds carry units/s, the kernel roofline (mean and
    min over the shares), the wall-clock with and without the per-rank allocation wait, and
    N x the measured step rate."""
    prep = _prep()
    npat = 1000
    total = npat * 125
    line = {"value": 5.0e9, "roofline": {"frac": 0.8, "effective_frac": 0.9}}
    cv = {"wall_s": 10.0, "wall_s_incl_alloc": 13.0, "hbm_alloc_s": 3.0,
          "models": {"8": {"wall_s": 1.25, "wall_s_incl_alloc": 4.25, "share_effective_roofline_frac": [0.9, 0.8],
                           "share_hbm_alloc_s": [3.0] * 8, "speedup": 8.0, "speedup_incl_alloc": 13.0 / 4.25}}}
    t = bench.scaling_table(line, cv, prep, npat)
    assert sorted(t) == ["1", "8"]
    assert t["1"]["measured"] and not t["8"]["measured"]
    assert t["1"]["units_per_s"] == total / 10.0 and t["1"]["units_per_s_incl_alloc"] == total / 13.0
    assert t["8"]["units_per_s"] == total / 1.25 and t["8"]["wall_s_incl_alloc"] == 4.25
    assert abs(t["8"]["effective_roofline_frac"] - 0.85) < 1e-12 and t["8"]["effective_roofline_frac_min"] == 0.8
    assert t["8"]["weak_units_per_s"] == 8 * 5.0e9 and t["8"]["hbm_alloc_s"] == 3.0
    t4 = bench.scaling_table(line, {"wall_s": 2.5, "wall_s_incl_alloc": 5.5, "hbm_alloc_s": 3.0}, prep, npat, world=4)
    assert sorted(t4) == ["4"] and t4["4"]["measured"] and t4["4"]["units_per_s"] == total / 2.5

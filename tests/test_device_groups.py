"""How kp_pass cuts a pass's groups into workgroups (host code, kp_device_groups; no GPU):
full workgroups first for a group wider than one, and consecutive groups of the same fold
cut together into mixed workgroups (at most two alphas each) when that needs fewer
workgroups -- what engine.fold_pieces relies on for the 11-mer's 7-penalty grid."""
import pytest

from kmerpapa_amd import engine


def _dg(sizes, folds=None, alphas=None, width=5):
    folds = folds or [0] * len(sizes)
    alphas = alphas or [float(i + 1) for i in range(len(sizes))]
    groups = [(f, a, 0.5 * a, [1.0 + j for j in range(n)]) for f, a, n in zip(folds, alphas, sizes)]
    return engine.device_groups(groups, width)


def test_wide_group_full_workgroups_first(monkeypatch):
    assert _dg([7]) == [(0, 5, 0), (5, 2, 0)]
    assert _dg([8], width=3) == [(0, 3, 0), (3, 3, 0), (6, 2, 0)]
    monkeypatch.setenv("KP_WIDE_SPLIT", "0")  # the near-equal split (A/B knob)
    assert _dg([7]) == [(0, 4, 0), (4, 3, 0)]


def test_same_fold_groups_become_mixed_workgroups():
    assert _dg([2, 3]) == [(0, 5, 3)]
    assert _dg([4, 1]) == [(0, 5, 1)]
    assert _dg([3, 4, 3]) == [(0, 5, 2), (5, 5, 3)]
    # a piece of the 11-mer grid: the last 2 penalties of one alpha, the first 3 of the next
    assert _dg([2, 3], alphas=[1.0, 2.0]) == [(0, 5, 3)]


def test_no_mixing_when_it_saves_nothing_or_needs_three_alphas():
    assert _dg([5, 2]) == [(0, 5, 0), (5, 2, 0)]          # 2 workgroups either way
    assert _dg([4, 2]) == [(0, 4, 0), (4, 2, 0)]
    assert _dg([2, 2, 1]) == [(0, 2, 0), (2, 2, 0), (4, 1, 0)]  # one workgroup would hold 3 alphas
    assert _dg([2, 3], folds=[0, 1]) == [(0, 2, 0), (2, 3, 0)]  # different folds never mix


def test_same_alpha_pieces_join_without_a_second_set():
    # two pieces of ONE (alpha, fold) group (e.g. a split group's lanes) join unmixed
    assert _dg([2, 3], alphas=[1.0, 1.0]) == [(0, 5, 0)]


def test_fold_pieces_run_as_one_workgroup_each():
    """Every 5-lane piece engine.plan_passes cuts from the 11-mer grid is one workgroup."""
    alphas, pens = [0.5, 1.0, 2.0, 3.0, 5.0, 7.0, 10.0], [2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 8.0]
    groups = [(f, a, 0.01 * a, list(pens)) for a in alphas for f in range(2)]
    passes, _ = engine.plan_passes(groups, 7, 5)
    mixed = 0
    for p in passes:
        dg = engine.device_groups(p, 5)
        assert len(dg) == 1 and dg[0][1] == sum(len(g[3]) for g in p)
        mixed += dg[0][2] > 0
    assert mixed == 10


def test_bad_arguments():
    with pytest.raises(engine.KPError):
        engine.device_groups([(0, 1.0, 1.0, [1.0])], 0)

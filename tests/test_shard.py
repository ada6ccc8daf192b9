"""Multi-rank sharding of the CV grid (kmerpapa_amd.shard), world_size 2 and 8 over gloo on the
CPU, with the host emulator of the blocked DP standing in for the GPU: the sharded CV
driver must return exactly the single-process roots, every group run exactly once."""
import os
import socket

import numpy as np
import pytest

from kmerpapa_amd import shard
from tests.fixtures import golden_json


def test_rank_groups_cover_every_lane_once_balanced():
    """Every lane in exactly one rank's share, shares within one lane of each other, and
    unshard puts the ranks' results back in the original lane order."""
    g55 = [(f, a, 0.1 * f + a, [3.0, 4.0, 5.0, 6.0, 7.0]) for a in (0.5, 1.0, 2.0, 5.0, 10.0) for f in shard.fold_order(5)]
    g77 = [(f, a, 0.1 * f + a, [2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 8.0]) for a in (0.5, 1.0, 2.0) for f in shard.fold_order(10)]
    gmix = [(f, 1.0, 1.0, [1.0] * (1 + f % 3)) for f in range(7)]
    for groups in (g55, g77, gmix):
        flat = [(g[0], g[1], c) for g in groups for c in g[3]]
        for world in (1, 2, 3, 4, 8):
            parts = [shard.rank_groups(groups, r, world) for r in range(world)]
            ids = [shard.rank_lane_ids(groups, r, world) for r in range(world)]
            got = [(g[0], g[1], c) for p in parts for g in p for c in g[3]]
            assert sorted(sum(ids, [])) == list(range(len(flat)))
            assert [flat[i] for i in sum(ids, [])] == got  # each rank's lanes are its ids, in order
            sizes = [sum(len(g[3]) for g in p) for p in parts]
            assert max(sizes) - min(sizes) <= 1, (len(groups), world, sizes)
            vals = [np.asarray(i, np.float64) for i in ids]  # a rank's results = its lanes' numbers
            assert np.array_equal(shard.unshard(groups, world, vals), np.arange(len(flat), dtype=np.float64))


def test_headline_grid_over_8_ranks_whole_groups():
    """The 5x5x5 grid over 8 ranks: 3 whole (alpha, fold) groups per rank; the leftover group
    is one of fold 4 (drawn last), cut into 1-lane pieces for ranks 0-4, which are the ranks
    holding a fold-0 group (they start when fold 0 is drawn); every 16-lane share packs as
    [5], [5], [5 + 1]."""
    from kmerpapa_amd import engine
    groups = [(f, a, 1.0, [3.0, 4.0, 5.0, 6.0, 7.0]) for a in (0.5, 1.0, 2.0, 5.0, 10.0) for f in shard.fold_order(5)]
    for r in range(8):
        mine = shard.rank_groups(groups, r, 8)
        sizes = sorted(len(g[3]) for g in mine)
        folds = {g[0] for g in mine}
        if r < 5:
            assert sizes == [1, 5, 5, 5] and 0 in folds
            one = [g for g in mine if len(g[3]) == 1][0]
            assert one[0] == 4
            passes, _ = engine.plan_passes(mine, engine.pass_cap(mine, 9, 5), 5)
            assert sorted(sum(len(g[3]) for g in p) for p in passes) == [5, 5, 6]
            assert min(g[0] for g in passes[0]) == 0  # the first pass is a fold-0 group
        else:
            assert sizes == [5, 5, 5]


def test_chunk_bounds_cover_every_group_once():
    for n in range(0, 30):
        lanes = [1 + (i * 7) % 5 for i in range(n)]
        for parts in (1, 2, 3, 4, 8):
            b = shard.chunk_bounds(lanes, parts)
            assert len(b) == parts + 1 and b[0] == 0 and b[-1] == n
            assert all(b[i] <= b[i + 1] for i in range(parts))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _work(rank, world, q)
    except Exception as e:  # reported to the parent instead of hanging it
        q.put((rank, None, repr(e), []))
    finally:
        dist.destroy_process_group()


def _work(rank, world, q):
    if True:
        from kmerpapa_amd.algorithms import bottum_up_array_penalty_plus_pseudo_CV as cvm
        from tests.emu import emu as E
        c = golden_json("small_dp.json")["cases"]["k3"]
        ctx = {k: tuple(v) for k, v in c["contextD"].items()}
        ran = []

        def counting(gen_pat, M, U, groups, devices=None, max_block=0):
            ran.extend((g[0], g[1], c) for g in groups for c in g[3])
            return E.run_groups(gen_pat, M, U, groups, devices=devices, max_block=max_block)
        run = shard.sharded_run_groups(counting, rank, world, shard.torch_all_gather())
        res = cvm.cv_roots(c["gen_pat"], ctx, c["alphas"], c["penalties"], c["nfolds"], c["seed"], 1, np.uint32,
                           run_groups=run)
        q.put((rank, res["train"].tobytes(), res["test"].tobytes(), ran))


@pytest.mark.parametrize("world", [2, 8])
def test_gloo_ranks_cv_matches_single_process(world):
    """world_size 2 and 8 over gloo (the 8-GPU job's rank count): each rank runs its
    lane-granular share, the all-gathered roots equal the single-process run's bytes."""
    import multiprocessing as mp
    from kmerpapa_amd.algorithms import bottum_up_array_penalty_plus_pseudo_CV as cvm
    from tests.emu import emu as E
    c = golden_json("small_dp.json")["cases"]["k3"]
    ctx = {k: tuple(v) for k, v in c["contextD"].items()}
    ref = cvm.cv_roots(c["gen_pat"], ctx, c["alphas"], c["penalties"], c["nfolds"], c["seed"], 1, np.uint32,
                       run_groups=E.run_groups)
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ran_all = []
    for rank, tr, te, ran in outs:
        assert tr is not None, f"rank {rank} failed: {te}"
        assert tr == ref["train"].tobytes() and te == ref["test"].tobytes(), f"rank {rank} roots differ"
        ran_all.extend(ran)
    want = [(f, a, p) for a in c["alphas"] for f in range(c["nfolds"]) for p in c["penalties"]]
    assert sorted(ran_all) == sorted(want)  # every lane (alpha, fold, penalty) exactly once over the ranks
    assert all(len(r) > 0 for _, _, _, r in outs)  # every rank did work (20 lanes over <= 8 ranks)


def test_engine_run_groups_lane_granular_over_devices(monkeypatch):
    """engine.run_groups splits the lanes over the GPUs of one process like the ranks of a
    torchrun job (contiguous equal runs, regrouped by (fold, alpha)) and returns them in
    the original lane order; every lane runs exactly once.  A stand-in plan replaces the
    GPU (each lane's "root" encodes its (fold, alpha, penalty))."""
    from kmerpapa_amd import engine
    ran = {}

    class FakePlan:
        info = {"lanes_per_workgroup": 5}  # Plan.info's piece width

        def __init__(self, dev):
            self.dev = dev

        def set_counts(self, M, U):
            pass

        def lanes_that_fit(self):
            return 7

        def require_lanes(self, n=1):
            return self.lanes_that_fit()

        def reserve(self, lanes):
            assert lanes <= 7

        def run(self, groups):
            lanes = [(g[0], g[1], c) for g in groups for c in g[3]]
            for ln in lanes:
                ran.setdefault(ln, []).append(self.dev)
            rt = np.array([f * 1000 + a * 10 + c for f, a, c in lanes], np.float32)
            return rt, -rt, np.arange(len(lanes), dtype=np.uint64)
    monkeypatch.setattr(engine, "get_plan", lambda dev, gp, mb=0, replica=0: FakePlan(dev))
    groups = [(f, a, 0.1, [3.0, 4.0, 5.0, 6.0, 7.0]) for a in (0.5, 1.0, 2.0, 5.0, 10.0) for f in range(5)]
    want = np.array([f * 1000 + a * 10 + c for f, a, _, pens in groups for c in pens], np.float32)
    for devs in ([0], [0, 1], [0, 1, 2], [3, 2, 1, 0, 4, 5, 6, 7]):
        ran.clear()
        rt, re, _ = engine.run_groups("NMN", None, None, groups, devices=devs)
        assert np.array_equal(rt, want) and np.array_equal(re, -want)
        assert len(ran) == 125 and all(len(v) == 1 for v in ran.values())
        per_dev = {}
        for v in ran.values():
            per_dev[v[0]] = per_dev.get(v[0], 0) + 1
        assert sorted(per_dev) == sorted(devs) and max(per_dev.values()) - min(per_dev.values()) <= 1


def test_cv_driver_prepares_devices_during_fold_split():
    """cv_roots hands the run_groups' prepare hook the lane shape of the grid (before the
    fold split, so betas are placeholders) exactly once, and the roots are unchanged."""
    from kmerpapa_amd.algorithms import bottum_up_array_penalty_plus_pseudo_CV as cvm
    from tests.emu import emu as E
    c = golden_json("small_dp.json")["cases"]["k3"]
    ctx = {k: tuple(v) for k, v in c["contextD"].items()}
    seen = []

    def run(gen_pat, M, U, groups, devices=None, max_block=0):
        return E.run_groups(gen_pat, M, U, groups, devices=devices, max_block=max_block)

    def prepare(gen_pat, groups, devices=None, max_block=0, itype=np.uint32):
        seen.append((gen_pat, [(g[0], g[1], list(g[3])) for g in groups]))
    run.prepare = prepare
    ref = cvm.cv_roots(c["gen_pat"], ctx, c["alphas"], c["penalties"], c["nfolds"], c["seed"], 1, np.uint32,
                       run_groups=E.run_groups)
    res = cvm.cv_roots(c["gen_pat"], ctx, c["alphas"], c["penalties"], c["nfolds"], c["seed"], 1, np.uint32,
                       run_groups=run)
    assert res["train"].tobytes() == ref["train"].tobytes() and res["test"].tobytes() == ref["test"].tobytes()
    assert len(seen) == 1 and seen[0][0] == c["gen_pat"]
    assert seen[0][1] == [(f, a, list(c["penalties"])) for a in c["alphas"] for f in shard.fold_order(c["nfolds"])]


def test_cv_driver_prepare_errors_surface():
    from kmerpapa_amd.algorithms import bottum_up_array_penalty_plus_pseudo_CV as cvm
    from tests.emu import emu as E
    c = golden_json("small_dp.json")["cases"]["k3"]
    ctx = {k: tuple(v) for k, v in c["contextD"].items()}

    def run(gen_pat, M, U, groups, devices=None, max_block=0):
        return E.run_groups(gen_pat, M, U, groups, devices=devices, max_block=max_block)

    def prepare(gen_pat, groups, devices=None, max_block=0, itype=np.uint32):
        raise MemoryError("lattice does not fit")
    run.prepare = prepare
    with pytest.raises(MemoryError):
        cvm.cv_roots(c["gen_pat"], ctx, c["alphas"], c["penalties"], c["nfolds"], c["seed"], 1, np.uint32,
                     run_groups=run)


def test_cv_driver_pipelined_fold_split_same_roots():
    """With a runner that takes a FoldFeed (fold-by-fold counts, lazy betas), cv_roots gives
    bit-identical roots and betas to the runner that gets the whole split at once,
    including the --iterations carry-over of the fold totals."""
    from kmerpapa_amd.algorithms import bottum_up_array_penalty_plus_pseudo_CV as cvm
    from tests.emu import emu as E
    c = golden_json("small_dp.json")["cases"]["k3"]
    ctx = {k: tuple(v) for k, v in c["contextD"].items()}
    calls = []

    def whole(gen_pat, M, U, groups, devices=None, max_block=0):  # no fold_feed attribute
        calls.append(type(M).__name__)
        return E.run_groups(gen_pat, M, U, groups, devices=devices, max_block=max_block)

    def fed(gen_pat, M, U, groups, devices=None, max_block=0):
        calls.append(type(M).__name__)
        return E.run_groups(gen_pat, M, U, groups, devices=devices, max_block=max_block)
    fed.fold_feed = True
    for it in (1, 2):
        calls.clear()
        a = cvm.cv_roots(c["gen_pat"], ctx, c["alphas"], c["penalties"], c["nfolds"], c["seed"], it, np.uint32,
                         run_groups=whole)
        b = cvm.cv_roots(c["gen_pat"], ctx, c["alphas"], c["penalties"], c["nfolds"], c["seed"], it, np.uint32,
                         run_groups=fed)
        assert calls == ["ndarray"] * it + ["FoldFeed"] * it
        for key in ("train", "test", "betas"):
            assert a[key].tobytes() == b[key].tobytes(), key


def test_engine_run_groups_fold_feed_order(monkeypatch):
    """engine.run_groups with a FoldFeed: all-data counts first, each fold uploaded once
    before the first pass that needs it, passes in fold order, lazy betas resolved when a
    pass runs, results in the original lane order; a failed split surfaces."""
    import threading
    from kmerpapa_amd import engine
    log = []

    class FakePlan:
        info = {"lanes_per_workgroup": 5}  # Plan.info's piece width

        def __init__(self, dev):
            self.dev = dev

        def counts_begin(self, M, U, nf):
            log.append(("begin", nf))

        def counts_fold(self, f, M, U):
            log.append(("fold", f))

        def lanes_that_fit(self):
            return 5

        def require_lanes(self, n=1):
            return self.lanes_that_fit()

        def reserve(self, lanes):
            pass

        def run(self, groups):
            for g in groups:
                assert ("fold", g[0]) in log
            b = [g[2]() if callable(g[2]) else g[2] for g in groups]
            log.append(("pass", tuple(g[0] for g in groups)))
            lanes = [(g[0], c, bb) for g, bb in zip(groups, b) for c in g[3]]
            rt = np.array([f * 100 + c + bb for f, c, bb in lanes], np.float32)
            return rt, -rt, np.zeros(len(lanes), np.uint64)
    monkeypatch.setattr(engine, "get_plan", lambda dev, gp, mb=0, replica=0: FakePlan(dev))
    nf = 4
    feed = engine.FoldFeed(np.zeros(3, np.uint32), np.zeros(3, np.uint32), nf)
    groups = [(f, a, (lambda f=f: 0.5 * f), [1.0, 2.0, 3.0]) for a in (1.0, 2.0) for f in (3, 1, 0, 2)]
    want = np.array([f * 100 + c + 0.5 * f for f, _, _, pens in groups for c in pens], np.float32)

    def produce():
        for f in range(nf):
            feed.put(f, np.zeros(3, np.uint32), np.zeros(3, np.uint32))
    th = threading.Thread(target=produce)
    th.start()
    rt, re, _ = engine.run_groups("NMN", feed, None, groups, devices=[0])
    th.join()
    assert np.array_equal(rt, want)
    assert log[0] == ("begin", nf)
    assert [e[1] for e in log if e[0] == "fold"] == [0, 1, 2, 3]
    passes = [e[1] for e in log if e[0] == "pass"]
    assert [max(p) for p in passes] == sorted(max(p) for p in passes)
    bad = engine.FoldFeed(np.zeros(3, np.uint32), np.zeros(3, np.uint32), nf)
    bad.put(0, np.zeros(3, np.uint32), np.zeros(3, np.uint32))
    bad.fail(ValueError("split failed"))
    with pytest.raises(RuntimeError):
        engine.run_groups("NMN", bad, None, groups, devices=[0])


def test_engine_run_groups_gpu_named_twice(monkeypatch):
    """A device list naming a GPU more than once (KMERPAPA_DEVICES=0,0: the multi-GPU path
    rehearsed on one GPU) gives every slot its own plan replica and host thread; lanes and
    results are as for distinct GPUs."""
    from kmerpapa_amd import engine
    made = []

    class FakePlan:
        info = {"lanes_per_workgroup": 5}  # Plan.info's piece width

        def __init__(self, dev, rep):
            self.key = (dev, rep)
            made.append(self.key)

        def set_counts(self, M, U):
            pass

        def lanes_that_fit(self):
            return 5

        def require_lanes(self, n=1):
            return self.lanes_that_fit()

        def reserve(self, lanes):
            pass

        def run(self, groups):
            lanes = [(g[0], g[1], c) for g in groups for c in g[3]]
            rt = np.array([f * 1000 + a * 10 + c for f, a, c in lanes], np.float32)
            return rt, -rt, np.zeros(len(lanes), np.uint64)
    monkeypatch.setattr(engine, "get_plan", lambda dev, gp, mb=0, replica=0: FakePlan(dev, replica))
    groups = [(f, a, 0.1, [3.0, 4.0, 5.0]) for a in (0.5, 1.0) for f in range(3)]
    want = np.array([f * 1000 + a * 10 + c for f, a, _, pens in groups for c in pens], np.float32)
    for devs in ([0, 0], [1, 0, 1, 1]):
        made.clear()
        rt, _, _ = engine.run_groups("NMN", None, None, groups, devices=devs)
        assert np.array_equal(rt, want)
        assert sorted(made) == sorted(zip(devs, engine._replicas(devs)))
    assert engine._replicas([1, 0, 1, 1]) == [0, 0, 1, 2]


def test_cv_driver_over_8_devices_with_emulator_plans(monkeypatch):
    """The CV driver's default runner (engine.run_groups with the pipelined fold feed) over 8
    distinct device ids, each slot's plan an emulator-backed stand-in of engine.Plan
    (tests/emu EmuPlan: counts_begin / counts_fold / run): the real lane-granular split,
    fold pieces, pass packing, feeder threads and lane re-ordering run 8 wide, and the
    roots and betas equal the single-process emulator run's bytes for a 5 x 5 grid."""
    from kmerpapa_amd import engine
    from kmerpapa_amd.algorithms import bottum_up_array_penalty_plus_pseudo_CV as cvm
    from tests.emu import emu as E
    c = golden_json("small_dp.json")["cases"]["k3"]
    ctx = {k: tuple(v) for k, v in c["contextD"].items()}
    alphas, pens, nf = [0.5, 1.0, 2.0, 5.0, 10.0], [1.0, 2.0, 3.0, 4.0, 5.0], 5
    plans = {}

    def get_plan(dev, gp, mb=0, replica=0):
        if (dev, replica) not in plans:
            plans[(dev, replica)] = E.EmuPlan(gp, mb)
        return plans[(dev, replica)]
    monkeypatch.setattr(engine, "get_plan", get_plan)
    ref = cvm.cv_roots(c["gen_pat"], ctx, alphas, pens, nf, 3, 1, np.uint32, run_groups=E.run_groups)
    devs = list(range(8))
    res = cvm.cv_roots(c["gen_pat"], ctx, alphas, pens, nf, 3, 1, np.uint32, devices=devs)
    for key in ("train", "test", "betas"):
        assert res[key].tobytes() == ref[key].tobytes(), key
    assert sorted(d for d, _ in plans) == devs
    lanes = {d: sum(n for p in plans[(d, 0)].passes for _, _, n in p) for d in devs}
    assert sum(lanes.values()) == 125 and max(lanes.values()) - min(lanes.values()) <= 1
    for d in devs:  # a share's passes run in fold order, each within the slot's reservation
        folds = [max(f for f, _, _ in p) for p in plans[(d, 0)].passes]
        assert folds == sorted(folds)
        assert all(sum(n for _, _, n in p) <= plans[(d, 0)].reserved for p in plans[(d, 0)].passes)


def test_prepare_groups_surfaces_plan_errors(monkeypatch):
    """engine.prepare_groups (run beside the fold split by the CV driver) re-raises an error
    from any device's preparation in the caller, e.g. the lattice not fitting one lane."""
    from kmerpapa_amd import engine

    class TooBig:
        info = {"lanes_per_workgroup": 5}

        def require_lanes(self, n=1):
            raise engine.KPError(-2, "does not fit")

        def reserve(self, lanes):
            raise AssertionError("nothing may be reserved")
    monkeypatch.setattr(engine, "get_plan", lambda dev, gp, mb=0, replica=0: TooBig())
    groups = [(f, 1.0, 1.0, [3.0, 4.0]) for f in range(4)]
    with pytest.raises(engine.KPError) as e:
        engine.prepare_groups("NNMNN", groups, devices=[0, 1])
    assert e.value.code == -2


def test_prepared_shares_at_the_counts_width(monkeypatch):
    """The CV driver's prepare hook gets the counts' width, and the shares it prepares are the
    ones run_groups will run: with 64-bit counts the 9-mer lattice's workgroup holds 4 lanes
    (engine.shard_width), so whole 4-lane pieces are dealt and a pass holds at most 5 lanes;
    the sharded wrapper (torchrun ranks) hands the same width and itype to the inner hook."""
    from kmerpapa_amd import engine
    gp = "NNNNMNNNN"
    assert engine.shard_width(gp, np.uint32) == 5 and engine.shard_width(gp, np.uint64) == 4
    groups = [(f, a, 1.0, [3.0, 4.0, 5.0, 6.0, 7.0]) for a in (0.5, 1.0, 2.0, 5.0, 10.0) for f in shard.fold_order(5)]
    reserved = {}

    class Plan:
        info = {"lanes_per_workgroup": 5}  # (the plan's width before counts: uint32)

        def __init__(self, dev):
            self.dev = dev

        def require_lanes(self, n=1):
            return 9

        def reserve(self, lanes):
            reserved[self.dev] = lanes
    monkeypatch.setattr(engine, "get_plan", lambda dev, gp, mb=0, replica=0: Plan(dev))
    for itype, width in ((np.uint32, 5), (np.uint64, 4)):
        reserved.clear()
        engine.prepare_groups(gp, groups, devices=list(range(8)), itype=itype)
        for d in range(8):
            mine = shard.rank_groups(groups, d, 8, width)
            passes, _ = engine.plan_passes(mine, engine.pass_cap(mine, 9, width), width)
            assert reserved[d] == max(sum(len(g[3]) for g in p) for p in passes) <= width + 1
    seen = []

    def inner(*a, **k):
        raise AssertionError("not run")

    def inner_prepare(gen_pat, grps, devices=None, max_block=0, itype=np.uint32):
        seen.append((grps, itype))
    inner.prepare = inner_prepare
    for r in (0, 7):
        run = shard.sharded_run_groups(inner, r, 8, all_gather=None)
        run.prepare(gp, groups, itype=np.uint64)
        assert seen[-1] == (shard.rank_groups(groups, r, 8, 4), np.uint64)

"""The unrestricted 9-mer lattice the reference accepts: counts over all 4^9 k-mers give
the general pattern NNNNNNNNN (LCA, cli.py:180-187) = 15^9 = 3.84e10 cells.  The
reference's CV layout would need 24 B per cell per fold (CV :93-102); this build's
value-only sweep needs 4 B per cell per lane = 154 GB, so one lane fits an MI355X.

* one CV lane over the whole lattice (19 launches, cells and score offsets far past
  2^32 and 2^35): every cell of two embedded sub-lattices equals the oracle's run on that
  sub-lattice with the full run's fold counts and beta, bit for bit, and the root's train,
  test and partition are pinned by the host tree re-derivation;
* a lattice whose single lane does not fit (NNNNNNNNNR, 461 GB per lane) is refused with
  KP_E_NOMEM by the engine and by the C-ABI, and nothing is run.

The counts total more than 2^32 - 1, so the reference's itype is uint64 (CV :94-97):
this also runs the 64-bit count kernels at full size.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GP = "NNNNNNNNN"


@pytest.fixture(scope="module")
def data():
    import bench
    from kmerpapa_amd import engine
    from kmerpapa_amd.CV_tools import fold_tables
    from kmerpapa_amd.pattern_utils import generality
    kmers, M, U = bench.synthetic_counts(GP, seed=9)
    assert len(kmers) == 4 ** 9
    itype = np.uint64 if int(M.sum() + U.sum()) > np.iinfo(np.uint32).max else np.uint32
    ctx = {k: (int(m), int(u)) for k, m, u in zip(kmers, M, U)}
    contexts, Mf, Uf = fold_tables(ctx, 5, np.random.RandomState(1), itype)
    Mk, Uk = engine.counts_in_kmer_order(GP, contexts, Mf, Uf, generality(GP), itype)
    ms, us = Mk.sum(axis=0, dtype=np.uint64), Uk.sum(axis=0, dtype=np.uint64)
    return {"contexts": contexts, "Mf": Mf, "Uf": Uf, "Mk": Mk, "Uk": Uk, "itype": itype,
            "mtr": ms.sum() - ms, "utr": us.sum() - us}


@pytest.mark.timeout(1200)
def test_unrestricted_9mer_lane_vs_oracle(data):
    import time
    from kmerpapa_amd import engine
    from kmerpapa_amd.score_utils import get_betas
    from oracle import oracle as O
    from oracle import treecheck as T
    from tests.fixtures import bits_equal
    from tests.test_gpu_fullsize import IUPAC, _embedded_cells, _threads
    assert data["itype"] == np.uint64
    engine.release_all()
    plan = engine.get_plan(engine.visible_devices()[0], GP, 0)
    try:
        assert plan.info["npat"] == 15 ** 9 and plan.info["bytes_per_lane"] > 150e9
        t0 = time.perf_counter()
        plan.set_counts(data["Mk"], data["Uk"])
        t_counts = time.perf_counter() - t0
        assert plan.require_lanes() >= 1
        alpha, fold, c = 1.0, 2, 5.0
        beta = float(get_betas(alpha, data["mtr"], data["utr"])[fold])
        t0 = time.perf_counter()
        plan.reserve(1)
        t_alloc = time.perf_counter() - t0
        rt, re, nl = plan.run([(fold, alpha, beta, [c])])
        st = plan.stats()
        assert st["units"] == 15 ** 9 and st["dp_launches"] == plan.info["high_levels"]
        print(f"NNNNNNNNN 1 lane: dp {st['dp_ms']:.1f} ms, pass {st['total_ms']:.1f} ms, counts {t_counts:.2f} s, "
              f"alloc {t_alloc:.2f} s, {int(nl[0])} patterns")
        sp = data
        for sub in ("NNNNNNAAA", "AANNNNNNV"):
            keep = [i for i, x in enumerate(sp["contexts"]) if all(x[j] in IUPAC[ch] for j, ch in enumerate(sub))]
            ctxs = [sp["contexts"][i] for i in keep]
            mf, uf = sp["Mf"][keep], sp["Uf"][keep]
            m2 = np.stack([mf[:, fold], mf.sum(axis=1) - mf[:, fold]], axis=1)
            u2 = np.stack([uf[:, fold], uf.sum(axis=1) - uf[:, fold]], axis=1)
            cells = _embedded_cells(GP, sub)
            assert cells.size == O.npat(sub)
            if sub == "AANNNNNNV":
                assert (cells * 4 > 2 ** 35).sum() > cells.size // 2  # score offsets past 2^35 bytes
            ref = O.cv_pass(sub, ctxs, m2, u2, alpha, [beta, beta], c, 64, threads=_threads())
            got = plan.gather_cells(0, cells)
            assert bits_equal(got, ref["score"][:, 0]), (sub, int(np.sum(got.view(np.uint32) !=
                                                                         ref["score"][:, 0].view(np.uint32))))
            del ref
        # the root: the whole optimal tree re-derived on the host
        lat = T.Lattice(GP)
        Mk, Uk = sp["Mk"].astype(np.int64), sp["Uk"].astype(np.int64)
        mte, ute = Mk[:, fold], Uk[:, fold]
        r = T.rederive(lat, lambda cells: plan.gather_cells(0, cells), Mk.sum(axis=1) - mte, Uk.sum(axis=1) - ute,
                       mte, ute, alpha, beta, c)
        assert r["root_train"].view(np.uint32) == np.float32(rt[0]).view(np.uint32)
        assert r["root_test"].view(np.uint32) == np.float32(re[0]).view(np.uint32)
        assert np.array_equal(plan.leaves(0), r["leaves"]) and r["leaves"].size == int(nl[0])
    finally:
        engine.release_all()


@pytest.mark.timeout(600)
def test_lattice_too_big_for_one_lane_refused(data):
    """NNNNNNNNNR (1.15e11 cells, 461 GB per lane): the plan builds, the engine refuses to
    plan a pass (KP_E_NOMEM with the lattice and sizes in the message), kp_reserve_lanes
    refuses too, and run_groups raises the same error instead of running zero-lane passes."""
    from kmerpapa_amd import engine
    engine.release_all()
    dev = engine.visible_devices()[0]
    plan = engine.Plan(engine.get_device(dev), GP + "R", 0)
    try:
        assert plan.info["bytes_per_lane"] > 400e9 and plan.lanes_that_fit() == 0
        with pytest.raises(engine.KPError) as e:
            plan.require_lanes()
        assert e.value.code == -2 and "NNNNNNNNNR" in str(e.value) and "--super_pattern" in str(e.value)
        with pytest.raises(engine.KPError) as e:
            plan.reserve(1)
        assert e.value.code == -2
    finally:
        plan.close()
    # through the runner (the CV driver's path): same refusal before any pass
    n = 4 ** 10 // 2
    M = np.zeros((n, 2), np.uint32)
    with pytest.raises(engine.KPError) as e:
        engine.run_groups(GP + "R", M, M, [(0, 1.0, 1.0, [3.0])], devices=[dev])
    assert e.value.code == -2
    engine.release_all()

"""GPU parity: the HIP lattice DP (through the C-ABI) against the reference's golden
vectors and against the CPU oracle.  Bar: bit-exact float32 scores (any NaN equals any
NaN), identical partitions (names and order), identical CVfile text.
"""
import io
import os
import random

import numpy as np
import pytest

from tests.fixtures import bits_equal, context_table, golden_json, golden_npz, write_count_files, write_joint_file

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from kmerpapa_amd import engine
    engine.load()
    assert engine.device_count() >= 1, "no GPU visible to the HIP runtime"
    return engine


def _kmer_rows(gp, kmers, rows, dtype):
    from kmerpapa_amd import engine
    from kmerpapa_amd.pattern_utils import generality
    M, _ = engine.counts_in_kmer_order(gp, list(kmers), rows, rows, generality(gp), dtype)
    return M


SMALL = golden_json("small_dp.json")


@pytest.mark.parametrize("case", ["k3", "k4", "k3zero", "k3big"])
@pytest.mark.parametrize("max_block", [0, 16, 200])
def test_small_lattices_full_arrays(eng, case, max_block):
    """Every cell's f32 train score and the root test -2LL of every fold, bit for bit."""
    c = SMALL["cases"][case]
    A = golden_npz("small_dp.npz")
    gp = c["gen_pat"]
    dtype = np.uint64 if c["itype"] == "uint64" else np.uint32
    kmers = [str(x) for x in A[f"{case}_kmers"]]
    Mk = _kmer_rows(gp, kmers, A[f"{case}_Mf"], dtype)
    Uk = _kmer_rows(gp, kmers, A[f"{case}_Uf"], dtype)
    nf = Mk.shape[1]
    plan = eng.Plan(eng.get_device(0), gp, max_block)
    plan.set_counts(Mk, Uk)
    for j, ps in enumerate(c["passes"]):
        groups = [(f, ps["alpha"], ps["betas"][f], [ps["penalty"]]) for f in range(nf)]
        rt, re, _ = plan.run(groups)
        ref = A[f"{case}_{j}_score"]
        for f in range(nf):
            score, code = plan.dump_lane(f)
            assert bits_equal(score, ref[:, f]), f"{case} pass {j} fold {f}: score array differs"
        assert bits_equal(rt, np.array(ps["root_train"], np.float32))
        assert bits_equal(re, np.array(ps["root_test"], np.float32))
    plan.close()


@pytest.mark.parametrize("max_block", [0, 16])
def test_block_setup_without_pair_table(eng, monkeypatch, max_block):
    """KP_HPD=0: the sweep's block setup from the packed digits and pair tables (the path
    plans take when the per-plan pair table is off or cannot be built: blocks with more
    than 64 high pairs, 2^29+ blocks, or no memory for it) -- config 2's 5-mer lattice,
    5 folds x 2 penalties, every lane's full score array equals the oracle's."""
    from kmerpapa_amd.CV_tools import fold_tables
    from kmerpapa_amd.pattern_utils import generality
    from kmerpapa_amd.score_utils import get_betas
    from oracle import oracle as O
    monkeypatch.setenv("KP_HPD", "0")
    ctx, gp, nm, nu = context_table(5)
    contexts, Mf, Uf = fold_tables(ctx, 5, np.random.RandomState(1), np.uint32)
    Mk, Uk = eng.counts_in_kmer_order(gp, contexts, Mf, Uf, generality(gp), np.uint32)
    ms, us = Mf.sum(axis=0, dtype=np.uint64), Uf.sum(axis=0, dtype=np.uint64)
    betas = get_betas(1.0, ms.sum() - ms, us.sum() - us)
    plan = eng.Plan(eng.get_device(0), gp, max_block)
    try:
        assert plan.info["high_levels"] > 1
        plan.set_counts(Mk, Uk)
        pens = [3.0, 6.0]
        plan.run([(f, 1.0, float(betas[f]), pens) for f in range(5)])
        for j, c in enumerate(pens):
            ref = O.cv_pass(gp, contexts, Mf, Uf, 1.0, betas, c, 32)
            for f in range(5):
                score, _ = plan.dump_lane(f * len(pens) + j)
                assert bits_equal(score, ref["score"][:, f]), (max_block, c, f)
    finally:
        plan.close()


@pytest.mark.parametrize("gen_pat,max_block,env", [
    ("NNNNMNNNN", 0, None), ("RYSWKMBDHVN", 16, None), ("NNNNNNN", 16, None), ("NNNN", 0, None),
    ("NNNNNNN", 16, ("KP_BLOCK_PERM", "3-0-5")), ("NNNNNNN", 16, ("KP_BLOCK_TILE", "2"))])
def test_device_block_list_matches_host_walk(eng, monkeypatch, gen_pat, max_block, env):
    """The plan's block list as the device builds it (kp_blocks_kernel: hlist, kpos, hdig,
    hnp) equals the host's block walk entry for entry; KP_BLOCK_TILE (an experiment order
    the host builds and uploads) goes through the same check."""
    if env:
        monkeypatch.setenv(*env)
    plan = eng.Plan(eng.get_device(0), gen_pat, max_block)
    try:
        assert plan.block_check() == 0
    finally:
        plan.close()


@pytest.mark.parametrize("case", ["k3", "k4", "k3zero", "k3big"])
def test_small_lattice_fits(eng, case):
    from kmerpapa_amd.algorithms import bottum_up_array_w_numba as fitm
    c = SMALL["cases"][case]
    ctx = {k: tuple(v) for k, v in c["contextD"].items()}

    class A:
        verbosity = 0
    for fo in c["fits"]:
        if "error" in fo:
            continue  # the reference raises ZeroDivisionError for alpha=0 with an empty k-mer
        sc, M, U, names = fitm.pattern_partition_bottom_up(c["gen_pat"], ctx, fo["alpha"], fo["beta"],
                                                           fo["penalty"], A, c["nmut"], c["nunmut"])
        assert float(sc) == fo["score"]
        assert int(M) == fo["M"] and int(U) == fo["U"]
        assert names == fo["names"]


def test_grid5_cvfile(eng):
    """Config 2: 5-mer 3x3 grid, 5 folds, seed 1 -> CVfile text and best (alpha, c)."""
    from kmerpapa_amd.algorithms import bottum_up_array_penalty_plus_pseudo_CV as cvm
    g = golden_json("grid5.json")
    ctx, gp, nm, nu = context_table(5)
    assert gp == g["gen_pat"]
    buf = io.StringIO()

    class A:
        nfolds = 5
        iterations = 1
        seed = 1
        verbosity = 0
        CVfile = buf
    best = cvm.pattern_partition_bottom_up(gp, ctx, g["alphas"], A, nm, nu, g["penalties"])
    assert buf.getvalue() == g["cvfile"]
    assert [best[0], best[1], best[2]] == g["best"]


def test_grid5_roots_per_fold(eng):
    from kmerpapa_amd.algorithms import bottum_up_array_penalty_plus_pseudo_CV as cvm
    g = golden_json("grid5.json")
    ctx, gp, nm, nu = context_table(5)
    res = cvm.cv_roots(gp, ctx, g["alphas"], g["penalties"], 5, 1, 1, np.uint32, devices=[0])
    for ps in g["passes"]:
        a_i = g["alphas"].index(ps["alpha"])
        p_i = g["penalties"].index(ps["penalty"])
        assert bits_equal(res["test"][0, a_i, p_i], np.array(ps["root_test"], np.float32))
        assert bits_equal(res["train"][0, a_i, p_i], np.array(ps["root_train"], np.float32))
        assert np.array_equal(res["betas"][0, a_i], np.array(ps["betas"]))


def test_grid5_multi_device_path_on_one_gpu(eng, monkeypatch):
    """The single-process multi-GPU path (engine.run_groups: lane-granular slots, one host
    thread, context and HIP stream per slot, fold-by-fold count upload) run on the one GPU
    of the box by naming it 2, 3 and 8 times (8 contexts, 8 streams, 8 host threads: the
    8-GPU job's fan-out): per-fold roots equal the oracle's and the reference's, and the
    CVfile and best point the reference's (config 2)."""
    from kmerpapa_amd.algorithms import bottum_up_array_penalty_plus_pseudo_CV as cvm
    from kmerpapa_amd.CV_tools import fold_tables
    from oracle import oracle as O
    g = golden_json("grid5.json")
    ctx, gp, nm, nu = context_table(5)
    contexts, Mf, Uf = fold_tables(ctx, 5, np.random.RandomState(1), np.uint32)
    for devs in ([0, 0], [0, 0, 0], [0] * 8):
        res = cvm.cv_roots(gp, ctx, g["alphas"], g["penalties"], 5, 1, 1, np.uint32, devices=devs)
        for ps in g["passes"]:
            a_i = g["alphas"].index(ps["alpha"])
            p_i = g["penalties"].index(ps["penalty"])
            assert bits_equal(res["test"][0, a_i, p_i], np.array(ps["root_test"], np.float32)), devs
            assert bits_equal(res["train"][0, a_i, p_i], np.array(ps["root_train"], np.float32)), devs
            if len(devs) == 8:
                ref = O.cv_pass(gp, contexts, Mf, Uf, ps["alpha"], res["betas"][0, a_i], ps["penalty"], 32)
                assert bits_equal(res["train"][0, a_i, p_i], ref["root_train"]), devs
                assert bits_equal(res["test"][0, a_i, p_i], ref["root_test"]), devs
    monkeypatch.setenv("KMERPAPA_DEVICES", ",".join(["0"] * 8))
    buf = io.StringIO()

    class A:
        nfolds = 5
        iterations = 1
        seed = 1
        verbosity = 0
        CVfile = buf
    best = cvm.pattern_partition_bottom_up(gp, ctx, g["alphas"], A, nm, nu, g["penalties"])
    assert buf.getvalue() == g["cvfile"]
    assert [best[0], best[1], best[2]] == g["best"]
    eng.release_all()  # the replicas' buffers


def test_iterations_carry_over(eng):
    """--iterations 2 reproduces the reference's fold totals (its carry-over of the previous
    iteration's aggregated rows, CV :134-137), roots and CVfile (5-mer, tests/golden/iter5.json)."""
    from kmerpapa_amd.algorithms import bottum_up_array_penalty_plus_pseudo_CV as cvm
    g = golden_json("iter5.json")
    if g is None:
        pytest.skip("iteration golden not generated")
    ctx, gp, nm, nu = context_table(5)
    res = cvm.cv_roots(gp, ctx, g["alphas"], g["penalties"], g["nfolds"], g["seed"], 2, np.uint32, devices=[0])
    for j, ps in enumerate(g["passes"]):
        it, a_i = divmod(j, len(g["alphas"]))
        assert np.array_equal(res["betas"][it, a_i], np.array(ps["betas"]))
        assert bits_equal(res["test"][it, a_i, 0], np.array(ps["root_test"], np.float32))
    buf = io.StringIO()

    class A:
        nfolds = g["nfolds"]
        iterations = 2
        seed = g["seed"]
        verbosity = 0
        CVfile = buf
    best = cvm.pattern_partition_bottom_up(gp, ctx, g["alphas"], A, nm, nu, g["penalties"])
    assert buf.getvalue() == g["cvfile"]
    assert [best[0], best[1], best[2]] == g["best"]


def test_fit5_partitions(eng):
    from kmerpapa_amd.algorithms import bottum_up_array_w_numba as fitm
    g = golden_json("fit5.json")
    ctx, gp, nm, nu = context_table(5)

    class A:
        verbosity = 0
    for fo in g["fits"]:
        sc, M, U, names = fitm.pattern_partition_bottom_up(gp, ctx, fo["alpha"], fo["beta"], fo["penalty"], A, nm, nu)
        assert float(sc) == fo["score"]
        assert names == fo["names"]


@pytest.mark.parametrize("run", ["fit", "fit_long", "grid", "super", "default_pen"])
def test_cli5_output_text(eng, run, tmp_path, capsys):
    """Config 1/2 through the CLI: the output table and CVfile are byte-identical."""
    from kmerpapa_amd import cli
    g = golden_json("cli5.json")[run]
    pos, bg = write_count_files(5, str(tmp_path))
    argv = []
    for a in g["argv"]:
        argv.append(pos if a.endswith("mutated_5mers.txt") else bg if a.endswith("background_5mers.txt") else a)
    out = tmp_path / "o.txt"
    cvf = tmp_path / "cv.txt"
    rc = cli.main(argv + ["-o", str(out), "-f", str(cvf)])
    assert rc == g["rc"]
    assert out.read_text() == g["output"]
    assert cvf.read_text() == g["cvfile"]


@pytest.mark.parametrize("run", ["smaller_k", "joint", "negative"])
def test_cli5b_input_variants(eng, run, tmp_path):
    """--test_smaller_k CV (k = 5 and 3), a joint count file and a --negative file through
    the CLI (native reader, array-backed table): output table and CVfile byte-identical to
    the reference's (golden cli5b.json)."""
    from kmerpapa_amd import cli
    g = golden_json("cli5b.json")[run]
    pos, bg = write_count_files(5, str(tmp_path))
    joint = write_joint_file(5, str(tmp_path))
    argv = []
    for a in g["argv"]:
        argv.append(pos if a.endswith("mutated_5mers.txt") else bg if a.endswith("background_5mers.txt")
                    else joint if a.endswith("joint_5mers.txt") else a)
    out = tmp_path / "o.txt"
    cvf = tmp_path / "cv.txt"
    rc = cli.main(argv + ["-o", str(out), "-f", str(cvf)])
    assert rc == g["rc"]
    assert out.read_text() == g["output"]
    assert cvf.read_text() == g["cvfile"]


def test_fit7_partition(eng):
    g = golden_json("fit7.json")
    if g is None:
        pytest.skip("7-mer fit golden not generated")
    from kmerpapa_amd.algorithms import bottum_up_array_w_numba as fitm
    ctx, gp, nm, nu = context_table(7)

    class A:
        verbosity = 0
    fo = g["fits"][0]
    sc, M, U, names = fitm.pattern_partition_bottom_up(gp, ctx, fo["alpha"], fo["beta"], fo["penalty"], A, nm, nu)
    assert float(sc) == fo["score"]
    assert names == fo["names"]


def test_9mer_sublattice_fit_vs_oracle(eng):
    """Synthetic 9-mer counts of the benchmark restricted to ANNNMNNNA (34M cells): the fit
    (score, M, U, partition in backtrack order) equals the oracle's."""
    import bench
    from kmerpapa_amd.algorithms import bottum_up_array_w_numba as fitm
    from oracle import oracle as O
    kmers, M, U = bench.synthetic_counts("ANNNMNNNA", seed=9)
    ctx = {k: (int(m), int(u)) for k, m, u in zip(kmers, M, U)}
    nm, nu = int(M.sum()), int(U.sum())
    my = nm / (nm + nu)
    alpha, pen = 1.0, 4.0
    beta = (alpha * (1.0 - my)) / my

    class A:
        verbosity = 0
    sc, Mr, Ur, names = fitm.pattern_partition_bottom_up("ANNNMNNNA", ctx, alpha, beta, pen, A, nm, nu)
    rs, rm, ru, rnames, _ = O.fit("ANNNMNNNA", list(ctx), M, U, alpha, beta, pen, 32)
    assert np.float32(sc).tobytes() == np.float32(rs).tobytes()
    assert (int(Mr), int(Ur)) == (rm, ru)
    assert names == rnames
    assert len(names) > 50


def _random_case(rng, k):
    from kmerpapa_amd.pattern_utils import matches
    gp = "".join(rng.choice("NNNNMRSWKYBDHVACGT") for _ in range(k))
    ctx = {}
    for kmer in matches(gp):
        bg = rng.randrange(0, 5000) if rng.random() > 0.1 else 0
        pos = rng.randrange(0, bg + 1) // rng.choice([1, 3, 30])
        ctx[kmer] = (pos, bg - pos)
    return gp, ctx


@pytest.mark.parametrize("seed", range(6))
def test_random_patterns_vs_oracle(eng, seed):
    """Random general patterns (mixed IUPAC codes) and counts: GPU == oracle, all cells."""
    from kmerpapa_amd.CV_tools import fold_tables
    from oracle import oracle as O
    rng = random.Random(seed)
    gp, ctx = _random_case(rng, rng.choice([3, 4, 5]))
    nf = rng.choice([2, 3, 5])
    contexts, Mf, Uf = fold_tables(ctx, nf, np.random.RandomState(seed), np.uint32)
    from kmerpapa_amd.pattern_utils import generality
    Mk, Uk = eng.counts_in_kmer_order(gp, contexts, Mf, Uf, generality(gp), np.uint32)
    alpha = rng.choice([0.1, 0.5, 2.0])
    tot_m = Mf.sum(axis=0).astype(np.uint64)
    tot_u = Uf.sum(axis=0).astype(np.uint64)
    mtr = tot_m.sum() - tot_m
    utr = tot_u.sum() - tot_u
    betas = (alpha * (1.0 - mtr / (mtr + utr))) / (mtr / (mtr + utr))
    pens = [0.0, 2.5, 7.0]
    plan = eng.Plan(eng.get_device(0), gp, rng.choice([0, 64]))
    plan.set_counts(Mk, Uk)
    rt, re, _ = plan.run([(f, alpha, float(betas[f]), pens) for f in range(nf)])
    for pi, c in enumerate(pens):
        ref = O.cv_pass(gp, contexts, Mf, Uf, alpha, betas, c, 32)
        for f in range(nf):
            lane = f * len(pens) + pi
            score, _ = plan.dump_lane(lane)
            assert bits_equal(score, ref["score"][:, f]), (gp, c, f)
            assert bits_equal(re[lane], ref["root_test"][f])
    plan.close()


@pytest.mark.parametrize("seed", range(10, 14))
def test_random_6mers_vs_oracle(eng, seed):
    """Random 6-position general patterns (at most two N), 1-8 penalties per group and
    block sizes 0 (default), 128 and 1024 cells: every cell's float32 score and every
    root test value equal the oracle's, bit for bit."""
    from kmerpapa_amd.CV_tools import fold_tables
    from kmerpapa_amd.pattern_utils import generality, matches
    from oracle import oracle as O
    rng = random.Random(seed)
    codes = list("MRSWKYACGTBDHV")
    gp = "".join(rng.choice(codes) for _ in range(6))
    for i in rng.sample(range(6), 2):
        gp = gp[:i] + "N" + gp[i + 1:]
    ctx = {}
    for kmer in matches(gp):
        bg = rng.randrange(0, 20000) if rng.random() > 0.05 else 0
        pos = rng.randrange(0, bg + 1) // rng.choice([1, 10, 100])
        ctx[kmer] = (pos, bg - pos)
    nf = rng.choice([2, 4])
    contexts, Mf, Uf = fold_tables(ctx, nf, np.random.RandomState(seed), np.uint32)
    Mk, Uk = eng.counts_in_kmer_order(gp, contexts, Mf, Uf, generality(gp), np.uint32)
    alpha = rng.choice([0.3, 1.0, 4.0])
    tot_m = Mf.sum(axis=0).astype(np.uint64)
    tot_u = Uf.sum(axis=0).astype(np.uint64)
    mtr = tot_m.sum() - tot_m
    utr = tot_u.sum() - tot_u
    betas = (alpha * (1.0 - mtr / (mtr + utr))) / (mtr / (mtr + utr))
    pens = sorted(rng.sample([0.0, 1.0, 2.5, 4.0, 5.5, 7.0, 9.0, 12.0], rng.randint(1, 8)))
    plan = eng.Plan(eng.get_device(0), gp, rng.choice([0, 128, 1024]))
    plan.set_counts(Mk, Uk)
    rt, re, _ = plan.run([(f, alpha, float(betas[f]), pens) for f in range(nf)])
    for pi, c in enumerate(pens):
        ref = O.cv_pass(gp, contexts, Mf, Uf, alpha, betas, c, 32)
        for f in range(nf):
            lane = f * len(pens) + pi
            score, _ = plan.dump_lane(lane)
            assert bits_equal(score, ref["score"][:, f]), (gp, c, f)
            assert bits_equal(re[lane], ref["root_test"][f])
    plan.close()


@pytest.mark.parametrize("gp", ["ACG", "AMG", "N", "MA", "TTNTT", "RYSWKM"])
def test_degenerate_lattices_fit_vs_oracle(eng, gp):
    """Edge lattices: a single cell (no ambiguous position), one ambiguous position, a
    1-mer, all-binary codes, zero counts: the fit (score, counts, partition and order)
    equals the oracle's."""
    from kmerpapa_amd.algorithms import bottum_up_array_w_numba as fitm
    from kmerpapa_amd.pattern_utils import matches
    from oracle import oracle as O
    rng = random.Random(len(gp) * 31 + ord(gp[0]))
    ctx = {}
    for kmer in matches(gp):
        bg = rng.randrange(0, 5000) if rng.random() > 0.2 else 0
        pos = rng.randrange(0, bg + 1) // 50
        ctx[kmer] = (pos, bg - pos)
    if all(v == (0, 0) for v in ctx.values()):
        ctx[next(iter(ctx))] = (3, 1000)
    nm = sum(v[0] for v in ctx.values())
    nu = sum(v[1] for v in ctx.values())
    my = nm / (nm + nu)
    alpha, pen = 0.5, 3.0
    beta = (alpha * (1.0 - my)) / my

    class A:
        verbosity = 0
    sc, Mr, Ur, names = fitm.pattern_partition_bottom_up(gp, ctx, alpha, beta, pen, A, nm, nu)
    M = np.array([ctx[k][0] for k in ctx], np.int64)
    U = np.array([ctx[k][1] for k in ctx], np.int64)
    rs, rm, ru, rnames, _ = O.fit(gp, list(ctx), M, U, alpha, beta, pen, 32)
    assert np.float32(sc).tobytes() == np.float32(rs).tobytes()
    assert (int(Mr), int(Ur)) == (rm, ru)
    assert names == rnames


@pytest.mark.parametrize("per_wg", [1, 2, 3, 4, 6, 7, 8])
def test_lanes_per_workgroup_vs_oracle(eng, per_wg, monkeypatch):
    """Every lanes-per-workgroup kernel instantiation (KP_LANES_PER_WG; the default is 5)
    on an 8-penalty group (6 or 7 for those widths) of a small-block 5-mer, split into
    device groups of full workgroups first (8 lanes at width 3: 3 + 3 + 2): all cells equal
    the oracle's."""
    from kmerpapa_amd.CV_tools import fold_tables
    from kmerpapa_amd.pattern_utils import generality
    from oracle import oracle as O
    monkeypatch.setenv("KP_LANES_PER_WG", str(per_wg))
    rng = random.Random(100 + per_wg)
    gp, ctx = _random_case(rng, 5)
    nf = 3
    contexts, Mf, Uf = fold_tables(ctx, nf, np.random.RandomState(per_wg), np.uint32)
    Mk, Uk = eng.counts_in_kmer_order(gp, contexts, Mf, Uf, generality(gp), np.uint32)
    alpha = 1.0
    tot_m = Mf.sum(axis=0).astype(np.uint64)
    tot_u = Uf.sum(axis=0).astype(np.uint64)
    mtr = tot_m.sum() - tot_m
    utr = tot_u.sum() - tot_u
    betas = (alpha * (1.0 - mtr / (mtr + utr))) / (mtr / (mtr + utr))
    pens = [0.5, 1.5, 2.5, 3.5, 4.5, 6.0, 8.0, 11.0]
    if per_wg in (6, 7):  # one group per workgroup at these widths
        pens = pens[:per_wg]
    plan = eng.Plan(eng.get_device(0), gp, 64)
    plan.set_counts(Mk, Uk)
    rt, re, _ = plan.run([(f, alpha, float(betas[f]), pens) for f in range(nf)])
    for pi, c in enumerate(pens):
        ref = O.cv_pass(gp, contexts, Mf, Uf, alpha, betas, c, 32)
        for f in range(nf):
            lane = f * len(pens) + pi
            score, _ = plan.dump_lane(lane)
            assert bits_equal(score, ref["score"][:, f]), (gp, per_wg, c, f)
            assert bits_equal(re[lane], ref["root_test"][f])
    plan.close()


@pytest.mark.parametrize("ws", ["0", "1"])
@pytest.mark.parametrize("gp,max_block,itype,exact,alpha", [("NNMNN", 0, np.uint32, 0, 0.5), ("NNMNN", 0, np.uint32, 1, 0.5),
                                                            ("RNNNS", 64, np.uint32, 0, 0.5), ("NNNMN", 0, np.uint64, 0, 0.5),
                                                            ("NNMNN", 0, np.uint32, 0, 0.0)])
def test_1lane_sweep_vs_oracle(eng, monkeypatch, gp, max_block, itype, exact, alpha, ws):
    """Every device group cut to one lane (KP_LANES_PER_WG=1): the 1-lane build of the sweep
    (ws 0) and the opt-in persistent wave-specialised sweep for 1-lane groups (ws 1,
    kp_dp_ws.h, KP_WS=1: producer waves gather block i + 1 while consumer waves run block i's
    levels, LDS-counter hand-over; every launch above high level 0 runs on it).  Every cell of
    every lane equals the oracle, with 32- and 64-bit counts, in KP_EXACT_LOGS mode, and with
    alpha = 0 and k-mers of no counts (NaN k-mer cells)."""
    from kmerpapa_amd.CV_tools import fold_tables
    from kmerpapa_amd.pattern_utils import generality, matches
    from oracle import oracle as O
    monkeypatch.setenv("KP_WS", ws)
    monkeypatch.setenv("KP_LANES_PER_WG", "1")
    monkeypatch.setenv("KP_EXACT_LOGS", str(exact))
    rng = np.random.RandomState(len(gp) + max_block)
    scale = 1e7 if itype == np.uint64 else 2e4
    ctx = {}
    for k in matches(gp):
        bg = int(rng.poisson(scale * rng.lognormal(0, 0.5)))
        ctx[k] = (int(rng.binomial(bg, 0.01 * rng.lognormal(0, 0.4))), bg)
        if alpha == 0.0 and rng.rand() < 0.1:
            ctx[k] = (0, 0)
    if itype == np.uint64:
        assert sum(m + u for m, u in ctx.values()) > 2 ** 32
    nf = 3
    contexts, Mf, Uf = fold_tables(ctx, nf, np.random.RandomState(3), itype)
    Mk, Uk = eng.counts_in_kmer_order(gp, contexts, Mf, Uf, generality(gp), itype)
    tot_m = Mf.sum(axis=0).astype(np.uint64)
    tot_u = Uf.sum(axis=0).astype(np.uint64)
    mtr = tot_m.sum() - tot_m
    utr = tot_u.sum() - tot_u
    betas = (alpha * (1.0 - mtr / (mtr + utr))) / (mtr / (mtr + utr))
    pens = [2.0, 5.0]
    plan = eng.Plan(eng.get_device(0), gp, max_block)
    plan.set_counts(Mk, Uk)
    assert plan.info["high_levels"] > 2
    rt, re, _ = plan.run([(f, alpha, float(betas[f]), pens) for f in range(nf)])
    bits = 64 if itype == np.uint64 else 32
    for pi, c in enumerate(pens):
        ref = O.cv_pass(gp, contexts, Mf, Uf, alpha, betas, c, bits)
        for f in range(nf):
            lane = f * len(pens) + pi
            score, _ = plan.dump_lane(lane)
            assert bits_equal(score, ref["score"][:, f]), (gp, c, f)
            assert bits_equal(rt[lane], ref["root_train"][f]) and bits_equal(re[lane], ref["root_test"][f])
    plan.close()


# (lane counts of consecutive same-fold groups with alternating alphas): one mixed 5-lane
# device group (2 + 3, 4 + 1), two mixed ones (3 + 4 + 3 -> [3 + 2], [2 + 3]), and a run that
# would need three alphas in one workgroup (2 + 2 + 1), which stays one device group per alpha
MIXES = {"2+3": [2, 3], "4+1": [4, 1], "3+4+3": [3, 4, 3], "2+2+1": [2, 2, 1]}


@pytest.mark.parametrize("exact", [0, 1])
@pytest.mark.parametrize("mix", sorted(MIXES))
def test_mixed_alpha_groups_vs_oracle(eng, mix, exact, monkeypatch):
    """Lanes of several (alpha, fold) groups of the SAME fold cut together into one device
    group (kp_group_dev.nl2: the group's last lanes take a second (alpha, beta); the count
    tables are shared, the logs are per alpha), as engine.fold_pieces makes them for grids
    whose penalty count is not a multiple of the workgroup width (the 11-mer's 7): every
    cell of every lane, the root test -2LL and the backtrack (which re-derives each lane's
    decisions with its own alpha and fails on a mismatch) against the oracle run with that
    lane's alpha, for the fast-log path and KP_EXACT_LOGS."""
    from kmerpapa_amd.CV_tools import fold_tables
    from kmerpapa_amd.pattern_utils import generality
    from oracle import oracle as O
    monkeypatch.setenv("KP_EXACT_LOGS", str(exact))
    rng = random.Random(200 + len(mix) + exact)
    gp, ctx = _random_case(rng, 5)
    nf = 2
    contexts, Mf, Uf = fold_tables(ctx, nf, np.random.RandomState(7), np.uint32)
    Mk, Uk = eng.counts_in_kmer_order(gp, contexts, Mf, Uf, generality(gp), np.uint32)
    tot_m = Mf.sum(axis=0).astype(np.uint64)
    tot_u = Uf.sum(axis=0).astype(np.uint64)
    mtr = tot_m.sum() - tot_m
    utr = tot_u.sum() - tot_u
    alphas = [0.5, 4.0, 1.5]
    betas = {a: (a * (1.0 - mtr / (mtr + utr))) / (mtr / (mtr + utr)) for a in alphas}
    allpens = [0.0, 1.5, 3.0, 4.5, 6.0, 8.0, 11.0]
    groups = []
    for f in range(nf):
        for i, n in enumerate(MIXES[mix]):
            a = alphas[i % len(alphas)]
            groups.append((f, a, float(betas[a][f]), allpens[i:i + n]))
    plan = eng.Plan(eng.get_device(0), gp, 64)
    plan.set_counts(Mk, Uk)
    rt, re, _ = plan.run(groups)
    lane = 0
    refs = {}
    for f, a, b, pens in groups:
        for c in pens:
            if (a, c) not in refs:
                refs[(a, c)] = O.cv_pass(gp, contexts, Mf, Uf, a, betas[a], c, 32)
            ref = refs[(a, c)]
            score, _ = plan.dump_lane(lane)
            assert bits_equal(score, ref["score"][:, f]), (mix, f, a, c)
            assert bits_equal(rt[lane], ref["score"][-1, f])
            assert bits_equal(re[lane], ref["root_test"][f])
            lane += 1
    plan.close()


def test_error_paths(eng):
    """Errors come back as exceptions with the library's message, never as wrong numbers."""
    dev = eng.get_device(0)
    plan = eng.Plan(dev, "NMN", 0)
    with pytest.raises(eng.KPError, match="counts"):
        plan.run([(0, 1.0, 1.0, [1.0])])  # no counts set
    with pytest.raises(ValueError):
        plan.run([(0, 1.0, 1.0, [1.0] * 9)])  # more than 8 penalties in a group
    n = plan.info["n_kmers"]
    plan.counts_begin(np.full(n, 5, np.uint32), np.full(n, 50, np.uint32), 3)
    plan.run([(-1, 1.0, 1.0, [1.0])])  # fit mode needs only the all-data counts
    with pytest.raises(eng.KPError, match="fold 1 are not set"):
        plan.run([(1, 1.0, 1.0, [1.0])])
    plan.counts_fold(1, np.full(n, 2, np.uint32), np.full(n, 20, np.uint32))
    plan.run([(1, 1.0, 1.0, [1.0])])
    with pytest.raises(eng.KPError, match="fold out of range"):
        plan.counts_fold(3, np.zeros(n, np.uint32), np.zeros(n, np.uint32))
    plan.close()
    with pytest.raises(eng.KPError):
        eng.Plan(dev, "NXN", 0)  # not an IUPAC code
    with pytest.raises(eng.KPError, match="too many blocks"):
        eng.Plan(dev, "NNNNNNNNNNNN", 0)  # 15^12 cells: more blocks than 32-bit ids


def test_cli_metrics_line(eng, tmp_path, monkeypatch):
    """$KMERPAPA_METRICS: one JSON line per run with the wall-clock of every phase."""
    import json
    from kmerpapa_amd import cli
    pos, bg = write_count_files(5, str(tmp_path))
    metrics = tmp_path / "m.jsonl"
    monkeypatch.setenv("KMERPAPA_METRICS", str(metrics))
    assert cli.main(["-p", pos, "-b", bg, "-c", "3", "5", "-a", "0.5", "1", "--nfolds", "3", "--seed", "2",
                     "-o", str(tmp_path / "o.txt")]) == 0
    rec = json.loads(metrics.read_text().splitlines()[-1])
    assert set(rec["phases_s"]) == {"read_input", "pattern_and_zero_fill", "cross_validation", "final_fit", "output"}
    assert rec["gen_pat"] == "NNMNN" and rec["patterns"] > 1
    assert abs(sum(rec["phases_s"].values()) - rec["total_s"]) < 0.05


def test_device_log_vs_libm(eng):
    """The DP's device log (ROCm ocml, through kp_math_log) against the host C library's
    log, which the oracle and the reference call: within 1 ulp everywhere; on the DP's range
    (p and 1 - p in (0, 1)) they differ in the last bit on about 4 % of inputs (measured
    3.9 %).  A 1-ulp change of a log moves a cell's float32 single-pattern term with
    probability ~1e-9; the parity tests proper compare the float32 scores,
    bit for bit."""
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    libm.log.argtypes = [ctypes.c_double]
    libm.log.restype = ctypes.c_double
    rng = np.random.RandomState(3)
    n = 100_000
    x = np.concatenate([rng.uniform(0.0, 1.0, n), 1.0 - rng.uniform(0.0, 0.07, n),
                        np.exp(rng.uniform(-745.0, 709.0, n)),
                        np.array([1.0, np.inf, 5e-324, 2.2250738585072014e-308, np.nextafter(1.0, 0)])])
    got = eng.get_device(0).log(x)
    want = np.array([libm.log(float(v)) for v in x])
    ulps = np.abs(got.view(np.int64) - want.view(np.int64))
    assert ulps.max() <= 1, x[np.argmax(ulps)]
    assert np.mean(ulps[:2 * n] != 0) < 0.1  # p, 1 - p: last-bit differences on ~4 %
    assert np.isneginf(eng.get_device(0).log(np.array([0.0]))[0])


def test_device_fast_log_within_1ulp(eng):
    """The table-free fdlibm log (kp_fast_log, fn 3 of kp_math_libm; the sweep's fast-path
    log in -DKP_FAST_LOG builds) on the GPU against the box's C library: within 1 ulp on
    the DP's range and across the whole normal range, as the store guard's premise needs
    (<= 2 ulp; kp_core.h kp_store_unsafe)."""
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    libm.log.argtypes = [ctypes.c_double]
    libm.log.restype = ctypes.c_double
    rng = np.random.RandomState(8)
    n = 100_000
    x = np.concatenate([rng.uniform(0.0, 1.0, n), 1.0 - rng.uniform(0.0, 0.07, n), rng.uniform(0.0, 1e-3, n),
                        np.exp(rng.uniform(-700.0, 709.0, n)),
                        np.array([1.0, 2.0, 0.5, 2.2250738585072014e-308, np.nextafter(1.0, 0), np.nextafter(1.0, 2)])])
    got = eng.get_device(0).libm(x, 3)
    want = np.array([libm.log(float(v)) for v in x])
    ulps = np.abs(got.view(np.int64) - want.view(np.int64))
    assert ulps.max() <= 1, x[np.argmax(ulps)]
    assert np.isneginf(eng.get_device(0).libm(np.array([0.0]), 3)[0])


def test_device_fma_log_within_2ulp(eng):
    """kp_fma_log (fn 4 of kp_math_libm: fdlibm's algorithm with the hardware reciprocal,
    Newton steps and fused multiply-adds; the sweep's fast-path log in -DKP_FMA_LOG builds)
    on the GPU against the box's C library: within 2 ulp on the DP's range and across the
    whole normal range -- the store guard's premise (kp_core.h kp_store_unsafe)."""
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    libm.log.argtypes = [ctypes.c_double]
    libm.log.restype = ctypes.c_double
    rng = np.random.RandomState(9)
    n = 100_000
    u = rng.uniform(0.0, 1.0, n)
    x = np.concatenate([u, 1.0 - u, u * 1e-6, 1.0 - u * 1e-6, 1.0 - rng.uniform(0.0, 0.07, n),
                        np.exp(rng.uniform(-700.0, 709.0, n)),
                        np.array([1.0, 2.0, 0.5, 2.2250738585072014e-308, np.nextafter(1.0, 0), np.nextafter(1.0, 2)])])
    got = eng.get_device(0).libm(x, 4)
    want = np.array([libm.log(float(v)) for v in x])
    ulps = np.abs(got.view(np.int64) - want.view(np.int64))
    assert ulps.max() <= 2, (x[np.argmax(ulps)], ulps.max())
    special = np.array([0.0, -1.0, np.inf, np.nan, 5e-324])
    assert np.array_equal(eng.get_device(0).libm(special, 4), eng.get_device(0).libm(special, 1), equal_nan=True)


def test_uint64_counts_multilevel_vs_oracle(eng):
    """Counts whose total exceeds 2^32 - 1 take the reference's uint64 itype (CV :94-97):
    the 64-bit count tables and kernels (their larger LDS tables put 4 lanes in a workgroup
    instead of 5) on a 2.3e6-cell lattice with four high levels, 2 folds x 5 penalties:
    every cell's float32 score and every root, bit for bit against the 64-bit oracle."""
    from kmerpapa_amd.CV_tools import fold_tables
    from kmerpapa_amd.pattern_utils import generality, matches
    from oracle import oracle as O
    gp = "NNNMNN"
    rng = np.random.RandomState(17)
    ctx = {}
    for kmer in matches(gp):
        bg = int(rng.randint(1_000_000, 4_000_000))
        ctx[kmer] = (int(rng.binomial(bg, 2e-4)), bg)
    assert sum(m + u for m, u in ctx.values()) > 2**32
    nf = 2
    contexts, Mf, Uf = fold_tables(ctx, nf, np.random.RandomState(2), np.uint64)
    Mk, Uk = eng.counts_in_kmer_order(gp, contexts, Mf, Uf, generality(gp), np.uint64)
    alpha = 0.7
    tot_m = Mf.sum(axis=0).astype(np.uint64)
    tot_u = Uf.sum(axis=0).astype(np.uint64)
    mtr = tot_m.sum() - tot_m
    utr = tot_u.sum() - tot_u
    betas = (alpha * (1.0 - mtr / (mtr + utr))) / (mtr / (mtr + utr))
    pens = [1.0, 3.0, 5.0, 7.0, 9.0]
    plan = eng.Plan(eng.get_device(0), gp, 0)
    assert plan.info["high_levels"] > 3
    plan.set_counts(Mk, Uk)
    rt, re, _ = plan.run([(f, alpha, float(betas[f]), pens) for f in range(nf)])
    for pi, c in enumerate(pens):
        ref = O.cv_pass(gp, contexts, Mf, Uf, alpha, betas, c, 64)
        for f in range(nf):
            lane = f * len(pens) + pi
            score, _ = plan.dump_lane(lane)
            assert bits_equal(score, ref["score"][:, f]), (c, f)
            assert bits_equal(rt[lane], ref["root_train"][f]) and bits_equal(re[lane], ref["root_test"][f])
    plan.close()


def test_device_libm_exact(eng):
    """The C library's log and log1p as restated for the GPU (kp_libm.h: the sweep's exact
    fallback, the backtrack's single terms, the k-mer cells' xlogy / xlog1py) equal this
    box's C library bit for bit, on the DP's ranges and across the float64 range."""
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    fns = {}
    for name in ("log", "log1p"):
        f = getattr(libm, name)
        f.argtypes = [ctypes.c_double]
        f.restype = ctypes.c_double
        fns[name] = f
    rng = np.random.RandomState(21)
    n = 200_000
    nans = np.array([0x7ff8000000000000, 0xfff8000000000000, 0x7ff8000000000123], np.uint64).view(np.float64)
    x = np.concatenate([rng.uniform(0.0, 1.0, n), 1.0 - rng.uniform(0.0, 1e-3, n), 1.0 + rng.uniform(-0.07, 0.07, n),
                        np.exp(rng.uniform(-745.0, 709.0, n)), nans,
                        np.array([0.0, 1.0, np.inf, 5e-324, np.nextafter(1.0, 0)])])
    dev = eng.get_device(0)
    for fn, name, xs in ((1, "log", x), (2, "log1p", np.concatenate([-x[:2 * n], x[2 * n:], [-1.0]]))):
        got = dev.libm(xs, fn)
        want = np.array([fns[name](float(v)) for v in xs])
        same = got.view(np.int64) == want.view(np.int64)  # NaNs too (an input NaN propagates)
        assert same.all(), (name, xs[~same][:5])
    # negative arguments (never reached by the DP: p, 1 - p in [0, 1]) give a NaN of the
    # hardware's own default encoding
    assert np.isnan(dev.libm(np.array([-1.0, -2.5]), 1)).all()


@pytest.mark.parametrize("seed", [30, 31])
def test_exact_logs_mode_same_scores(eng, seed, monkeypatch):
    """KP_EXACT_LOGS=1 (every cell's single term from the C library's logs, no fast device
    log) gives the same float32 scores as the default guarded fast path and as the oracle:
    the fallback path itself is right, and the fast path's guard lets nothing through."""
    from kmerpapa_amd.CV_tools import fold_tables
    from kmerpapa_amd.pattern_utils import generality
    from oracle import oracle as O
    rng = random.Random(seed)
    gp, ctx = _random_case(rng, 5)
    nf = 3
    contexts, Mf, Uf = fold_tables(ctx, nf, np.random.RandomState(seed), np.uint32)
    Mk, Uk = eng.counts_in_kmer_order(gp, contexts, Mf, Uf, generality(gp), np.uint32)
    alpha = 0.5
    tot_m = Mf.sum(axis=0).astype(np.uint64)
    tot_u = Uf.sum(axis=0).astype(np.uint64)
    mtr, utr = tot_m.sum() - tot_m, tot_u.sum() - tot_u
    betas = (alpha * (1.0 - mtr / (mtr + utr))) / (mtr / (mtr + utr))
    pens = [0.0, 3.0, 6.5]
    groups = [(f, alpha, float(betas[f]), pens) for f in range(nf)]
    scores = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("KP_EXACT_LOGS", mode)
        plan = eng.Plan(eng.get_device(0), gp, 64)
        plan.set_counts(Mk, Uk)
        rt, re, _ = plan.run(groups)
        scores[mode] = [plan.dump_lane(ln)[0] for ln in range(nf * len(pens))] + [rt, re]
        plan.close()
    for a, b in zip(scores["0"], scores["1"]):
        assert bits_equal(a, b)
    for pi, c in enumerate(pens):
        ref = O.cv_pass(gp, contexts, Mf, Uf, alpha, betas, c, 32)
        for f in range(nf):
            assert bits_equal(scores["1"][f * len(pens) + pi], ref["score"][:, f])


def test_zero_pseudo_count_nan_bits_vs_oracle(eng):
    """alpha = 0 with empty k-mers makes p = 0/0 (NaN) in some cells: every stored float32
    equals the oracle's bit for bit, NaN encodings included (the C library's log lets an
    input NaN through unchanged, and so must the GPU's restatement)."""
    from kmerpapa_amd.CV_tools import fold_tables
    from kmerpapa_amd.pattern_utils import generality
    from oracle import oracle as O
    rng = random.Random(77)
    gp, ctx = _random_case(rng, 5)
    for kmer in list(ctx)[::7]:
        ctx[kmer] = (0, 0)
    nf = 3
    contexts, Mf, Uf = fold_tables(ctx, nf, np.random.RandomState(77), np.uint32)
    Mk, Uk = eng.counts_in_kmer_order(gp, contexts, Mf, Uf, generality(gp), np.uint32)
    tot_m = Mf.sum(axis=0).astype(np.uint64)
    tot_u = Uf.sum(axis=0).astype(np.uint64)
    mtr, utr = tot_m.sum() - tot_m, tot_u.sum() - tot_u
    betas = (0.0 * (1.0 - mtr / (mtr + utr))) / (mtr / (mtr + utr))
    pens = [0.0, 4.0]
    plan = eng.Plan(eng.get_device(0), gp, 0)
    plan.set_counts(Mk, Uk)
    plan.run([(f, 0.0, float(betas[f]), pens) for f in range(nf)])
    nan_seen = False
    for pi, c in enumerate(pens):
        ref = O.cv_pass(gp, contexts, Mf, Uf, 0.0, betas, c, 32)
        for f in range(nf):
            score, _ = plan.dump_lane(f * len(pens) + pi)
            assert np.array_equal(score.view(np.uint32), ref["score"][:, f].view(np.uint32)), (c, f)
            nan_seen = nan_seen or bool(np.isnan(score).any())
    plan.close()
    assert nan_seen


def test_negative_penalty_takes_exact_logs(eng):
    """A group outside the fast path's premise (a negative penalty: the single term's parts
    no longer all >= 0) takes the C library's logs for every cell: still the oracle's
    scores bit for bit."""
    from kmerpapa_amd.CV_tools import fold_tables
    from kmerpapa_amd.pattern_utils import generality
    from oracle import oracle as O
    rng = random.Random(91)
    gp, ctx = _random_case(rng, 5)
    nf = 2
    contexts, Mf, Uf = fold_tables(ctx, nf, np.random.RandomState(91), np.uint32)
    Mk, Uk = eng.counts_in_kmer_order(gp, contexts, Mf, Uf, generality(gp), np.uint32)
    alpha = 0.5
    tot_m = Mf.sum(axis=0).astype(np.uint64)
    tot_u = Uf.sum(axis=0).astype(np.uint64)
    mtr, utr = tot_m.sum() - tot_m, tot_u.sum() - tot_u
    betas = (alpha * (1.0 - mtr / (mtr + utr))) / (mtr / (mtr + utr))
    pens = [-2.0, 3.0]
    plan = eng.Plan(eng.get_device(0), gp, 0)
    plan.set_counts(Mk, Uk)
    plan.run([(f, alpha, float(betas[f]), pens) for f in range(nf)])
    for pi, c in enumerate(pens):
        ref = O.cv_pass(gp, contexts, Mf, Uf, alpha, betas, c, 32)
        for f in range(nf):
            score, _ = plan.dump_lane(f * len(pens) + pi)
            assert np.array_equal(score.view(np.uint32), ref["score"][:, f].view(np.uint32)), (c, f)
    plan.close()


def test_fold_tables_fill_beside_passes(eng):
    """kp_counts_fold is asynchronous (the plan's count stream, one event per fold that the
    fold's passes wait on) and engine.run_groups queues each fold from a feeder thread as it
    arrives, so fold f + 1's table fills while fold f's pass runs.  With folds arriving
    15 ms apart over 25 ms passes, the roots equal those of the all-folds-at-once upload
    (kp_set_counts), bit for bit."""
    import threading
    import time
    from kmerpapa_amd.pattern_utils import generality
    gp, nf = "NNNNMNNN", 4
    rng = np.random.RandomState(11)
    nk = generality(gp)
    Mk = rng.randint(0, 60, size=(nk, nf)).astype(np.uint32)
    Uk = rng.randint(60, 2000, size=(nk, nf)).astype(np.uint32)
    groups = [(f, a, 1.0 + 0.1 * f + 0.01 * a, [2.0, 3.0, 4.0, 5.0, 6.0]) for a in (1.0, 3.0) for f in range(nf)]
    plan = eng.get_plan(0, gp)
    plan.set_counts(Mk, Uk)
    want = plan.run(groups)
    feed = eng.FoldFeed(Mk.sum(axis=1, dtype=np.uint32), Uk.sum(axis=1, dtype=np.uint32), nf)

    def produce():
        for f in range(nf):
            time.sleep(0.015)
            feed.put(f, Mk[:, f].copy(), Uk[:, f].copy())
    th = threading.Thread(target=produce)
    th.start()
    got = eng.run_groups(gp, feed, None, groups, devices=[0])
    th.join()
    for w, g in zip(want[:2], got[:2]):
        assert bits_equal(g, w)
    assert np.array_equal(want[2], got[2])

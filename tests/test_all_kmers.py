"""--score all_kmers (one rate per k-mer; reference
src/kmerpapa/algorithms/all_kmers_CV.py :8-63).

CPU: the oracle restatement (oracle/allkmers.py) reproduces the per-alpha test losses the
reference printed in its own CLI runs on its 5-mer test data (tests/golden/allk5.json,
make_golden.py job allk5), digit for digit.
GPU: the product path (kp_allkmers_cv, csrc/kp_allk.h) -- the CLI's output table and
stderr byte-identical to those runs, and the float64 loss sums bit-identical to the
oracle on the 9-mer benchmark counts (131,072 k-mers) and on edge cases (alpha = 0 with
empty k-mers: 0/0 rates, NaN sums, compared with the oracle's per-row evaluation as the
reference's loop runs it)."""
import numpy as np
import pytest

from tests.fixtures import context_table, golden_json, write_count_files

G = golden_json("allk5.json")


def _argv_value(argv, flag, n=1):
    i = argv.index(flag)
    return argv[i + 1:i + 1 + n]


@pytest.mark.parametrize("run", ["grid", "iter"])
def test_oracle_all_kmers_losses_match_reference(run):
    if G is None:
        pytest.skip("all_kmers golden not generated")
    from kmerpapa_amd.CV_tools import make_all_folds_contextD_kmers
    from kmerpapa_amd.pattern_utils import generality
    from kmerpapa_amd.score_utils import get_betas
    from oracle import allkmers as OA
    g = G[run]
    argv = g["argv"]
    i = argv.index("-a")
    alphas = []
    for tok in argv[i + 1:]:
        if tok.startswith("-"):
            break
        alphas.append(float(tok))
    nf = int(_argv_value(argv, "--nfolds")[0])
    seed = int(_argv_value(argv, "--seed")[0])
    nit = int(_argv_value(argv, "-i")[0]) if "-i" in argv else 1
    ctx, gp, _, _ = context_table(5)
    n = generality(gp)
    M_mem = np.zeros((n, nf), np.uint64)
    U_mem = np.zeros((n, nf), np.uint64)
    prng = np.random.RandomState(seed)
    test_loss = {a: [] for a in alphas}
    for _ in range(nit):
        make_all_folds_contextD_kmers(ctx, U_mem, M_mem, gp, prng)
        ms, us = M_mem.sum(axis=0), U_mem.sum(axis=0)
        mtr, utr = sum(ms) - ms, sum(us) - us
        betas = np.array([get_betas(a, mtr, utr) for a in alphas])
        _, te = OA.allkmers_sums(M_mem, U_mem, alphas, betas)
        for a_i, a in enumerate(alphas):
            test_loss[a].extend(list(te[a_i]))
    got = [f"alpha={a} test_loss={sum(test_loss[a]) / nit}" for a in alphas]
    want = [ln for ln in g["stderr"].splitlines() if ln.startswith("alpha=")]
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("run", ["grid", "iter"])
def test_all_kmers_cli_matches_reference(run, tmp_path, capsys):
    if G is None:
        pytest.skip("all_kmers golden not generated")
    from kmerpapa_amd import cli
    g = G[run]
    pos, bg = write_count_files(5, str(tmp_path))
    argv = list(g["argv"])
    argv[argv.index("-p") + 1] = str(pos)
    argv[argv.index("-b") + 1] = str(bg)
    out = tmp_path / "out.txt"
    rc = cli.main(argv + ["-o", str(out)])
    err = capsys.readouterr().err
    assert rc == g["rc"]
    assert out.read_text() == g["output"]
    want = [ln for ln in g["stderr"].splitlines() if ln.startswith(("alpha=", "CV DONE", "LL=", "loss="))]
    got = [ln for ln in err.splitlines() if ln.startswith(("alpha=", "CV DONE", "LL=", "loss="))]
    assert got == want


def _bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


@pytest.mark.gpu
def test_all_kmers_gpu_sums_vs_oracle_9mer():
    """The benchmark's synthetic 9-mer counts (131,072 k-mers), 5 folds, 5 pseudo counts:
    every (alpha, fold) train and test sum equals the oracle's bit for bit."""
    import bench
    from kmerpapa_amd import engine
    from kmerpapa_amd.CV_tools import make_all_folds_contextD_kmers
    from kmerpapa_amd.score_utils import get_betas
    from oracle import allkmers as OA
    kmers, M, U = bench.synthetic_counts("NNNNMNNNN", seed=9)
    ctx = {k: (int(m), int(u)) for k, m, u in zip(kmers, M, U)}
    nf, alphas = 5, [0.5, 1.0, 2.0, 5.0, 10.0]
    M_mem = np.zeros((len(kmers), nf), np.uint64)
    U_mem = np.zeros((len(kmers), nf), np.uint64)
    make_all_folds_contextD_kmers(ctx, U_mem, M_mem, "NNNNMNNNN", np.random.RandomState(1))
    ms, us = M_mem.sum(axis=0), U_mem.sum(axis=0)
    betas = np.array([get_betas(a, sum(ms) - ms, sum(us) - us) for a in alphas])
    dev = engine.get_device(engine.visible_devices()[0])
    tr, te = dev.allkmers_cv(M_mem, U_mem, alphas, betas)
    otr, ote = OA.allkmers_sums(M_mem, U_mem, alphas, betas)
    assert np.array_equal(_bits(tr), _bits(otr)) and np.array_equal(_bits(te), _bits(ote))


@pytest.mark.gpu
def test_all_kmers_gpu_edge_cases_vs_oracle():
    """alpha = 0 with k-mers whose counts are all zero (p = 0/0 -> NaN terms), a k-mer with
    positives only, one fold holding everything, and no k-mers at all: bit-identical to the
    oracle (NaN payloads included)."""
    from kmerpapa_amd import engine
    from oracle import allkmers as OA
    rng = np.random.RandomState(5)
    n, nf = 4099, 3
    M = rng.poisson(3.0, size=(n, nf)).astype(np.uint64)
    U = rng.poisson(2000.0, size=(n, nf)).astype(np.uint64)
    M[:50] = 0
    U[:50] = 0
    U[50:60] = 0
    M[60:70, 1:] = 0
    U[60:70, 1:] = 0
    alphas = [0.0, 0.3, 4.0]
    betas = np.array([[0.0, 0.0, 0.0], [1e4, 2e4, 3e4], [5e5, 6e5, 7e5]])
    dev = engine.get_device(engine.visible_devices()[0])
    tr, te = dev.allkmers_cv(M, U, alphas, betas)
    otr, ote = OA.allkmers_sums(M, U, alphas, betas, per_row=True)  # the reference's per-k-mer rows
    assert np.isnan(tr[0]).any()
    assert np.array_equal(_bits(tr), _bits(otr)) and np.array_equal(_bits(te), _bits(ote))
    e_tr, e_te = dev.allkmers_cv(np.zeros((0, nf), np.uint64), np.zeros((0, nf), np.uint64), alphas, betas)
    assert (e_tr == 0).all() and (e_te == 0).all()

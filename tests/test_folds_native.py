"""The C++ fold split (kp_fold_split, kmerpapa_amd/csrc/kp_folds.h) against numpy itself:
same folds and the same final MT19937 state as the reference's colour-by-colour
RandomState.hypergeometric walk (CV_tools.py:5-62), for small and huge counts, zero
colours, HYP (sample <= 10) and HRUA draws.  Host code: no GPU needed."""
import numpy as np
import pytest

from kmerpapa_amd import engine
from kmerpapa_amd.CV_tools import _split_colors_numpy


def _pair(colors, nf, seed, itype=np.uint64):
    p1, p2 = np.random.RandomState(seed), np.random.RandomState(seed)
    a = _split_colors_numpy(np.asarray(colors, dtype=itype), nf, itype, p1)
    b = engine.fold_split(np.asarray(colors, dtype=itype), nf, p2)
    s1, s2 = p1.get_state(), p2.get_state()
    return a, b, s1, s2


@pytest.mark.parametrize("kind", range(6))
def test_fold_split_matches_numpy_stream(kind):
    rng = np.random.RandomState(100 + kind)
    for trial in range(60):
        n = int(rng.randint(1, 80))
        if kind == 0:
            colors = rng.randint(0, 12, size=n)            # mostly HYP draws
        elif kind == 1:
            colors = rng.randint(0, 5000, size=n)
        elif kind == 2:
            colors = rng.randint(0, 2 ** 31, size=n) // (1 + rng.randint(0, 1000, size=n))
        elif kind == 3:
            colors = np.where(rng.rand(n) < 0.4, 0, rng.randint(0, 10 ** 7, size=n))
        elif kind == 4:
            colors = rng.randint(0, 2 ** 33, size=n)      # > 2^32 totals (uint64 itype)
        else:
            colors = rng.randint(7800, 8600, size=n)      # loggam arguments either side of its table
        nf = int(rng.randint(1, 8))
        a, b, s1, s2 = _pair(colors, nf, int(rng.randint(0, 2 ** 31)))
        assert np.array_equal(a, b), (kind, trial)
        assert np.array_equal(s1[1], s2[1]) and s1[2] == s2[2], "RandomState advanced differently"


def test_fold_split_edge_cases():
    for colors in ([0], [5], [0, 0, 0], [1, 0, 0, 7], [10 ** 9, 1]):
        for nf in (1, 2, 5):
            a, b, s1, s2 = _pair(colors, nf, 3)
            assert np.array_equal(a, b)
            assert np.array_equal(s1[1], s2[1]) and s1[2] == s2[2]


def test_fold_split_continues_the_callers_stream():
    """Two successive splits on one RandomState (CV iterations) stay in lock step."""
    colors = np.random.RandomState(1).randint(0, 3000, size=500).astype(np.uint64)
    p1, p2 = np.random.RandomState(9), np.random.RandomState(9)
    for _ in range(3):
        assert np.array_equal(_split_colors_numpy(colors, 4, np.uint64, p1), engine.fold_split(colors, 4, p2))
    assert p1.randint(0, 2 ** 30) == p2.randint(0, 2 ** 30)


@pytest.mark.parametrize("nf", [2, 3, 5, 10])
def test_fold_stream_matches_fold_tables(nf):
    """CV_tools.fold_stream (one kp_fold_sample per fold, the CV driver's pipelined split)
    draws exactly fold_tables' folds and leaves the stream in the same state."""
    from kmerpapa_amd.CV_tools import fold_stream, fold_tables
    rng = np.random.RandomState(nf)
    ctx = {}
    for _ in range(400):
        ctx["".join(rng.choice(list("ACGT"), 6))] = (int(rng.randint(0, 40)), int(rng.randint(0, 5000)))
    for itype in (np.uint32, np.uint64):
        p1, p2 = np.random.RandomState(11), np.random.RandomState(11)
        _, M, U = fold_tables(ctx, nf, p1, itype)
        got = list(fold_stream(ctx, nf, p2, itype))
        assert [g[0] for g in got] == list(range(nf))
        for f, Mf, Uf in got:
            assert Mf.dtype == itype and np.array_equal(Mf, M[:, f]) and np.array_equal(Uf, U[:, f])
        s1, s2 = p1.get_state(), p2.get_state()
        assert np.array_equal(s1[1], s2[1]) and s1[2] == s2[2]


def test_fold_split_vector_and_scalar_paths_agree():
    """kp_folds.h evaluates HRUA's d10 and first candidate as two AVX2 + FMA chains when the
    host has them (loggam_sum4_pair), else with the scalar loggam: both give numpy's draws.
    Here: a 9-mer-sized split (131,072 k-mers' M and U colours, counts up to ~1e5, totals
    ~2.7e9) in two processes, one forced scalar (KP_FOLDS_SCALAR=1): identical folds."""
    import hashlib
    import os
    import subprocess
    import sys
    code = ("import numpy as np, hashlib; from kmerpapa_amd import engine; "
            "r = np.random.RandomState(5); c = np.concatenate([r.poisson(0.5, 131072), r.poisson(2e4, 131072)]); "
            "print(hashlib.sha1(engine.fold_split(c.astype(np.uint64), 5, np.random.RandomState(1)).tobytes()).hexdigest())")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    for scalar in (False, True):
        env = dict(os.environ)
        env.pop("KP_FOLDS_SCALAR", None)
        if scalar:
            env["KP_FOLDS_SCALAR"] = "1"
        outs.append(subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True,
                                   check=True).stdout.strip())
    assert outs[0] == outs[1] and len(outs[0]) == 40
    assert hashlib.sha1(b"").hexdigest() not in outs

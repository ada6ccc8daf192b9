"""Pins the CPU oracle (oracle/kp_oracle.c) to vectors the reference itself produced:
every cell's float32 train/test score, aggregated counts and back-pointers, bit for bit
(any NaN equals any NaN: the reference's NaN sign from 0/0 is meaningless)."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.fixtures import bits_equal, golden_json, golden_npz

SMALL = golden_json("small_dp.json")
CASES = ["k3", "k4", "k3zero", "k3big"]


@pytest.mark.parametrize("case", CASES)
def test_oracle_cv_full_arrays(case):
    c = SMALL["cases"][case]
    A = golden_npz("small_dp.npz")
    bits = 64 if c["itype"] == "uint64" else 32
    kmers = [str(x) for x in A[f"{case}_kmers"]]
    for j, ps in enumerate(c["passes"]):
        r = O.cv_pass(c["gen_pat"], kmers, A[f"{case}_Mf"], A[f"{case}_Uf"], ps["alpha"], ps["betas"],
                      ps["penalty"], bits)
        assert bits_equal(r["score"], A[f"{case}_{j}_score"])
        assert bits_equal(r["test"], A[f"{case}_{j}_test"])
        assert np.array_equal(r["M"], A[f"{case}_{j}_M"].astype(np.uint64))
        assert np.array_equal(r["U"], A[f"{case}_{j}_U"].astype(np.uint64))


@pytest.mark.parametrize("case", CASES)
def test_oracle_fit(case):
    c = SMALL["cases"][case]
    A = golden_npz("small_dp.npz")
    bits = 64 if c["itype"] == "uint64" else 32
    ctx = c["contextD"]
    ks = sorted(ctx)
    M0 = [ctx[k][0] for k in ks]
    U0 = [ctx[k][1] for k in ks]
    for j, fo in enumerate(c["fits"]):
        if "error" in fo:
            continue
        sc, M, U, names, arrs = O.fit(c["gen_pat"], ks, M0, U0, fo["alpha"], fo["beta"], fo["penalty"], bits)
        assert float(sc) == fo["score"] and M == fo["M"] and U == fo["U"]
        assert names == fo["names"]
        assert bits_equal(arrs["score"], A[f"{case}_fit_{j}_score"])
        assert np.array_equal(arrs["backtrack"], A[f"{case}_fit_{j}_backtrack"])


def test_oracle_fit5_partitions():
    from tests.fixtures import context_table
    g = golden_json("fit5.json")
    ctx, gp, nm, nu = context_table(5)
    ks = sorted(ctx)
    for fo in g["fits"]:
        sc, M, U, names, _ = O.fit(gp, ks, [ctx[k][0] for k in ks], [ctx[k][1] for k in ks], fo["alpha"],
                                   fo["beta"], fo["penalty"], 32)
        assert float(sc) == fo["score"]
        assert names == fo["names"]


def test_oracle_grid5_roots():
    """Config 2 through the oracle: per-fold root train/test of all 9 (alpha, c)."""
    g = golden_json("grid5.json")
    F = golden_npz("folds.npz")
    kmers = [str(x) for x in F["kmers5"]]
    for ps in g["passes"][:3]:  # 3 of the 9 passes keep the CPU suite short
        r = O.cv_pass(g["gen_pat"], kmers, F["M5"], F["U5"], ps["alpha"], ps["betas"], ps["penalty"], 32)
        assert bits_equal(r["root_train"], np.array(ps["root_train"], np.float32))
        assert bits_equal(r["root_test"], np.array(ps["root_test"], np.float32))


def test_oracle_cv7_roots_vs_reference():
    """Config 3 (7-mer test data, 34,171,875 cells, 5 folds) through the oracle: per-fold
    root train/test values of two of the grid's nine (alpha, c) points equal the reference's
    own (tests/golden/cv7.json, one reference process per point, make_golden.py cv7p_*).
    The oracle runs each level over the host's cores (same values as one thread)."""
    import os
    g = golden_json("cv7.json")
    if g is None:
        pytest.skip("cv7 golden not generated")
    F = golden_npz("folds.npz")
    kmers = [str(x) for x in F["kmers7"]]
    threads = max(1, min(8, len(os.sched_getaffinity(0))))
    for ps in (g["passes"][0], g["passes"][-1]):
        r = O.cv_pass(g["gen_pat"], kmers, F["M7"], F["U7"], ps["alpha"], ps["betas"], ps["penalty"], 32,
                      threads=threads)
        assert bits_equal(r["root_train"], np.array(ps["root_train"], np.float32))
        assert bits_equal(r["root_test"], np.array(ps["root_test"], np.float32))

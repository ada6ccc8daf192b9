"""Pins the pure-Python restatement (oracle/pyref.py, the reference-equivalent Python path
bench.py's cpu_baseline times) to the vectors the reference itself produced and to the C
oracle, bit for bit."""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import pyref
from tests.fixtures import bits_equal, golden_json, golden_npz

SMALL = golden_json("small_dp.json")


@pytest.mark.parametrize("case", ["k3", "k4", "k3zero", "k3big"])
def test_pyref_cv_full_arrays_vs_reference(case):
    c = SMALL["cases"][case]
    A = golden_npz("small_dp.npz")
    bits = 64 if c["itype"] == "uint64" else 32
    kmers = [str(x) for x in A[f"{case}_kmers"]]
    nf = A[f"{case}_Mf"].shape[1]
    for j, ps in enumerate(c["passes"][:2]):
        M = O._scatter(c["gen_pat"], kmers, A[f"{case}_Mf"], nf)
        U = O._scatter(c["gen_pat"], kmers, A[f"{case}_Uf"], nf)
        score, test = pyref.cv_pass(c["gen_pat"], M, U, ps["alpha"], ps["betas"], ps["penalty"], bits)
        assert bits_equal(score, A[f"{case}_{j}_score"])
        assert bits_equal(test, A[f"{case}_{j}_test"])
        assert np.array_equal(M, A[f"{case}_{j}_M"].astype(np.uint64))


def test_pyref_vs_oracle_5mer_grid_point():
    """Config 2's lattice (NNMNN, 151,875 cells, 5 folds of the reference's test data): full
    arrays equal the C oracle's and the roots equal the reference's (grid5.json)."""
    g = golden_json("grid5.json")
    F = golden_npz("folds.npz")
    kmers = [str(x) for x in F["kmers5"]]
    ps = g["passes"][4]
    M = O._scatter(g["gen_pat"], kmers, F["M5"], 5)
    U = O._scatter(g["gen_pat"], kmers, F["U5"], 5)
    score, test = pyref.cv_pass(g["gen_pat"], M, U, ps["alpha"], ps["betas"], ps["penalty"], 32)
    r = O.cv_pass(g["gen_pat"], kmers, F["M5"], F["U5"], ps["alpha"], ps["betas"], ps["penalty"], 32)
    assert bits_equal(score, r["score"]) and bits_equal(test, r["test"])
    root = O.cell_index(g["gen_pat"], g["gen_pat"])
    assert bits_equal(test[root], np.array(ps["root_test"], np.float32))
    assert bits_equal(score[root], np.array(ps["root_train"], np.float32))

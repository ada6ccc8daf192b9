"""ctypes front-end of the CPU oracle (``kp_oracle.c``).

TEST INFRASTRUCTURE ONLY: imported by tests/, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of bench.py -- never by the product package ``kmerpapa_amd``.
It is deliberately self-contained (its own IUPAC tables and index arithmetic) so the
checker does not share code with the thing it checks.

Reference functions restated here:
  * backtrack / get_right  -- src/kmerpapa/algorithms/bottum_up_array_w_numba.py:8-24
  * CV root read-out        -- bottum_up_array_penalty_plus_pseudo_CV.py:158-163
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(HERE, "libkp_oracle.so")

_PERM = {"A": "A", "C": "C", "G": "G", "T": "T", "R": "AGR", "Y": "CTY", "S": "GCS",
         "W": "ATW", "K": "GTK", "M": "ACM", "B": "CGTSYKB", "D": "AGTRWKD",
         "H": "ACTMWYH", "V": "ACGMRSV", "N": "ACGTRYSWKMBDHVN"}
_SPLIT = {"R": "AG", "Y": "CT", "S": "GC", "W": "AT", "K": "GT", "M": "AC",
          "V": "AS CR GM", "H": "AY CW TM", "D": "AK GW TR", "B": "CK GY TS",
          "N": "SW KM RY AB CD GH TV"}

_lib = None


def build():
    """Compile ``libkp_oracle.so`` (gcc, no FMA contraction)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        f32p = ctypes.POINTER(ctypes.c_float)
        f64p = ctypes.POINTER(ctypes.c_double)
        L.kpo_npat.argtypes = [ctypes.c_char_p]
        L.kpo_npat.restype = ctypes.c_uint64
        L.kpo_cv.argtypes = [ctypes.c_char_p, ctypes.c_int, u64p, u64p, ctypes.c_int, ctypes.c_double,
                             f64p, ctypes.c_double, f32p, f32p, ctypes.c_int]
        L.kpo_cv.restype = ctypes.c_int
        L.kpo_fit.argtypes = [ctypes.c_char_p, u64p, u64p, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                              ctypes.c_double, f32p, u64p, ctypes.c_int]
        L.kpo_fit.restype = ctypes.c_int
        L.kpo_cv_lane.argtypes = [ctypes.c_char_p, ctypes.c_uint64, u64p, u64p, u64p, ctypes.c_int,
                                  ctypes.c_double, ctypes.c_double, ctypes.c_double, f32p, ctypes.c_int]
        L.kpo_cv_lane.restype = ctypes.c_int
        L.kpo_libm_array.argtypes = [f64p, f64p, ctypes.c_uint64, ctypes.c_int]
        L.kpo_libm_array.restype = None
        _lib = L
    return _lib


def _ptr(a, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


def cell_index(gen_pat, pattern):
    """Mixed-radix cell index, position 0 least significant."""
    idx, w = 0, 1
    for g, x in zip(gen_pat, pattern):
        idx += _PERM[g].index(x) * w
        w *= len(_PERM[g])
    return idx


def cell_pattern(gen_pat, num):
    out = []
    for g in gen_pat:
        num, d = divmod(int(num), len(_PERM[g]))
        out.append(_PERM[g][d])
    return "".join(out)


def npat(gen_pat):
    return int(lib().kpo_npat(gen_pat.encode()))


def _scatter(gen_pat, contexts, rows, nf):
    arr = np.zeros((npat(gen_pat), nf), dtype=np.uint64)
    idx = np.array([cell_index(gen_pat, c) for c in contexts], dtype=np.int64)
    arr[idx] = np.asarray(rows, dtype=np.uint64).reshape(len(contexts), nf)
    return arr


def cv_pass(gen_pat, contexts, Mf, Uf, alpha, betas, penalty, itype_bits=32, threads=1):
    """One CV pass for a single (alpha, penalty) over all folds (CV module :143-163).
    ``threads`` > 1 splits every level over OpenMP threads (same values).

    ``contexts`` are k-mers and ``Mf``/``Uf`` their ``[n_kmers, nf]`` fold counts.
    Returns a dict with the full ``score``/``test``/``M``/``U`` arrays and the root rows.
    """
    Mf = np.asarray(Mf)
    nf = Mf.shape[1]
    M = _scatter(gen_pat, contexts, Mf, nf)
    U = _scatter(gen_pat, contexts, Uf, nf)
    n = M.shape[0]
    score = np.empty((n, nf), dtype=np.float32)
    test = np.empty((n, nf), dtype=np.float32)
    b = np.ascontiguousarray(betas, dtype=np.float64)
    rc = lib().kpo_cv(gen_pat.encode(), nf, _ptr(M, ctypes.c_uint64), _ptr(U, ctypes.c_uint64),
                      int(itype_bits), float(alpha), _ptr(b, ctypes.c_double), float(penalty),
                      _ptr(score, ctypes.c_float), _ptr(test, ctypes.c_float), int(threads))
    if rc:
        raise RuntimeError(f"kpo_cv failed ({rc})")
    root = cell_index(gen_pat, gen_pat)
    return {"score": score, "test": test, "M": M, "U": U,
            "root_train": score[root].copy(), "root_test": test[root].copy()}


def cv_lane(gen_pat, kcell, m, u, alpha, beta, penalty, itype_bits=32, threads=1, out=None):
    """Train scores (float32 ``[npat]``, reference cell order) of ONE CV lane over the whole
    lattice of ``gen_pat`` (kpo_cv_lane: the kpo_cv recurrence for one fold, train counts
    only, 12 B/cell).  ``kcell`` = cell index of each k-mer, ``m``/``u`` = its train counts
    (all data - the lane's fold).  ``out`` may be a preallocated float32 array."""
    kcell = np.ascontiguousarray(kcell, dtype=np.uint64)
    m = np.ascontiguousarray(m, dtype=np.uint64)
    u = np.ascontiguousarray(u, dtype=np.uint64)
    n = npat(gen_pat)
    score = np.empty(n, np.float32) if out is None else out
    assert score.dtype == np.float32 and score.size == n and score.flags.c_contiguous
    rc = lib().kpo_cv_lane(gen_pat.encode(), kcell.size, _ptr(kcell, ctypes.c_uint64), _ptr(m, ctypes.c_uint64),
                           _ptr(u, ctypes.c_uint64), int(itype_bits), float(alpha), float(beta), float(penalty),
                           _ptr(score, ctypes.c_float), int(threads))
    if rc:
        raise RuntimeError(f"kpo_cv_lane failed ({rc})")
    return score


def libm(x, fn="log"):
    """The host C library's ``log`` / ``log1p`` over a float64 array."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    lib().kpo_libm_array(_ptr(x, ctypes.c_double), _ptr(y, ctypes.c_double), x.size, 1 if fn == "log1p" else 0)
    return y


def _right(super_pat, left):
    """get_right (Fit :8-15): the other half of the split at the position that differs."""
    out = []
    for s, x in zip(super_pat, left):
        if s == x:
            out.append(s)
        else:
            for pair in _SPLIT[s].split():
                if x in pair:
                    out.append(pair[1] if pair[0] == x else pair[0])
                    break
    return "".join(out)


def names_from_backtrack(gen_pat, bt):
    """backtrack (Fit :17-24), iteratively: left subtree first, then right."""
    out = []
    stack = [gen_pat]
    while stack:
        pat = stack.pop()
        num = cell_index(gen_pat, pat)
        left = int(bt[num])
        if left == num:
            out.append(pat)
            continue
        lp = cell_pattern(gen_pat, left)
        stack.append(_right(pat, lp))
        stack.append(lp)
    return out


def fit(gen_pat, contexts, M0, U0, alpha, beta, penalty, itype_bits=32, threads=1):
    """Fit DP + backtrack (Fit :67-124).  Returns (score_f32, M_root, U_root, names, arrays)."""
    M = _scatter(gen_pat, contexts, np.asarray(M0).reshape(-1, 1), 1).reshape(-1)
    U = _scatter(gen_pat, contexts, np.asarray(U0).reshape(-1, 1), 1).reshape(-1)
    n = M.shape[0]
    score = np.empty(n, dtype=np.float32)
    bt = np.empty(n, dtype=np.uint64)
    rc = lib().kpo_fit(gen_pat.encode(), _ptr(M, ctypes.c_uint64), _ptr(U, ctypes.c_uint64),
                       int(itype_bits), float(alpha), float(beta), float(penalty),
                       _ptr(score, ctypes.c_float), _ptr(bt, ctypes.c_uint64), int(threads))
    if rc:
        raise RuntimeError(f"kpo_fit failed ({rc})")
    root = cell_index(gen_pat, gen_pat)
    names = names_from_backtrack(gen_pat, bt)
    return score[root], int(M[root]), int(U[root]), names, {"score": score, "backtrack": bt, "M": M, "U": U}

"""ctypes front-end of the test-only emulator (see kp_emu.hip).  TEST INFRASTRUCTURE."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_PATH = os.path.join(HERE, "libkp_emu.so")
_lib = None

GROUP_DT = np.dtype([("fold", "<i4"), ("lane0", "<i4"), ("nl", "<i4"), ("nl2", "<i4"),
                     ("alpha", "<f8"), ("beta", "<f8"), ("pen", "<f8", (8,)), ("alpha2", "<f8"), ("beta2", "<f8")])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_PATH):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        _lib = ctypes.CDLL(_PATH)
        _lib.emu_last_error.restype = ctypes.c_char_p
    return _lib


def run(gen_pat, M, U, groups, max_block=4096, dump=False):
    """groups: list of (fold, alpha, beta, [penalties]).  M, U: [n_kmers, nf] k-mer order."""
    M = np.ascontiguousarray(M)
    U = np.ascontiguousarray(U, dtype=M.dtype)
    nf = M.shape[1]
    recs = np.zeros(len(groups), dtype=GROUP_DT)
    lane = 0
    for i, (fold, a, b, pens) in enumerate(groups):
        recs[i]["fold"] = fold
        recs[i]["lane0"] = lane
        recs[i]["nl"] = len(pens)
        recs[i]["alpha"] = a
        recs[i]["beta"] = b
        recs[i]["pen"][:len(pens)] = pens
        lane += len(pens)
    L = lane
    rt = np.zeros(L, np.float32)
    re = np.zeros(L, np.float32)
    nlv = np.zeros(L, np.uint64)
    npat = 1
    from kmerpapa_amd.pattern_utils import pattern_max, generality
    npat = pattern_max(gen_pat)
    nk = generality(gen_pat)
    ds = np.zeros(L * npat, np.float32) if dump else None
    dc = np.zeros(L * npat, np.uint8) if dump else None
    leaves = np.zeros(L * nk, np.uint64)
    P = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)
    rc = lib().emu_run(gen_pat.encode(), ctypes.c_uint32(max_block), P(M), P(U), nf, M.dtype.itemsize,
                       P(recs), len(groups), P(rt), P(re), P(nlv), P(ds), P(dc), P(leaves))
    if rc:
        raise RuntimeError(lib().emu_last_error().decode())
    out = {"root_train": rt, "root_test": re, "n_leaves": nlv,
           "leaves": [leaves[i * nk:i * nk + int(nlv[i])] for i in range(L)]}
    if dump:
        out["score"] = ds.reshape(L, npat)
        out["code"] = dc.reshape(L, npat)
    return out


def run_groups(gen_pat, M, U, groups, devices=None, max_block=0):
    """Drop-in for kmerpapa_amd.engine.run_groups backed by the emulator (CPU tests only);
    takes a FoldFeed for M like the engine (waits for every fold)."""
    from kmerpapa_amd.engine import materialize
    M, U, groups = materialize(M, U, groups)
    out = run(gen_pat, M, U, groups, max_block=max_block or 4096)
    return out["root_train"], out["root_test"], out["n_leaves"]


run_groups.fold_feed = True

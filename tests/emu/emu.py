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


class EmuPlan:
    """Stand-in for ``engine.Plan`` backed by the emulator (CPU tests only): the same
    count-upload interface (set_counts, or counts_begin + counts_fold one fold at a time,
    as kp_counts_begin / kp_counts_fold) and ``run(groups)`` returning per-lane roots, so
    engine.run_groups' real plan / fold-feed / pass-packing code runs unchanged.  Like the
    device's slot-major count tables (slot 0 = all data, slot 1 + f = fold f), a group of
    fold f sees train = all data - fold f and test = fold f."""

    def __init__(self, gen_pat, max_block=0, width=5, fit=7):
        from kmerpapa_amd.pattern_utils import generality, pattern_max
        self.gen_pat = gen_pat
        self.max_block = max_block or 4096
        self.info = {"lanes_per_workgroup": width, "npat": pattern_max(gen_pat), "n_kmers": generality(gen_pat)}
        self.fit = fit
        self.all = None
        self.folds = {}
        self.reserved = 0
        self.passes = []

    def set_counts(self, M, U):
        M = np.asarray(M)
        U = np.asarray(U, dtype=M.dtype)
        if M.ndim == 1:
            M, U = M.reshape(-1, 1), U.reshape(-1, 1)
        self.all = (M.sum(axis=1, dtype=M.dtype), U.sum(axis=1, dtype=M.dtype))
        self.folds = {f: (M[:, f].copy(), U[:, f].copy()) for f in range(M.shape[1])}

    def counts_begin(self, M_all, U_all, nf):
        self.all = (np.asarray(M_all).copy(), np.asarray(U_all, dtype=np.asarray(M_all).dtype).copy())
        self.folds = {}

    def counts_fold(self, fold, M_fold, U_fold):
        dt = self.all[0].dtype
        self.folds[fold] = (np.asarray(M_fold, dt).copy(), np.asarray(U_fold, dt).copy())

    def lanes_that_fit(self):
        return self.fit

    def require_lanes(self, n=1):
        return self.lanes_that_fit()

    def reserve(self, lanes):
        self.reserved = max(self.reserved, int(lanes))

    def run(self, groups):
        rt, re, nl = [], [], []
        lanes = 0
        for f, a, b, pens in groups:
            if f not in self.folds:
                raise RuntimeError(f"fold {f} has not been uploaded")  # kp_pass: KP_E_STATE
            b = float(b() if callable(b) else b)
            mf, uf = self.folds[f]
            M2 = np.stack([mf, self.all[0] - mf], axis=1)
            U2 = np.stack([uf, self.all[1] - uf], axis=1)
            out = run(self.gen_pat, M2, U2, [(0, a, b, list(pens))], max_block=self.max_block)
            rt.append(out["root_train"])
            re.append(out["root_test"])
            nl.append(out["n_leaves"])
            lanes += len(pens)
        if lanes > max(self.reserved, self.fit):
            raise RuntimeError("pass wider than the reserved lane buffers")
        self.passes.append([(g[0], g[1], len(g[3])) for g in groups])
        return np.concatenate(rt), np.concatenate(re), np.concatenate(nl)

#!/usr/bin/env python3
"""Golden-vector generator (test infrastructure, run ONLY in the build container).

Runs the upstream reference (kmerPaPa v0.2.4, read-only at /root/reference) under a
tiny stand-in for ``numba.njit`` (identity decorator) and ``skopt`` (stubs), and
records inputs and outputs of the penalized-likelihood lattice DP as small data
fixtures under ``tests/golden/``.  The stand-in lives in a temporary directory
created by this script; nothing of the reference is copied into the repository,
only numbers it produced.

Canonical interpreter: /opt/conda/bin/python3.9 (numpy 1.26, scipy 1.7) which follows
the numpy<2 promotion rules of the reference's pinned numpy 1.23.3.

Usage:  python3 tests/golden/make_golden.py [--jobs small,grid5,fit5,cli5,cli5b,fit7,cv7,allk5]
        (config 3 grid: one process per point, --jobs cv7p_<alpha>_<c>, then --jobs cv7merge)
The GPU box never runs this file (no /root/reference there).
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import textwrap

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"
REF_DATA = "/root/reference/test_data"
CANON_PY = "/opt/conda/bin/python3.9"

SHIM = {
    "numba/__init__.py": textwrap.dedent("""
        def njit(*a, **k):
            if len(a) == 1 and callable(a[0]) and not k:
                return a[0]
            return lambda f: f
        jit = njit
    """),
    "skopt/__init__.py": "def gp_minimize(*a, **k):\n    raise RuntimeError('skopt stub')\n",
    "skopt/space.py": "class Real:\n    def __init__(self,*a,**k): pass\nclass Integer(Real): pass\n",
    "skopt/utils.py": "def use_named_args(space):\n    return lambda f: f\n",
}


def make_shim(tmp):
    for rel, txt in SHIM.items():
        p = os.path.join(tmp, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as fh:
            fh.write(txt)


# ----------------------------------------------------------------------------
# helpers executed inside the child interpreter (reference importable there)
# ----------------------------------------------------------------------------

def _read_counts(name):
    d = {}
    with open(os.path.join(REF_DATA, name)) as fh:
        for line in fh:
            a, b = line.split()
            d[a] = int(b)
    return d


def _context(k):
    """contextD exactly as cli.main builds it (read_input + zero fill)."""
    import kmerpapa.io_utils as io
    from kmerpapa.pattern_utils import LCA_pattern_of_kmers, matches

    class A:  # argparse stand-in
        positive = open(os.path.join(REF_DATA, f"mutated_{k}mers.txt"))
        background = open(os.path.join(REF_DATA, f"background_{k}mers.txt"))
        negative = None
        joint_context_counts = None
    ctx, nu, nm = io.read_input(A, None)
    gp = LCA_pattern_of_kmers(list(ctx.keys()))
    for c in matches(gp):
        if c not in ctx:
            ctx[c] = (0, 0)
    return ctx, gp, nu, nm


class _Args:
    def __init__(self, nfolds, seed, iterations=1, verbosity=0, CVfile=None):
        self.nfolds = nfolds
        self.seed = seed
        self.iterations = iterations
        self.verbosity = verbosity
        self.CVfile = CVfile


def _hook_cv(record_full):
    """Wrap the CV kernel so the root call snapshots the DP arrays of each (a, c)."""
    import kmerpapa.algorithms.bottum_up_array_penalty_plus_pseudo_CV as cvm
    orig = cvm.handle_pattern
    log = []

    def wrapped(score_mem, test_score_mem, pattern, M_mem, U_mem, alpha, betas, penalty):
        orig(score_mem, test_score_mem, pattern, M_mem, U_mem, alpha, betas, penalty)
        root = tuple(ord(x) for x in cvm.__dict__["_golden_root"])
        if tuple(int(v) for v in pattern) == root:
            rec = {"alpha": float(alpha), "penalty": float(penalty),
                   "betas": [float(b) for b in betas]}
            pn = cvm.gen_pat_num
            rec["root_train"] = score_mem[pn].copy()
            rec["root_test"] = test_score_mem[pn].copy()
            if record_full:
                rec["score"] = score_mem.copy()
                rec["test"] = test_score_mem.copy()
                rec["M"] = M_mem.copy()
                rec["U"] = U_mem.copy()
            log.append(rec)
    cvm.handle_pattern = wrapped
    return cvm, log


def _run_cv(ctx, gp, alphas, penalties, nf, seed, nm, nu, record_full, iterations=1):
    import io as _io
    cvm, log = _hook_cv(record_full)
    cvm._golden_root = gp
    buf = _io.StringIO()
    args = _Args(nf, seed, iterations=iterations, CVfile=buf)
    res = cvm.pattern_partition_bottom_up(gp, ctx, alphas, args, nm, nu, penalties)
    return res, log, buf.getvalue()


def _fold_tables(ctx, gp, nf, seed, itype):
    import numpy as np
    import kmerpapa.CV_tools as cvt
    from kmerpapa.pattern_utils import pattern_max, PatternEnumeration
    npat = pattern_max(gp)
    U = np.zeros((npat, nf), dtype=itype)
    M = np.zeros((npat, nf), dtype=itype)
    prng = np.random.RandomState(seed)
    cvt.make_all_folds_contextD_patterns(ctx, U, M, gp, prng, itype)
    PE = PatternEnumeration(gp)
    kmers = sorted(ctx)
    idx = [PE.pattern2num(x) for x in kmers]
    return kmers, M[idx].copy(), U[idx].copy()


def _hook_fit(record_full):
    import kmerpapa.algorithms.bottum_up_array_w_numba as fm
    orig = fm.handle_pattern
    box = {}

    def wrapped(pattern, score_mem, backtrack_mem, M_mem, U_mem):
        orig(pattern, score_mem, backtrack_mem, M_mem, U_mem)
        box["arrs"] = (score_mem, backtrack_mem, M_mem, U_mem)
    fm.handle_pattern = wrapped
    return fm, box


def _run_fit(ctx, gp, alpha, penalty, nm, nu, record_full=False):
    fm, box = _hook_fit(record_full)
    my = nm / (nm + nu)
    beta = (alpha * (1.0 - my)) / my
    try:
        sc, M, U, names = fm.pattern_partition_bottom_up(gp, ctx, alpha, beta, penalty, _Args(None, None), nm, nu)
    except Exception as e:  # the reference's own failure mode is part of its behaviour
        return {"alpha": alpha, "beta": beta, "penalty": penalty, "error": type(e).__name__}, None
    out = {"alpha": alpha, "beta": beta, "penalty": penalty, "score": float(sc),
           "score_f32_hex": float(sc).hex(), "M": int(M), "U": int(U), "names": list(names)}
    arrs = None
    if record_full and "arrs" in box:
        s, b, Mm, Um = box["arrs"]
        arrs = {"score": s.copy(), "backtrack": b.copy(), "M": Mm.copy(), "U": Um.copy()}
    return out, arrs


def _ctx_from(ctx):
    return {k: tuple(int(x) for x in v) for k, v in ctx.items()}


def job_small(out):
    """Enumeration tables, fold splits, full DP arrays on 3/4-mer lattices, edge cases."""
    import numpy as np
    import kmerpapa.pattern_utils as pu
    import kmerpapa.CV_tools as cvt
    from kmerpapa.io_utils import downsize_contextD

    # --- enumeration order / indices ---
    enum = {}
    for gp in ["NNMNN", "SWSW", "NMN", "RYK", "BDHV", "ANT", "NNNN"]:
        lv = pu.pattern_level(gp)
        per = [list(pu.subpatterns_level(gp, L)) for L in range(lv + 1)]
        gpo = tuple(ord(x) for x in gp)
        per_ord = [["".join(chr(c) for c in t) for t in pu.subpatterns_level_ord_np(gpo, lv, L)]
                   for L in range(lv + 1)]
        PE = pu.PatternEnumeration(gp)
        rec = {"pattern_max": pu.pattern_max(gp), "level": lv,
               "level_sizes": [len(x) for x in per],
               "sha_levels": hashlib.sha256("|".join(",".join(x) for x in per).encode()).hexdigest(),
               "sha_levels_ord": hashlib.sha256("|".join(",".join(x) for x in per_ord).encode()).hexdigest(),
               "sha_nums": hashlib.sha256(",".join(str(PE.pattern2num(p)) for x in per for p in x).encode()).hexdigest(),
               "matches": list(pu.matches(gp)) if pu.generality(gp) <= 64 else None}
        if pu.pattern_max(gp) <= 3000:
            rec["levels"] = per
            rec["levels_ord"] = per_ord
            rec["nums"] = [[PE.pattern2num(p) for p in lvl] for lvl in per]
        enum[gp] = rec
    lca = {}
    for group in [["AAT", "CAT", "GAT"], ["ACGT", "TCGA"], ["AAAAA"], ["GCA", "GCC", "GCT", "GCG"]]:
        lca["|".join(group)] = pu.LCA_pattern_of_kmers(group)
    with open(os.path.join(out, "enum.json"), "w") as fh:
        json.dump({"enum": enum, "lca": lca}, fh)

    # --- CV_tools on fixed inputs (RNG stream parity) ---
    kt = np.array([[1, 100, 200], [10, 1000, 2000]])
    f1 = cvt.make_all_folds(kt, 10, 2, np.random.RandomState(0))
    ctxA = {"AAA": (10, 100), "CAA": (200, 1000), "GAA": (500, 2000), "TAA": (300, 1000)}
    Ua = np.zeros((pu.pattern_max("NAA"), 10), dtype=np.uint64)
    Ma = np.zeros_like(Ua)
    cvt.make_all_folds_contextD_patterns(ctxA, Ua, Ma, "NAA", np.random.RandomState(0))
    Uk = np.zeros((4, 3), dtype=np.uint64)
    Mk = np.zeros_like(Uk)
    cvt.make_all_folds_contextD_kmers(ctxA, Uk, Mk, "NAA", np.random.RandomState(3))
    ctx5, gp5, nu5, nm5 = _context(5)
    kmers5, Mf5, Uf5 = _fold_tables(ctx5, gp5, 5, 1, np.uint32)
    ctx7, gp7, nu7, nm7 = _context(7)
    kmers7, Mf7, Uf7 = _fold_tables(ctx7, gp7, 5, 1, np.uint32)
    np.savez_compressed(os.path.join(out, "folds.npz"),
                        make_all_folds=f1, ctxA_U=Ua, ctxA_M=Ma, kmersA_U=Uk, kmersA_M=Mk,
                        kmers5=np.array(kmers5), M5=Mf5, U5=Uf5,
                        kmers7=np.array(kmers7), M7=Mf7, U7=Uf7)
    meta = {"gp5": gp5, "nu5": nu5, "nm5": nm5, "gp7": gp7, "nu7": nu7, "nm7": nm7}

    # --- full DP arrays on small lattices ---
    full = {}
    cases = []
    c3, g3 = downsize_contextD(ctx5, gp5, 3)
    c4, g4 = downsize_contextD(ctx5, gp5, 4)
    c3 = _ctx_from(c3)
    c4 = _ctx_from(c4)
    cases.append(("k3", c3, g3, [0.5, 1.0], [3.0, 0.0], 5, 1, np.uint32))
    cases.append(("k4", c4, g4, [0.8], [2.0, 6.0], 5, 7, np.uint32))
    # alpha = 0 edge case and zero-count k-mers (drop some k-mers -> zero filled)
    c3z = dict(c3)
    for i, key in enumerate(sorted(c3z)):
        if i % 7 == 0:
            c3z[key] = (0, 0)
        elif i % 11 == 0:
            c3z[key] = (0, c3z[key][1])
    cases.append(("k3zero", c3z, g3, [0.0, 2.0], [3.0], 3, 5, np.uint32))
    # uint64 itype: totals above 2**32-1
    c3big = {k: (v[0] * 40, v[1] * 40) for k, v in c3.items()}
    cases.append(("k3big", c3big, g3, [1.0], [4.0], 4, 2, np.uint64))
    arrays = {}
    for name, ctx, gp, alphas, pens, nf, seed, itype in cases:
        nm = sum(v[0] for v in ctx.values())
        nu = sum(v[1] for v in ctx.values())
        res, log, cvtext = _run_cv(ctx, gp, alphas, pens, nf, seed, nm, nu, True)
        kmers, Mf, Uf = _fold_tables(ctx, gp, nf, seed, itype)
        arrays[f"{name}_Mf"] = Mf
        arrays[f"{name}_Uf"] = Uf
        arrays[f"{name}_kmers"] = np.array(kmers)
        recs = []
        for j, r in enumerate(log):
            for key in ("score", "test", "M", "U"):
                arrays[f"{name}_{j}_{key}"] = r[key]
            recs.append({"alpha": r["alpha"], "penalty": r["penalty"], "betas": r["betas"],
                         "root_train": [float(x) for x in r["root_train"]],
                         "root_test": [float(x) for x in r["root_test"]]})
        fits = []
        for a in alphas:
            for c in pens:
                fo, fa = _run_fit(ctx, gp, a, c, nm, nu, record_full=True)
                if fa is not None:
                    arrays[f"{name}_fit_{len(fits)}_score"] = fa["score"]
                    arrays[f"{name}_fit_{len(fits)}_backtrack"] = fa["backtrack"]
                fits.append(fo)
        full[name] = {"gen_pat": gp, "alphas": alphas, "penalties": pens, "nfolds": nf, "seed": seed,
                      "itype": np.dtype(itype).name, "nmut": nm, "nunmut": nu,
                      "best": [res[0], res[1], float(res[2])], "cvfile": cvtext,
                      "passes": recs, "fits": fits, "contextD": {k: list(v) for k, v in ctx.items()}}
    # repeated CV (iterations=2) exercises the reference's M_sum carry-over
    nm = sum(v[0] for v in c3.values())
    nu = sum(v[1] for v in c3.values())
    res, log, cvtext = _run_cv(c3, g3, [0.5, 1.0], [3.0], 3, 11, nm, nu, False, iterations=2)
    full["k3iter2"] = {"gen_pat": g3, "alphas": [0.5, 1.0], "penalties": [3.0], "nfolds": 3, "seed": 11,
                       "iterations": 2, "itype": "uint32", "nmut": nm, "nunmut": nu,
                       "best": [res[0], res[1], float(res[2])], "cvfile": cvtext,
                       "passes": [{"alpha": r["alpha"], "penalty": r["penalty"], "betas": r["betas"],
                                   "root_train": [float(x) for x in r["root_train"]],
                                   "root_test": [float(x) for x in r["root_test"]]} for r in log]}
    np.savez_compressed(os.path.join(out, "small_dp.npz"), **arrays)
    with open(os.path.join(out, "small_dp.json"), "w") as fh:
        json.dump({"meta": meta, "cases": full}, fh)


def job_grid5(out):
    """5-mer 3x3 grid, 5 folds, seed 1: per-(a,c) roots and CVfile text."""
    ctx, gp, nu, nm = _context(5)
    alphas = [0.5, 1.0, 10.0]
    pens = [3.0, 5.0, 7.0]
    res, log, cvtext = _run_cv(ctx, gp, alphas, pens, 5, 1, nm, nu, False)
    recs = [{"alpha": r["alpha"], "penalty": r["penalty"], "betas": r["betas"],
             "root_train": [float(x) for x in r["root_train"]],
             "root_test": [float(x) for x in r["root_test"]]} for r in log]
    with open(os.path.join(out, "grid5.json"), "w") as fh:
        json.dump({"gen_pat": gp, "alphas": alphas, "penalties": pens, "nfolds": 5, "seed": 1,
                   "best": [res[0], res[1], float(res[2])], "cvfile": cvtext, "passes": recs}, fh)


def job_fit5(out):
    ctx, gp, nu, nm = _context(5)
    fits = [_run_fit(ctx, gp, 0.5, 3.0, nm, nu)[0], _run_fit(ctx, gp, 1.0, 5.0, nm, nu)[0],
            _run_fit(ctx, gp, 0.8, 0.0, nm, nu)[0]]
    with open(os.path.join(out, "fit5.json"), "w") as fh:
        json.dump({"gen_pat": gp, "nmut": nm, "nunmut": nu, "fits": fits}, fh)


def job_cli5(out):
    """Whole-CLI text outputs (output table + CVfile) for configs 1 and 2."""
    import io as _io
    import contextlib
    from kmerpapa import cli
    pos = os.path.join(REF_DATA, "mutated_5mers.txt")
    bg = os.path.join(REF_DATA, "background_5mers.txt")
    res = {}
    with tempfile.TemporaryDirectory() as td:
        runs = {
            "fit": ["-p", pos, "-b", bg, "-c", "3", "-a", "0.5"],
            "fit_long": ["-p", pos, "-b", bg, "-c", "5", "-a", "1", "-l"],
            "grid": ["-p", pos, "-b", bg, "-c", "3", "5", "7", "-a", "0.5", "1", "10",
                     "--nfolds", "5", "--seed", "1"],
            "super": ["-p", pos, "-b", bg, "-c", "4", "-a", "0.5", "-s", "NNCNN"],
            "default_pen": ["-p", pos, "-b", bg, "-a", "2"],
        }
        for name, argv in runs.items():
            o = os.path.join(td, name + ".out")
            f = os.path.join(td, name + ".cv")
            err = _io.StringIO()
            with contextlib.redirect_stderr(err):
                rc = cli.main(argv + ["-o", o, "-f", f])
            res[name] = {"argv": argv, "rc": rc, "output": open(o).read(),
                         "cvfile": open(f).read(), "stderr": err.getvalue()}
    with open(os.path.join(out, "cli5.json"), "w") as fh:
        json.dump(res, fh)


def _joint_lines(pos_counts, bg_counts):
    """"kmer positive background" lines (read_joint_kmer_counts format) in background order."""
    return "".join(f"{x} {pos_counts.get(x, 0)} {c}\n" for x, c in bg_counts.items())


def job_cli5b(out):
    """CLI input variants and --test_smaller_k on the 5-mer data (ref cli.py:118-318,
    io_utils.py:3-217): joint count file, --negative file, CV over k = 5 and 3.

    The k = 3 lattice (675 cells) is small enough that the CV module's np.empty arrays
    (CV :93-102) come from recycled heap memory, and its fold totals sum those rows
    (CV :134-137): the reference's own k = 3 numbers then depend on the heap (a fresh
    process gives 1328534.5, after the k = 5 pass 1328536.125).  The vectors pin the
    zero-initialised arrays the reference gets for every large lattice (SURVEY.md 8(a)
    a3 quirk iii): np.empty is zeros in the CV module for this job."""
    import io as _io
    import contextlib
    import types
    import numpy as np
    import kmerpapa.algorithms.bottum_up_array_penalty_plus_pseudo_CV as cvm
    np_zeroed = types.ModuleType("numpy_zeroed_empty")
    np_zeroed.__dict__.update(np.__dict__)
    np_zeroed.empty = np.zeros
    cvm.np = np_zeroed
    from kmerpapa import cli
    pos = os.path.join(REF_DATA, "mutated_5mers.txt")
    bg = os.path.join(REF_DATA, "background_5mers.txt")
    res = {}
    with tempfile.TemporaryDirectory() as td:
        joint = os.path.join(td, "joint_5mers.txt")
        with open(joint, "w") as fh:
            fh.write(_joint_lines(_read_counts("mutated_5mers.txt"), _read_counts("background_5mers.txt")))
        runs = {
            "smaller_k": ["-p", pos, "-b", bg, "-c", "3", "5", "-a", "1", "--nfolds", "2", "--seed", "3",
                          "--test_smaller_k"],
            "joint": ["-j", joint, "-c", "3", "-a", "0.5"],
            "negative": ["-p", pos, "-n", bg, "-c", "4", "-a", "1"],
        }
        for name, argv in runs.items():
            o = os.path.join(td, name + ".out")
            f = os.path.join(td, name + ".cv")
            err = _io.StringIO()
            with contextlib.redirect_stderr(err):
                rc = cli.main(argv + ["-o", o, "-f", f])
            res[name] = {"argv": argv, "rc": rc, "output": open(o).read(),
                         "cvfile": open(f).read(), "stderr": err.getvalue()}
    with open(os.path.join(out, "cli5b.json"), "w") as fh:
        json.dump(res, fh)


def job_allk5(out):
    """--score all_kmers CLI runs on the 5-mer data (ref all_kmers_CV.py, cli.py:226-271)."""
    import io as _io
    import contextlib
    from kmerpapa import cli
    pos = os.path.join(REF_DATA, "mutated_5mers.txt")
    bg = os.path.join(REF_DATA, "background_5mers.txt")
    res = {}
    with tempfile.TemporaryDirectory() as td:
        runs = {
            "grid": ["-p", pos, "-b", bg, "--score", "all_kmers", "-a", "0.5", "1", "10", "--nfolds", "5",
                     "--seed", "1"],
            "iter": ["-p", pos, "-b", bg, "--score", "all_kmers", "-a", "0.2", "3", "--nfolds", "3", "--seed", "7",
                     "-i", "2", "-l"],
        }
        for name, argv in runs.items():
            o = os.path.join(td, name + ".out")
            err = _io.StringIO()
            with contextlib.redirect_stderr(err):
                rc = cli.main(argv + ["-o", o])
            res[name] = {"argv": argv, "rc": rc, "output": open(o).read(), "stderr": err.getvalue()}
    with open(os.path.join(out, "allk5.json"), "w") as fh:
        json.dump(res, fh)


def job_iter5(out):
    """--iterations 2 on the 5-mer lattice.  The reference sums M_mem over ALL rows for
    the fold totals (CV :134-137); in iteration 0 the aggregated rows come from np.empty,
    which is zero only for allocations large enough to get fresh pages (a 3-mer lattice
    gets recycled heap memory = undefined values), so the carry-over is pinned here."""
    ctx, gp, nu, nm = _context(5)
    res, log, cvtext = _run_cv(ctx, gp, [0.5, 2.0], [4.0], 3, 11, nm, nu, False, iterations=2)
    recs = [{"alpha": r["alpha"], "penalty": r["penalty"], "betas": r["betas"],
             "root_train": [float(x) for x in r["root_train"]],
             "root_test": [float(x) for x in r["root_test"]]} for r in log]
    with open(os.path.join(out, "iter5.json"), "w") as fh:
        json.dump({"gen_pat": gp, "alphas": [0.5, 2.0], "penalties": [4.0], "nfolds": 3, "seed": 11,
                   "iterations": 2, "nmut": nm, "nunmut": nu, "best": [res[0], res[1], float(res[2])],
                   "cvfile": cvtext, "passes": recs}, fh)


def job_fit7(out):
    ctx, gp, nu, nm = _context(7)
    fo, _ = _run_fit(ctx, gp, 0.5, 3.0, nm, nu)
    with open(os.path.join(out, "fit7.json"), "w") as fh:
        json.dump({"gen_pat": gp, "nmut": nm, "nunmut": nu, "fits": [fo]}, fh)


def job_cv7(out):
    ctx, gp, nu, nm = _context(7)
    res, log, cvtext = _run_cv(ctx, gp, [0.5], [3.0], 5, 1, nm, nu, False)
    recs = [{"alpha": r["alpha"], "penalty": r["penalty"], "betas": r["betas"],
             "root_train": [float(x) for x in r["root_train"]],
             "root_test": [float(x) for x in r["root_test"]]} for r in log]
    with open(os.path.join(out, "cv7.json"), "w") as fh:
        json.dump({"gen_pat": gp, "alphas": [0.5], "penalties": [3.0], "nfolds": 5, "seed": 1,
                   "best": [res[0], res[1], float(res[2])], "cvfile": cvtext, "passes": recs}, fh)


CV7_ALPHAS = [0.5, 1.0, 10.0]
CV7_PENALTIES = [3.0, 5.0, 7.0]


def job_cv7p(out, alpha, penalty):
    """One grid point of the 7-mer 3x3 grid (config 3), run the way the reference's README
    fans a grid out (README.md:39-51: one --CV_only process per (c, a), same seed, so the
    same fold split): roots of every fold and the CVfile row of that point."""
    ctx, gp, nu, nm = _context(7)
    res, log, cvtext = _run_cv(ctx, gp, [alpha], [penalty], 5, 1, nm, nu, False)
    recs = [{"alpha": r["alpha"], "penalty": r["penalty"], "betas": r["betas"],
             "root_train": [float(x) for x in r["root_train"]],
             "root_test": [float(x) for x in r["root_test"]]} for r in log]
    os.makedirs(os.path.join(out, "cv7_points"), exist_ok=True)
    with open(os.path.join(out, "cv7_points", f"a{alpha}_c{penalty}.json"), "w") as fh:
        json.dump({"gen_pat": gp, "alpha": alpha, "penalty": penalty, "nfolds": 5, "seed": 1,
                   "best": [res[0], res[1], float(res[2])], "cvfile": cvtext, "passes": recs}, fh)


def job_cv7merge(out):
    """Merge the nine cv7 points into cv7.json: CVfile rows in the reference's alpha-major,
    c-minor order (CV :165-177) and the grid's best point (strict "<" in that order)."""
    pts = []
    for a in CV7_ALPHAS:
        for c in CV7_PENALTIES:
            with open(os.path.join(out, "cv7_points", f"a{a}_c{c}.json")) as fh:
                pts.append(json.load(fh))
    best = None
    for p in pts:
        if best is None or p["best"][2] < best[2]:
            best = p["best"]
    with open(os.path.join(out, "cv7.json"), "w") as fh:
        json.dump({"gen_pat": pts[0]["gen_pat"], "alphas": CV7_ALPHAS, "penalties": CV7_PENALTIES,
                   "nfolds": 5, "seed": 1, "best": best, "cvfile": "".join(p["cvfile"] for p in pts),
                   "passes": [p["passes"][0] for p in pts]}, fh)


def job_data(out):
    """The reference's k-mer count files as one npz (inputs of configs 1-3)."""
    import numpy as np
    arrays = {}
    for k in (5, 7):
        for kind in ("mutated", "background"):
            d = _read_counts(f"{kind}_{k}mers.txt")
            keys = list(d)  # file order kept
            arrays[f"{kind}{k}_kmers"] = np.array(keys)
            arrays[f"{kind}{k}_counts"] = np.array([d[x] for x in keys], dtype=np.int64)
    np.savez_compressed(os.path.join(out, "test_data.npz"), **arrays)


def _child(job, out):
    if job.startswith("cv7p_"):  # cv7p_<alpha>_<penalty>
        _, a, c = job.split("_")
        job_cv7p(out, float(a), float(c))
        return
    globals()["job_" + job](out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", default="small,grid5,fit5,cli5")
    ap.add_argument("--python", default=CANON_PY)
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--child", default=None)
    a = ap.parse_args()
    if a.child:
        _child(a.child, a.out)
        return
    if a.jobs in ("data", "cv7merge"):
        globals()["job_" + a.jobs](a.out)
        return
    with tempfile.TemporaryDirectory() as tmp:
        make_shim(tmp)
        env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1",
                   PYTHONPATH=tmp + os.pathsep + REF_SRC, PYTHONWARNINGS="ignore")
        for job in a.jobs.split(","):
            print("golden job", job, flush=True)
            subprocess.run([a.python, os.path.abspath(__file__), "--child", job, "--out", a.out],
                           env=env, check=True, cwd=tmp)


if __name__ == "__main__":
    main()

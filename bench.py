#!/usr/bin/env python3
"""Benchmark of the MI355X lattice DP on BASELINE.json's headline workload.

Workload: synthetic 9-mer counts, general pattern NNNNMNNNN
(131,072 k-mers, 7,688,671,875 lattice cells), 5x5 (pseudo-count alpha x penalty c)
grid, 5-fold CV, fold split with seed 1 exactly as the reference does it.

A step = one pass of the hot path over one batch: one (alpha, fold) group with its 5
penalties as 5 lanes, i.e. the full DP over all 7.69e9 cells for 5 (cell, fold, alpha, c)
units each = 3.84e10 units.  The full 5x5x5 CV is 25 such steps.  With N ranks
(torch.distributed.run, one GPU per rank) every rank runs its own groups
(group = (step * N + rank) mod 25): per-GPU work is fixed, "scaling": "weak", and no
collective touches the data path; the barrier and the max-time
reduction use gloo on the host.

Timed region: K steps between two barriers; inputs (fold counts, per-block count tables)
are resident in HBM before it starts.  Units = cells x lanes, summed over ranks.
The roofline object prices the DP sweep kernel (kp_dp_kernel, all launches of one pass)
against HBM: ``achieved`` = the bytes the blocked sweep must move per pass -- every
high-position split pair reads two child-block rows (2 x 4 B per unit) and every cell is
written once (4 B): (8 P_high + 4) B per unit, P_high = split pairs per cell at high
positions -- over the HIP-event time of the pass's launches.  ``traffic`` is
the rocprofv3 PMC L2-to-fabric byte count of the same pass (FETCH_SIZE x2 + WRITE_SIZE;
it includes Infinity-Cache hits, so it is an upper bound on HBM bytes), taken from the
committed profile whose kernel tag matches this build and launch configuration.  The
floor (4 B read + 4 B written per unit, every row moved once) and the SURVEY.md 8(d)
naive per-cell figure (16 B per split pair, ...) are reported beside it.
The cpu_baseline leg times the CPU oracle (oracle/kp_oracle.c, a C restatement of the
reference's DP) on a bounded sample of the same counts: the reference's own fan-out
(README.md:39-51, one process per grid point) as one single-threaded oracle task per
(alpha, c) on every host core, and one task alone on one core.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from kmerpapa_amd import engine  # noqa: E402  (loads libamdhip64 before torch does)
from kmerpapa_amd.CV_tools import fold_tables  # noqa: E402
from kmerpapa_amd.pattern_utils import KmerEnumeration, generality  # noqa: E402

GEN_PAT = "NNNNMNNNN"
ALPHAS = [0.5, 1.0, 2.0, 5.0, 10.0]
PENALTIES = [3.0, 4.0, 5.0, 6.0, 7.0]
NFOLDS = 5
PEAK_HBM_GBS = 8000.0
# BASELINE.json configs[4]: synthetic 11-mers, 7x7 grid, 10-fold CV.  The all-N 11-mer
# lattice (1.7e12 cells) needs >= 41 TB per lane, so -- as SURVEY.md 8(d) prescribes -- the
# flanks are fixed by a super-pattern: ANNNNMNNNNA has the 9-mer's 7.69e9 cells.
CONFIGS = {
    "9mer": dict(gen_pat="NNNNMNNNN", alphas=ALPHAS, penalties=PENALTIES, nfolds=5),
    "11mer": dict(gen_pat="ANNNNMNNNNA", alphas=[0.5, 1.0, 2.0, 3.0, 5.0, 7.0, 10.0],
                  penalties=[2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 8.0], nfolds=10),
}


def synthetic_counts(gen_pat=GEN_PAT, seed=9):
    """Synthetic k-mer counts, k-mers in KmerEnumeration order.

    bg ~ Poisson(LogNormal(log 1.5e4, 0.8)); rate = 2.7e-5 * f[x3] * f[x5] * LogNormal(0, 0.3)
    with f = {A: .6, C: 1, G: 1.8, T: .8} on the two bases flanking the centre;
    positives ~ Binomial(bg, rate).  Returns (kmers, M, U).
    """
    rng = np.random.RandomState(seed)
    KE = KmerEnumeration(gen_pat)
    n = generality(gen_pat)
    kmers = [KE.num2kmer(i) for i in range(n)]
    bg = rng.poisson(rng.lognormal(math.log(1.5e4), 0.8, size=n))
    f = {"A": 0.6, "C": 1.0, "G": 1.8, "T": 0.8}
    mid = len(gen_pat) // 2
    fl = np.array([f[k[mid - 1]] * f[k[mid + 1]] for k in kmers])
    rate = 2.7e-5 * fl * rng.lognormal(0.0, 0.3, size=n)
    pos = rng.binomial(bg, np.minimum(rate, 1.0))
    return kmers, pos.astype(np.int64), (bg - pos).astype(np.int64)


def kmer_table(kmers, M, U):
    """The CLI's array-backed count table (io_utils.KmerCounts, sorted 2-bit codes) of a
    k-mer list: what the native reader hands the CV driver."""
    from kmerpapa_amd.io_utils import KmerCounts
    k = len(kmers[0])
    raw = np.frombuffer("".join(kmers).encode("ascii"), np.uint8).reshape(len(kmers), k)
    lut = np.zeros(256, np.uint64)
    for i, ch in enumerate("ACGT"):
        lut[ord(ch)] = i
    codes = np.zeros(len(kmers), np.uint64)
    for j in range(k):
        codes = codes * np.uint64(4) + lut[raw[:, j]]
    o = np.argsort(codes, kind="stable")
    return KmerCounts(k, codes[o], np.asarray(M, np.int64)[o], np.asarray(U, np.int64)[o])


def prepare(gen_pat, seed=1, alphas=ALPHAS, penalties=PENALTIES, nfolds=NFOLDS):
    """Fold split (reference RNG stream) and betas for every (alpha, fold)."""
    kmers, M, U = synthetic_counts(gen_pat)
    table = kmer_table(kmers, M, U)
    total = int(M.sum() + U.sum())
    itype = np.uint64 if total > np.iinfo(np.uint32).max else np.uint32
    t0 = time.time()
    contexts, Mf, Uf = fold_tables(table, nfolds, np.random.RandomState(seed), itype)
    t_fold = time.time() - t0
    Mk, Uk = engine.counts_in_kmer_order(gen_pat, contexts, Mf, Uf, generality(gen_pat), itype)
    msum = Mk.sum(axis=0, dtype=np.uint64)
    usum = Uk.sum(axis=0, dtype=np.uint64)
    mtr, utr = msum.sum() - msum, usum.sum() - usum
    from kmerpapa_amd.shard import fold_order
    groups = []
    for a in alphas:
        my = mtr / (mtr + utr)
        betas = (a * (1.0 - my)) / my
        for f in fold_order(nfolds):  # the CV driver's group order (fold 0 last)
            groups.append((f, a, float(betas[f]), list(penalties)))
    return {"Mk": Mk, "Uk": Uk, "groups": groups, "itype": itype, "t_fold_s": t_fold, "contexts": list(table),
            "ctx": table, "Mf": Mf, "Uf": Uf, "total": total, "gen_pat": gen_pat, "alphas": list(alphas),
            "penalties": list(penalties), "nfolds": nfolds}


def host_cores():
    """Host cores this job may use: $OMP_NUM_THREADS (the GPU box sets its per-GPU CPU
    share there), else the affinity mask."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n)


def pairs_per_cell(gen_pat):
    """Split pairs per lattice cell (7.0 / 10.3 / 13.7 at the 5- / 7- /
    9-mer): a CPU's cell rate falls with it, so every sample states its own."""
    info = engine.plan_info(gen_pat)
    return info["pairs_total"] / info["npat"]


def cpu_baseline(prep, cores=None):
    """Time the CPU oracle on a bounded sample of the same counts: the sub-lattice with the
    two outermost ambiguous positions fixed to 'A' (3.4e7 cells for the 9-mer), one (alpha, c)
    over all folds per task.  Tasks run as the reference's README fans a grid out (one
    independent single-threaded job per (alpha, c)), one per host core of this job's CPU
    share, concurrently; one task alone on one core, and one task with its levels split
    over every core by OpenMP (kpo_cv's threads), are reported beside it.  Every sample
    states its split pairs per cell beside the workload's: the samples are smaller
    lattices with fewer pairs per cell, so their cells/s overstate the CPU's rate on the
    workload itself (about in the ratio of pairs per cell)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    gp = prep["gen_pat"]
    amb = [i for i, x in enumerate(gp) if x != "A"]
    fixed = {amb[0], amb[-1]}
    sub = "".join("A" if i in fixed else x for i, x in enumerate(gp))
    keep = [j for j, c in enumerate(prep["contexts"]) if all(c[i] == "A" for i in fixed)]
    ctxs = [prep["contexts"][i] for i in keep]
    Mf = prep["Mf"][keep]
    Uf = prep["Uf"][keep]
    nf = prep["nfolds"]
    bits = 8 * np.dtype(prep["itype"]).itemsize
    beta = {(g[1], g[0]): g[2] for g in prep["groups"]}
    tasks = [(a, [beta[(a, f)] for f in range(nf)], c) for a in prep["alphas"] for c in prep["penalties"]]
    O.lib()

    def one(task, threads=1):
        a, betas, c = task
        O.cv_pass(sub, ctxs, Mf, Uf, a, betas, c, bits, threads=threads)  # ctypes drops the GIL
    t0 = time.time()
    one(tasks[0])
    t1 = time.time() - t0
    cores = cores or host_cores()
    online = os.cpu_count()
    # memory: ~4.1 GB per concurrent 9-mer sample task
    par = max(1, min(cores, len(tasks)))
    t0 = time.time()
    with ThreadPoolExecutor(par) as ex:
        list(ex.map(one, [tasks[i % len(tasks)] for i in range(par)]))
    tn = time.time() - t0
    t0 = time.time()
    one(tasks[0], threads=cores)
    tomp = time.time() - t0
    units = O.npat(sub) * nf
    share = (f"{cores} = this job's CPU share of the {online}-CPU host (OMP_NUM_THREADS, set by the GPU pool "
             f"for one GPU; the host's other CPUs serve its other GPUs)") if online and online > cores else \
        f"{cores} = every online CPU"
    return {"value": units * par / tn, "unit": "cells*folds*(alpha,c)/s", "cores": par, "kind": "port",
            "host_cpus_online": online, "cpu_share": share,
            "all_cpus_extrapolated": (units * par / tn) / par * online if online else None,
            "single_core_value": units / t1,
            "sample_pairs_per_cell": pairs_per_cell(sub), "workload_pairs_per_cell": pairs_per_cell(gp),
            "sample": f"oracle/kp_oracle.c kpo_cv (1 thread per task) on sub-lattice {sub} of the same counts "
                      f"({O.npat(sub)} cells x {nf} folds per (alpha,c) task, {pairs_per_cell(sub):.2f} split pairs "
                      f"per cell against the workload's {pairs_per_cell(gp):.2f}): {par} concurrent tasks on "
                      f"{par} host cores in {tn:.1f} s; 1 task alone on 1 core in {t1:.1f} s",
            "openmp": {"value": units / tomp, "threads": cores,
                       "sample": f"kpo_cv, one (alpha,c) task on {sub} with each level's cells split over "
                                 f"{cores} OpenMP threads: {tomp:.1f} s"},
            "python": python_baseline(prep, tasks, par)}


def python_baseline(prep, tasks, par):
    """The reference-equivalent pure-Python path (oracle/pyref.py: the reference's CV pass
    as plain Python, what it runs without numba) on a smaller sample of the same counts --
    the four outermost ambiguous positions fixed to 'A' (151,875 cells for the 9-mer) --
    one (alpha, c) task per host core, each in its own Python process (the README's
    one-process-per-grid-point fan-out)."""
    import subprocess
    import tempfile
    from oracle import oracle as O
    gp = prep["gen_pat"]
    amb = [i for i, x in enumerate(gp) if x != "A"]
    fixed = set(amb[:2] + amb[-2:])
    sub = "".join("A" if i in fixed else x for i, x in enumerate(gp))
    keep = [j for j, c in enumerate(prep["contexts"]) if all(c[i] == "A" for i in fixed)]
    ctxs = [prep["contexts"][i] for i in keep]
    nf = prep["nfolds"]
    M = O._scatter(sub, ctxs, prep["Mf"][keep], nf)
    U = O._scatter(sub, ctxs, prep["Uf"][keep], nf)
    bits = 8 * np.dtype(prep["itype"]).itemsize
    with tempfile.TemporaryDirectory() as tmp:
        paths = []
        for i in range(par):
            a, betas, c = tasks[i % len(tasks)]
            paths.append(os.path.join(tmp, f"t{i}.npz"))
            np.savez(paths[-1], gen_pat=sub, M=M, U=U, alpha=a, betas=np.array(betas), penalty=c, itype_bits=bits)
        t0 = time.time()
        procs = [subprocess.Popen([sys.executable, "-m", "oracle.pyref", p], cwd=ROOT, stdout=subprocess.PIPE,
                                  text=True) for p in paths]
        outs = [pr.communicate()[0] for pr in procs]
        tn = time.time() - t0
        if any(pr.returncode for pr in procs):
            raise RuntimeError("pure-Python baseline task failed")
    secs = [float(o.split()[-1]) for o in outs]
    units = O.npat(sub) * nf
    online = os.cpu_count()
    return {"value": units * par / tn, "unit": "cells*folds*(alpha,c)/s", "cores": par,
            "kind": "reference-equivalent pure Python (oracle/pyref.py)",
            "single_core_value": units / (sum(secs) / len(secs)),
            "all_cpus_extrapolated": (units * par / tn) / par * online if online else None,
            "sample_pairs_per_cell": pairs_per_cell(sub), "workload_pairs_per_cell": pairs_per_cell(gp),
            "sample": f"oracle/pyref.py cv_pass on sub-lattice {sub} of the same counts ({O.npat(sub)} cells x "
                      f"{nf} folds per (alpha,c) task, {pairs_per_cell(sub):.2f} split pairs per cell against the "
                      f"workload's {pairs_per_cell(gp):.2f}): {par} processes on {par} host cores in {tn:.1f} s "
                      f"(per task {min(secs):.1f}-{max(secs):.1f} s)"}


def committed_traffic(gen_pat, n_lanes, kernel_tag):
    """HBM bytes per DP pass measured with rocprofv3 PMC counters: the newest
    profiles/<round>/pmc_*.json (tools/pmc_json.py) taken with the same kernel build."""
    import glob
    best = None
    for fn in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_*.json"))):
        try:
            d = json.load(open(fn))
        except ValueError:
            continue
        if d.get("gen_pat") == gen_pat and d.get("lanes") == n_lanes and d.get("kernel_tag") == kernel_tag:
            best = dict(d, source=os.path.relpath(fn, ROOT))
    return best


def cv_shares(prep, world, cap, width=None):
    """The passes each of ``world`` ranks runs for the full grid (lane-granular shares,
    kmerpapa_amd.shard.rank_groups, in engine.plan_passes' fold order, at most ``cap`` lanes
    per pass, fold pieces of ``width`` lanes)."""
    from kmerpapa_amd.engine import plan_passes
    from kmerpapa_amd.shard import rank_groups
    return [plan_passes(rank_groups(prep["groups"], r, world), cap, width)[0] for r in range(world)]


def cv_run(plan, prep, gen_pat, groups):
    """One job's CV work as the CV driver runs it (cv_roots with the engine): the fold
    split drawn on a host thread and handed over fold by fold, the all-data counts in k-mer
    order computed beside fold 0's draw (CV_tools.fold_feed -> engine.FoldFeed), the plan's table build beside it (a
    second build, timed), then ``groups``' passes in fold order, each fold uploaded when
    it arrives (engine.run_groups).  Lane buffers are already allocated (the one-time
    allocation is reported separately).  Returns the wall-clock and its parts."""
    import threading
    from kmerpapa_amd.CV_tools import fold_feed
    nf, itype = prep["nfolds"], prep["itype"]
    box = {}
    t0 = time.perf_counter()

    def tables():
        box["p"] = engine.Plan(plan.device, gen_pat, 0)
        box["t_tables"] = time.perf_counter() - t0
    th = threading.Thread(target=tables)
    th.start()
    feed, pr = fold_feed(prep["ctx"], gen_pat, nf, np.random.RandomState(1), itype)
    th.join()
    t_start = time.perf_counter() - t0
    engine.PASS_LOG = log = []
    try:
        engine.run_groups(gen_pat, feed, None, groups, devices=[plan.device.device])
    finally:
        engine.PASS_LOG = None
    pr.join()
    wall = time.perf_counter() - t0
    box["p"].close()
    fold_t = [t - t0 for t in feed.t_put]
    return {"wall_s": wall, "plan_tables_s": box["t_tables"], "fold_ready_s": [round(x, 4) for x in fold_t],
            "fold_split_s": fold_t[-1], "passes_start_s": t_start, "lanes": sum(len(g[3]) for g in groups),
            # per pass: lanes, [counts wait + upload, start, end] in s from the job's start
            "passes": [[n, round(w, 4), round(a - t0, 4), round(b - t0, 4)] for _, n, w, a, b, _ in log],
            # the sweep kernels' HIP-event time and compulsory bytes over the share's passes
            "kernel_ms": sum(st.get("dp_ms", 0.0) for *_, st in log),
            "compulsory_bytes": sum(st.get("gather_bytes", 0.0) for *_, st in log),
            "units": sum(st.get("units", 0) for *_, st in log)}


def shadow_host_side(prep, gen_pat):
    """The host work every rank of a multi-GPU job does before and beside its passes (cv_run
    without the passes): the plan's host-side table build, the all-data counts in k-mer
    order and the whole fold split drawn fold by fold.  No GPU: a shadow rank must not hold
    a context on the GPU the modelled rank measures on (other processes' contexts and
    queues on the same device slowed its passes ~2x), while a real rank has a GPU of its
    own."""
    from kmerpapa_amd.CV_tools import all_counts, fold_stream
    nf, itype = prep["nfolds"], prep["itype"]
    nk = engine.plan_info(gen_pat)["n_kmers"]
    contexts, Ma, Ua = all_counts(prep["ctx"], itype)
    idx = engine.kmer_order(gen_pat, contexts)
    M_all = np.zeros(nk, itype)
    M_all[idx] = Ma
    for f, Mf, Uf in fold_stream(prep["ctx"], nf, np.random.RandomState(1), itype):
        mk = np.zeros(nk, itype)
        mk[idx] = Mf


def shadow_main(config, gen_pat):
    """``bench.py --shadow``: a stand-in for another rank's process.  Prepares the same
    counts, says "ready", then runs shadow_host_side once per "go" line on stdin, answering
    "done SECONDS"; exits on EOF."""
    cfg = dict(CONFIGS[config])
    prep = prepare(gen_pat, alphas=cfg["alphas"], penalties=cfg["penalties"], nfolds=cfg["nfolds"])
    print("ready", flush=True)
    for line in sys.stdin:
        if line.strip() != "go":
            continue
        t0 = time.perf_counter()
        shadow_host_side(prep, gen_pat)
        print(f"done {time.perf_counter() - t0:.4f}", flush=True)


class Shadows:
    """Pool of shadow rank processes (``bench.py --shadow``), one Python process each -- as
    the ranks of a real job are -- so the modelled rank sees N concurrent host sides with
    their own interpreters and GILs."""

    def __init__(self, n, config, gen_pat):
        import subprocess
        self.procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--shadow", "--config", config,
                                        "--pattern", gen_pat], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                       text=True, cwd=ROOT) for _ in range(n)]
        for p in self.procs:
            if p.stdout.readline().strip() != "ready":
                raise RuntimeError("shadow rank failed to start")

    def go(self, n):
        for p in self.procs[:n]:
            p.stdin.write("go\n")
            p.stdin.flush()

    def wait(self, n):
        out = []
        for p in self.procs[:n]:
            line = p.stdout.readline().split()
            if not line or line[0] != "done":
                raise RuntimeError("shadow rank failed")
            out.append(float(line[1]))
        return out

    def close(self):
        for p in self.procs:
            p.stdin.close()
            p.wait(timeout=60)


def note(msg):
    """A progress line on stderr (the JSON line is stdout's only content)."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def model_world(plan, prep, gen_pat, world, shadows):
    """Modelled wall-clock of the full CV on ``world`` GPUs: every rank's lane-granular share
    (shard.rank_groups) is run as that rank runs it (cv_run: its own pipelined fold split,
    table build and passes), one share after the other on this GPU, each while world - 1
    shadow rank processes do the other ranks' host side at the same time
    (shadow_host_side).  Only the GPU part is serialised; there is no data-path collective
    (SURVEY.md 8e), so the job's wall-clock is the slowest share."""
    from kmerpapa_amd.shard import rank_groups
    shares, shadow_s = [], []
    for r in range(world):
        shadows.go(world - 1)
        shares.append(cv_run(plan, prep, gen_pat, rank_groups(prep["groups"], r, world)))
        shadow_s += shadows.wait(world - 1)
        note(f"model {world} GPUs: share {r} {shares[-1]['wall_s']:.2f} s")
    alloc = [prep["t_alloc"] for _ in shares]  # every rank's GPU in the state this one was in
    fracs = [x["compulsory_bytes"] / (x["kernel_ms"] / 1e3) / 1e9 / PEAK_HBM_GBS for x in shares if x["kernel_ms"]]
    return {"world": world, "share_s": [round(x["wall_s"], 4) for x in shares],
            "share_lanes": [x["lanes"] for x in shares],
            # each rank allocates its lane buffers once, in parallel with the others, and waits
            # as long as this run's allocation did (the wait is the driver finishing its wipe of
            # HBM earlier processes freed, not a cost per byte allocated: DESIGN.md 2)
            "share_hbm_alloc_s": [round(a, 4) for a in alloc],
            "wall_s_incl_alloc": max(x["wall_s"] + a for x, a in zip(shares, alloc)),
            "units": sum(x["units"] for x in shares),
            "share_kernel_ms": [round(x["kernel_ms"], 2) for x in shares],
            "share_effective_roofline_frac": [round(f, 4) for f in fracs],
            "share_passes_start_s": [round(x["passes_start_s"], 4) for x in shares],
            "share_fold_split_s": [round(x["fold_split_s"], 4) for x in shares],
            "share_fold0_s": [x["fold_ready_s"][0] for x in shares],
            "share_passes": [x["passes"] for x in shares],
            "shadow_host_side_s": [round(min(shadow_s), 4), round(max(shadow_s), 4)] if shadow_s else None,
            "wall_s": max(x["wall_s"] for x in shares)}


def full_cv(plan, prep, gen_pat, rank, world, cap, model_worlds=(2, 4, 8)):
    """The whole grid x folds as the CV driver runs it (cv_run: pipelined fold split,
    this rank's lane-granular share of the passes in fold order, root read-out) on the plan
    the timed steps used.  The one-time HBM allocation of the lane buffers happened before
    (the run's widest pass); ``wall_s`` excludes it and ``wall_s_incl_alloc`` adds it as
    measured.  On this platform that time is a wait for the driver to finish wiping HBM
    that earlier processes freed (~36 GB/s of freed bytes, whatever the request's size;
    1 ms for 150 GB on a GPU idle for a few seconds: tools/alloc_seq.sh).  At
    world 1 it also models the wall-clock of a job on 2, 4 and 8 GPUs (model_world), each
    rank waiting as long in parallel."""
    from kmerpapa_amd.shard import rank_groups
    out = cv_run(plan, prep, gen_pat, rank_groups(prep["groups"], rank, world))
    note(f"full CV (rank {rank} of {world}) {out['wall_s']:.2f} s")
    out["hbm_alloc_s"] = prep["t_alloc"]
    out["wall_s_incl_alloc"] = out["wall_s"] + out["hbm_alloc_s"]
    if world == 1 and model_worlds:
        out["models"] = {}
        shadows = Shadows(max(model_worlds) - 1, prep["config"], gen_pat)
        try:
            for w in model_worlds:
                m = model_world(plan, prep, gen_pat, w, shadows)
                m["speedup"] = out["wall_s"] / m["wall_s"]
                m["speedup_incl_alloc"] = out["wall_s_incl_alloc"] / m["wall_s_incl_alloc"]
                out["models"][str(w)] = m
        finally:
            shadows.close()
    return out


def scaling_table(line, cv, prep, npat, world=1):
    """patterns scored/s, kernel roofline fraction and CV wall-clock (with and without the
    one-time lane allocation) at every GPU count north_star names: N = 1 measured (the
    line's own step rate and roofline, the full CV run), N = 2, 4, 8 modelled (model_world:
    every rank's share run on this GPU beside N - 1 concurrent host sides).  units_per_s =
    the whole grid's units (cells x folds x (alpha, c)) / CV wall-clock; effective_roofline_frac
    = the sweep kernels' compulsory (algorithmic) bytes / their HIP-event time / 8 TB/s, per
    GPU (min and mean over the ranks; the measured line's also as roofline_frac, its PMC-based
    headline fraction); weak_units_per_s = N x the measured per-GPU step rate (what the
    driver's scaling run measures).  Under torchrun (world > 1) the entry of N = world is the
    measured job itself (wall-clock max over ranks) and nothing is modelled."""
    total = npat * sum(len(g[3]) for g in prep["groups"])
    out = {str(world): {"units_per_s": total / cv["wall_s"], "units_per_s_incl_alloc": total / cv["wall_s_incl_alloc"],
                 "effective_roofline_frac": line["roofline"]["effective_frac"],
                 "effective_roofline_frac_min": line["roofline"]["effective_frac"],
                 "roofline_frac": line["roofline"]["frac"],
                 "wall_s": cv["wall_s"], "wall_s_incl_alloc": cv["wall_s_incl_alloc"],
                 "hbm_alloc_s": cv["hbm_alloc_s"], "weak_units_per_s": line["value"], "measured": True}}
    for w, m in (cv.get("models") or {}).items():
        fr = m["share_effective_roofline_frac"]
        out[w] = {"units_per_s": total / m["wall_s"], "units_per_s_incl_alloc": total / m["wall_s_incl_alloc"],
                  "effective_roofline_frac": sum(fr) / len(fr) if fr else None,
                  "effective_roofline_frac_min": min(fr) if fr else None,
                  "wall_s": m["wall_s"], "wall_s_incl_alloc": m["wall_s_incl_alloc"],
                  "hbm_alloc_s": max(m["share_hbm_alloc_s"]), "speedup": m["speedup"],
                  "speedup_incl_alloc": m["speedup_incl_alloc"], "weak_units_per_s": int(w) * line["value"],
                  "measured": False}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="9mer", choices=sorted(CONFIGS),
                    help="9mer = BASELINE configs[3] (the headline); 11mer = configs[4] (super-pattern restricted)")
    ap.add_argument("--pattern", default=None, help="override the config's general pattern")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-cores", type=int, default=0,
                    help="host cores for the CPU baseline (default: this job's CPU share, host_cores())")
    ap.add_argument("--max-block", type=int, default=0)
    ap.add_argument("--no-full-cv", action="store_true", help="skip the full grid CV wall-clock leg")
    ap.add_argument("--model-worlds", default="2,4,8",
                    help="GPU counts whose full-CV wall-clock is modelled at N=1 (comma list, empty = none)")
    ap.add_argument("--shadow", action="store_true", help=argparse.SUPPRESS)  # a modelled rank's host side
    a = ap.parse_args()
    if a.shadow:
        return shadow_main(a.config, a.pattern or CONFIGS[a.config]["gen_pat"])

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # host-side barrier / max only (no data-path collective)
        dist.init_process_group("gloo")

    cfg = dict(CONFIGS[a.config])
    if a.pattern:
        cfg["gen_pat"] = a.pattern
    gen_pat = cfg["gen_pat"]
    prep = prepare(gen_pat, alphas=cfg["alphas"], penalties=cfg["penalties"], nfolds=cfg["nfolds"])
    prep["config"] = a.config
    ndev = engine.device_count()
    prep["device"] = local % max(1, ndev)  # one GPU per rank (several ranks per GPU only in rehearsals)
    groups = prep["groups"]

    def barrier():
        if dist is not None:
            dist.barrier()

    def max_over_ranks(x):
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    t0 = time.perf_counter()
    plan = engine.get_plan(prep["device"], gen_pat, a.max_block)
    prep["t_plan"] = time.perf_counter() - t0
    plan.set_counts(prep["Mk"], prep["Uk"])  # first: the count width sets lanes_per_workgroup
    width = plan.info["lanes_per_workgroup"]
    cap = engine.pass_cap(groups, plan.lanes_that_fit(), width)
    # a step = one pass of the whole grid's CV plan on one GPU (engine.plan_passes: fold
    # pieces of one workgroup's lanes; 9-mer: one (alpha, fold) group of 5 penalties; 11-mer:
    # 5 of a fold's 49 (alpha, c) lanes, some spanning two alphas)
    step_passes = engine.plan_passes(groups, cap, width)[0]
    model_worlds = tuple(int(x) for x in a.model_worlds.split(",") if x.strip())
    worlds = () if a.no_full_cv else ((world,) + model_worlds if world == 1 else (world,))
    most = max([sum(len(g[3]) for g in p) for p in step_passes] +
               [sum(len(g[3]) for g in p) for w in worlds for passes in cv_shares(prep, w, cap, width) for p in passes])
    t0 = time.perf_counter()
    plan.reserve(most)  # the one large allocation of the run: the widest pass any modelled rank runs
    prep["t_alloc"] = time.perf_counter() - t0
    prep["alloc_lanes"] = most

    def step(s):
        plan.run(step_passes[(s * world + rank) % len(step_passes)])
        return plan.stats()

    for s in range(a.warmup):
        step(s)

    barrier()
    t_start = time.perf_counter()
    stats = [step(a.warmup + s) for s in range(a.steps)]
    t_end = time.perf_counter()
    barrier()
    elapsed = max_over_ranks(t_end - t_start)
    note(f"{a.steps} timed steps {elapsed / a.steps * 1e3:.1f} ms/step")

    # BASELINE.json's second metric: the full grid CV wall-clock (fold split, count tables,
    # passes, root read-out), max over ranks; at N=1 also the modelled 8-GPU wall-clock
    cv = None
    if not a.no_full_cv:
        barrier()
        cv = full_cv(plan, prep, gen_pat, rank, world, cap, model_worlds)
        cv["wall_s_incl_alloc"] = max_over_ranks(cv["wall_s_incl_alloc"])  # (each rank: its wall + its allocation)
        cv["hbm_alloc_s"] = max_over_ranks(cv["hbm_alloc_s"])
        cv["wall_s"] = max_over_ranks(cv["wall_s"])

    units_rank = sum(s["units"] for s in stats)
    units = units_rank * world
    dp_ms = sum(s["dp_ms"] for s in stats)
    launches = sum(s["dp_launches"] for s in stats)
    dp_s = dp_ms / 1e3
    must = sum(s["gather_bytes"] for s in stats)  # (8 P_high + 4) B per unit, blocked sweep
    naive = sum(s["alg_bytes"] for s in stats)     # SURVEY.md 8(d) per-cell figure
    floor = 8.0 * units_rank                       # every row read once + written once
    lanes = round(units_rank / a.steps / plan.info["npat"])  # lanes per step (pieces of a fold may be narrower)
    tag = engine.kernel_tag()
    tr = committed_traffic(gen_pat, lanes, tag)

    if rank == 0:
        ms_step = elapsed / a.steps * 1e3
        eff_gbs = must / dp_s / 1e9
        roof = {"bound": "hbm", "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "traffic": (tr["hbm_bytes_per_pass"] if tr else None),
                "kernel": "kp_dp_kernel (all launches of one pass)",
                "kernel_ms_per_pass": dp_ms / a.steps, "launches_per_pass": launches / a.steps,
                "avg_launch_ms": dp_ms / max(1, launches),
                # effective (algorithmic) bandwidth: the bytes the blocked sweep must move
                "effective_gbs": eff_gbs, "effective_frac": eff_gbs / PEAK_HBM_GBS,
                "effective_bytes_per_unit": must / units_rank,
                "effective_basis": "ALGORITHMIC bytes, not a measured HBM rate: (8 P_high + 4) B per unit (two "
                                   "child-row reads per high-position split pair + one score write; DESIGN.md 3) / "
                                   "HIP-event time of the pass's kp_dp_kernel launches; part of those bytes are "
                                   "Infinity-Cache and L2 hits, so it can exceed what HBM delivers",
                "floor_bytes_per_unit": 8.0, "floor_frac": floor / dp_s / 1e9 / PEAK_HBM_GBS,
                "naive_equivalent_bytes_per_unit": naive / units_rank,
                "naive_equivalent_gbs": naive / dp_s / 1e9}
        if tr:
            # the headline fraction: MEASURED fabric bytes (PMC) over the same kernel time
            roof["achieved"] = tr["hbm_bytes_per_pass"] / (dp_s / a.steps) / 1e9
            roof["frac"] = roof["achieved"] / PEAK_HBM_GBS
            roof["frac_basis"] = ("fabric (L2-miss, includes Infinity-Cache hits) - upper bound on HBM: rocprofv3 "
                                  "FETCH_SIZE x2 + WRITE_SIZE over the pass's kp_dp_kernel dispatches (committed "
                                  "profile at this kernel_tag) / HIP-event kernel time of this run; no gfx950 "
                                  "counter separates Infinity-Cache hits from DRAM reads (DESIGN.md 5)")
            roof["traffic_source"] = tr.get("source")
        else:
            roof["achieved"] = eff_gbs
            roof["frac"] = eff_gbs / PEAK_HBM_GBS
            roof["frac_basis"] = "effective (no PMC profile committed at this kernel_tag): see effective_basis"
        n_gpus = min(world, max(1, ndev))
        line = {
            "metric": "patterns scored/sec (lattice cells x folds x (alpha,c)), 9-mer 5-fold CV 5x5 grid"
                      if (a.config == "9mer" and not a.pattern) else
                      f"patterns scored/sec, general pattern {gen_pat} ({a.config} config)",
            "value": units / elapsed,
            "unit": "cell-scores/s",
            "n_gpus": n_gpus,
            "ranks": world,
            "rehearsal": world > n_gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": f"f32 (scores, split sums) + f64 (single-pattern term); "
                     f"u{8 * np.dtype(prep['itype']).itemsize} counts",
            "data": "synthetic",
            "config": {"workload": f"synthetic {len(gen_pat)}-mer counts, general pattern {gen_pat} "
                                   f"({plan.info['npat']} cells), {len(prep['alphas'])}x{len(prep['penalties'])} "
                                   f"(alpha, c) grid, {prep['nfolds']}-fold CV; step = one pass of the grid's CV plan: "
                                   f"{lanes} (alpha, fold, c) lanes of one fold over the whole lattice",
                       "name": a.config, "gen_pat": gen_pat, "cells": plan.info["npat"], "lanes_per_step": lanes,
                       "units_per_step": plan.info["npat"] * lanes, "block_cells": plan.info["block"],
                       "alphas": prep["alphas"], "penalties": prep["penalties"], "nfolds": prep["nfolds"]},
            "roofline": roof,
            "backtrack_ms_per_step": sum(s["backtrack_ms"] for s in stats) / a.steps,
            "cv_full_grid_wall_s": cv["wall_s"] if cv else None,
            "cv_full_grid": cv,
            "fold_split_s": prep["t_fold_s"],

            "kernel_tag": tag,
        }
        if cv:
            line["scaling_by_gpus"] = scaling_table(line, cv, prep, plan.info["npat"], world)
            line["hbm_alloc"] = {"lanes": prep["alloc_lanes"], "s": prep["t_alloc"],
                                 "bytes": prep["alloc_lanes"] * plan.info["bytes_per_lane"]}
        if cv and "models" in cv:
            line["cv_full_grid_wall_s_model"] = {w: m["wall_s"] for w, m in cv["models"].items()}
            line["cv_full_grid_speedup_model"] = {w: m["speedup"] for w, m in cv["models"].items()}
            if "8" in cv["models"]:
                line["cv_full_grid_wall_s_model_8gpu"] = cv["models"]["8"]["wall_s"]
                line["cv_full_grid_speedup_model_8gpu"] = cv["models"]["8"]["speedup"]
        if not a.no_cpu_baseline and world == 1:
            note("cpu baseline")
            line["cpu_baseline"] = cpu_baseline(prep, a.cpu_cores or None)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

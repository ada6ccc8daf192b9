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
The roofline object prices the DP sweep kernel (kp_dp_kernel): algorithmic bytes per
SURVEY.md §8d (16 B per split pair, 8 B per cell written, 6 s per aggregated cell, 2 s
per k-mer, per lane) over the HIP-event duration of its launches; "traffic" is the
PMC-measured HBM bytes per pass (profiles/, rocprofv3 FETCH_SIZE/WRITE_SIZE with the
gfx950 x2 FETCH correction) when a matching profile summary is committed.
The cpu_baseline leg times the CPU oracle (oracle/kp_oracle.c, a single-threaded C
port of the reference's DP) on a bounded sample of the same counts.
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


def prepare(gen_pat, seed=1, alphas=ALPHAS, penalties=PENALTIES, nfolds=NFOLDS):
    """Fold split (reference RNG stream) and betas for every (alpha, fold)."""
    kmers, M, U = synthetic_counts(gen_pat)
    ctx = {k: (int(m), int(u)) for k, m, u in zip(kmers, M, U)}
    total = int(M.sum() + U.sum())
    itype = np.uint64 if total > np.iinfo(np.uint32).max else np.uint32
    t0 = time.time()
    contexts, Mf, Uf = fold_tables(ctx, nfolds, np.random.RandomState(seed), itype)
    t_fold = time.time() - t0
    Mk, Uk = engine.counts_in_kmer_order(gen_pat, contexts, Mf, Uf, generality(gen_pat), itype)
    msum = Mk.sum(axis=0, dtype=np.uint64)
    usum = Uk.sum(axis=0, dtype=np.uint64)
    mtr, utr = msum.sum() - msum, usum.sum() - usum
    groups = []
    for a in alphas:
        my = mtr / (mtr + utr)
        betas = (a * (1.0 - my)) / my
        for f in range(nfolds):
            groups.append((f, a, float(betas[f]), list(penalties)))
    return {"Mk": Mk, "Uk": Uk, "groups": groups, "itype": itype, "t_fold_s": t_fold, "contexts": contexts,
            "Mf": Mf, "Uf": Uf, "total": total, "gen_pat": gen_pat, "alphas": list(alphas),
            "penalties": list(penalties), "nfolds": nfolds}


def cpu_baseline(prep, seconds_hint=15.0):
    """Time the single-threaded CPU oracle on a bounded sample of the same counts: the
    sub-lattice with the two outermost ambiguous positions fixed to 'A' (3.4e7 cells),
    one (alpha, c) over all folds."""
    from oracle import oracle as O
    gp = prep["gen_pat"]
    # fix the two outermost still-ambiguous positions to A: a 15^6 x 3 = 3.4e7-cell sample
    amb = [i for i, x in enumerate(gp) if x != "A"]
    fixed = {amb[0], amb[-1]}
    sub = "".join("A" if i in fixed else x for i, x in enumerate(gp))
    keep = [j for j, c in enumerate(prep["contexts"]) if all(c[i] == "A" for i in fixed)]
    ctxs = [prep["contexts"][i] for i in keep]
    Mf = prep["Mf"][keep]
    Uf = prep["Uf"][keep]
    g = prep["groups"][0]
    nf = prep["nfolds"]
    betas = [prep["groups"][f][2] for f in range(nf)]
    bits = 8 * np.dtype(prep["itype"]).itemsize
    t0 = time.time()
    O.cv_pass(sub, ctxs, Mf, Uf, g[1], betas, g[3][0], bits)
    dt = time.time() - t0
    units = O.npat(sub) * nf
    return {"value": units / dt, "unit": "cells*folds*(alpha,c)/s", "cores": 1, "kind": "port",
            "sample": f"oracle/kp_oracle.c kpo_cv on sub-lattice {sub} of the same counts "
                      f"({O.npat(sub)} cells x {nf} folds, 1 (alpha,c)) in {dt:.1f} s on 1 host core"}


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


def full_cv(plan, prep, rank, world):
    """The whole 5x5 grid x 5 folds as the CV driver runs it: this rank's share of the
    (alpha, fold) groups, one pass each, root read-out included."""
    from kmerpapa_amd.engine import pack_passes
    from kmerpapa_amd.shard import rank_groups
    t0 = time.perf_counter()
    mine = rank_groups(prep["groups"], rank, world)  # lane-granular share (15-16 lanes at N=8)
    roots = [plan.run(p) for p in pack_passes(mine, min(plan.lanes_that_fit(), 8))]
    return time.perf_counter() - t0, len(mine), roots


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="9mer", choices=sorted(CONFIGS),
                    help="9mer = BASELINE configs[3] (the headline); 11mer = configs[4] (super-pattern restricted)")
    ap.add_argument("--pattern", default=None, help="override the config's general pattern")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--max-block", type=int, default=0)
    ap.add_argument("--no-full-cv", action="store_true", help="skip the full 5x5x5 CV wall-clock leg")
    a = ap.parse_args()

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
    ndev = engine.device_count()
    dev = engine.get_device(local % max(1, ndev))  # one GPU per rank (several ranks per GPU only in rehearsals)
    t0 = time.time()
    plan = engine.Plan(dev, gen_pat, a.max_block)
    plan.set_counts(prep["Mk"], prep["Uk"])
    t_setup = time.time() - t0
    groups = prep["groups"]

    def step(s):
        g = groups[(s * world + rank) % len(groups)]
        plan.run([g])
        return plan.stats()

    for s in range(a.warmup):
        step(s)

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    t_start = time.perf_counter()
    stats = [step(a.warmup + s) for s in range(a.steps)]
    t_end = time.perf_counter()
    barrier()
    elapsed = t_end - t_start
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    units_rank = sum(s["units"] for s in stats)
    units = units_rank * world
    dp_ms = sum(s["dp_ms"] for s in stats)
    alg = sum(s["alg_bytes"] for s in stats)
    achieved = alg / (dp_ms / 1e3) / 1e9
    lanes = len(groups[0][3])
    tag = engine.kernel_tag()
    tr = committed_traffic(gen_pat, lanes, tag)

    # 9-mer 5-fold CV wall-clock (BASELINE.json's second metric): fold split (host, every
    # rank) + this rank's passes, max over ranks
    cv_wall = None
    if not a.no_full_cv:
        barrier()
        t_cv, n_mine, _ = full_cv(plan, prep, rank, world)
        cv_wall = prep["t_fold_s"] + t_setup + t_cv
        if dist is not None:
            import torch
            t = torch.tensor([cv_wall], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            cv_wall = float(t.item())
    if rank == 0:
        ms_step = elapsed / a.steps * 1e3
        passes_full_cv = math.ceil(len(groups) / world)
        line = {
            "metric": "patterns scored/sec (lattice cells x folds x (alpha,c)), 9-mer 5-fold CV 5x5 grid"
                      if (a.config == "9mer" and not a.pattern) else
                      f"patterns scored/sec, {a.config} config, general pattern {gen_pat}",
            "value": units / elapsed,
            "unit": "cell-scores/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 (scores, split sums) + f64 (single-pattern term); u32 counts",
            "data": "synthetic",
            "config": {"workload": f"synthetic {len(gen_pat)}-mer counts, general pattern {gen_pat} "
                                   f"({plan.info['npat']} cells), {len(prep['alphas'])}x{len(prep['penalties'])} "
                                   f"(alpha, c) grid, {prep['nfolds']}-fold CV; step = one (alpha, fold) group x "
                                   f"{lanes} penalties over the whole lattice",
                       "name": a.config, "gen_pat": gen_pat, "cells": plan.info["npat"], "lanes_per_step": lanes,
                       "units_per_step": plan.info["npat"] * lanes, "block_cells": plan.info["block"],
                       "alphas": prep["alphas"], "penalties": prep["penalties"], "nfolds": prep["nfolds"]},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBS,
                         "traffic": (tr["hbm_bytes_per_pass"] if tr else None),
                         "kernel": "kp_dp_kernel (all launches of one pass)",
                         "alg_bytes_per_pass": alg / a.steps,
                         "alg_bytes_per_unit": alg / units_rank,
                         "basis": "SURVEY.md 8(d) per-unit algorithmic bytes x units / HIP-event time of the "
                                  "pass's kp_dp_kernel launches; traffic = PMC HBM bytes per pass"},
            "dp_kernel_ms_per_step": dp_ms / a.steps,
            "dp_kernel_launches_per_step": sum(s["dp_launches"] for s in stats) / a.steps,
            "dp_kernel_avg_launch_ms": dp_ms / max(1, sum(s["dp_launches"] for s in stats)),
            "backtrack_ms_per_step": sum(s["backtrack_ms"] for s in stats) / a.steps,
            "cv_full_grid_wall_s": cv_wall,
            "cv_full_grid_wall_s_estimate": prep["t_fold_s"] + t_setup + passes_full_cv * ms_step / 1e3,
            "fold_split_s": prep["t_fold_s"],
            "setup_s": t_setup,
            "kernel_tag": tag,
        }
        if tr:
            line["roofline"]["traffic_source"] = tr.get("source")
            line["roofline"]["traffic_gbs"] = tr["hbm_bytes_per_pass"] / (dp_ms / a.steps / 1e3) / 1e9
            line["roofline"]["traffic_frac"] = line["roofline"]["traffic_gbs"] / PEAK_HBM_GBS
        if not a.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(prep)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

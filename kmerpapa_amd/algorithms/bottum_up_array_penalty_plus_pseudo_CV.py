"""Cross-validated penalized-likelihood pattern partition -- drop-in for the reference's
``kmerpapa.algorithms.bottum_up_array_penalty_plus_pseudo_CV`` (v0.2.4).

``pattern_partition_bottom_up(gen_pat, contextD, alphas, args, nmut, nunmut, penalties,
index_mut=0)`` keeps the reference's signature, return value ``(best_alpha,
best_penalty, best_test_loss)``, stderr lines and CVfile rows (CV module :81-177).

What moved to the GPU: the whole level sweep (CV :143-157, ``handle_pattern`` :26-78 and
``score_test_folds`` :15-20) for every (alpha, penalty, fold) at once -- one lane per
(penalty, fold), lanes of one (alpha, fold) sharing counts -- and the root read-out
(:158-163).  What stays on the host, bit-identical to the reference: the fold split
(``RandomState.hypergeometric`` stream, CV :124-130), fold totals and betas (:134-141),
the numpy<2 float64 sum of the root test values (:159, :171), the strict-"<" selection
in alpha-major order (:165-177).
"""
import sys
import threading

import numpy as np

from .. import engine
from ..CV_tools import fold_feed, fold_tables
from ..pattern_utils import code, generality, pattern_level, perm_code
from ..score_utils import get_betas
from ..shard import fold_order


def _itype(nmut, nunmut):
    """uint32 unless the totals need 64 bits (CV :94-97)."""
    return np.uint64 if nmut + nunmut > np.iinfo(np.uint32).max else np.uint32


def _cells_per_kmer(gen_pat):
    """For every k-mer (KmerEnumeration order): number of lattice cells that contain it."""
    mult = np.ones(1, dtype=np.uint64)
    for g in gen_pat:
        per = np.array([sum(1 for x in perm_code[g] if nuc in code[x]) for nuc in code[g]], dtype=np.uint64)
        mult = (per[:, None] * mult[None, :]).reshape(-1)  # position 0 fastest
    return mult


def cv_roots(gen_pat, contextD, alphas, penalties, nfolds, seed, iterations, itype, devices=None, verbose=0,
             max_block=0, run_groups=None):
    """Root train/test values of every (iteration, alpha, penalty, fold).

    Returns a dict with arrays ``train``/``test`` of shape
    ``[iterations, n_alpha, n_penalty, nfolds]`` (float32) and ``betas``
    ``[iterations, n_alpha, nfolds]``.  ``run_groups`` defaults to the GPU engine.

    With a runner that takes fold-by-fold counts (``run_groups.fold_feed``, the engine's),
    the fold split is drawn on a host thread (CV_tools.fold_stream) and handed over fold by
    fold (engine.FoldFeed): the GPUs start on fold 0 while the later folds are drawn, and
    a fold's betas are computed when it arrives.  Same draws, same numbers.
    """
    run_groups = run_groups or engine.run_groups
    pipelined = bool(getattr(run_groups, "fold_feed", False))
    prng = np.random.RandomState(seed)
    na, nc = len(alphas), len(penalties)
    train = np.zeros((iterations, na, nc, nfolds), np.float32)
    test = np.zeros((iterations, na, nc, nfolds), np.float32)
    betas_all = np.zeros((iterations, na, nfolds))
    n_kmers = generality(gen_pat)
    mult = None
    prevM = prevU = None
    prepare = getattr(run_groups, "prepare", None)
    for it in range(iterations):
        if verbose > 0 and iterations > 1:
            print('CV Iteration', it, file=sys.stderr)
        th = None
        box = {}
        if prepare is not None and it == 0:
            # the GPUs' lattice tables and lane buffers are set up while the host draws the
            # fold split (the native split releases the GIL); only lane counts and the
            # counts' width matter here (a multi-GPU share depends on the width)
            shape = [(f, a, 1.0, list(penalties[c0:c0 + engine.MAX_GROUP_LANES]))
                     for a in alphas for f in fold_order(nfolds) for c0 in range(0, nc, engine.MAX_GROUP_LANES)]

            def _prep():
                try:
                    prepare(gen_pat, shape, devices=devices, max_block=max_block, itype=itype)
                except Exception as e:  # re-raised below, in the caller's thread
                    box["error"] = e
            th = threading.Thread(target=_prep)
            th.start()
        # fold totals = column sums of M_mem over ALL rows (CV :134-137).  From the
        # second iteration on, the aggregated rows still hold the previous iteration's
        # sums: every k-mer count of the previous split appears once per containing
        # cell other than the k-mer itself.  Reproduced as the reference computes it.
        carryM = np.zeros(nfolds, np.uint64)
        carryU = np.zeros(nfolds, np.uint64)
        if prevM is not None:
            if mult is None:
                mult = _cells_per_kmer(gen_pat) - np.uint64(1)
            carryM = (prevM.astype(np.uint64) * mult[:, None]).sum(axis=0, dtype=np.uint64)
            carryU = (prevU.astype(np.uint64) * mult[:, None]).sum(axis=0, dtype=np.uint64)
        producer = None
        try:
            if pipelined:
                done = (lambda: print('CV sampling DONE', file=sys.stderr)) if verbose > 0 else None
                feed, producer = fold_feed(contextD, gen_pat, nfolds, prng, itype, on_done=done)
                M_all, U_all = feed.M_all, feed.U_all
                M_tot = M_all.sum(dtype=np.uint64) + carryM.sum(dtype=np.uint64)  # = M_sum.sum()
                U_tot = U_all.sum(dtype=np.uint64) + carryU.sum(dtype=np.uint64)
                counts_M, counts_U = feed, None
            else:
                contexts, Mf, Uf = fold_tables(contextD, nfolds, prng, itype)
                if verbose > 0:
                    print('CV sampling DONE', file=sys.stderr)
                Mk, Uk = engine.counts_in_kmer_order(gen_pat, contexts, Mf, Uf, n_kmers, itype)
                M_sum = Mk.sum(axis=0, dtype=np.uint64) + carryM
                U_sum = Uk.sum(axis=0, dtype=np.uint64) + carryU
                counts_M, counts_U = Mk, Uk
        finally:
            if th is not None:
                th.join()
        if th is not None and "error" in box:
            if producer is not None:
                producer.join()
            raise box["error"]

        lock = threading.Lock()
        cache = {}

        def fold_betas(f, feed=counts_M if pipelined else None):
            """Betas of fold f for every alpha (CV :138-141): get_betas over the fold's
            train totals M_sum.sum() - M_sum[f] (uint64, as the reference)."""
            with lock:
                if f not in cache:
                    if feed is not None:
                        Mfk, Ufk = feed.get(f)
                        mtr = np.array([M_tot - (Mfk.sum(dtype=np.uint64) + carryM[f])], np.uint64)
                        utr = np.array([U_tot - (Ufk.sum(dtype=np.uint64) + carryU[f])], np.uint64)
                    else:
                        mtr = (M_sum.sum() - M_sum)[f:f + 1]
                        utr = (U_sum.sum() - U_sum)[f:f + 1]
                    cache[f] = [float(get_betas(alpha, mtr, utr)[0]) for alpha in alphas]
                return cache[f]

        groups, where = [], []
        for a_i, alpha in enumerate(alphas):
            for f in fold_order(nfolds):  # fold 0 last (shard.fold_order); lanes map back by `where`
                beta = (lambda a_i=a_i, f=f: fold_betas(f)[a_i]) if pipelined else fold_betas(f)[a_i]
                for c0 in range(0, nc, engine.MAX_GROUP_LANES):
                    chunk = list(penalties[c0:c0 + engine.MAX_GROUP_LANES])
                    groups.append((f, alpha, beta, chunk))
                    where.extend((a_i, c0 + j, f) for j in range(len(chunk)))
        try:
            rt, re, _ = run_groups(gen_pat, counts_M, counts_U, groups, devices=devices, max_block=max_block)
        finally:
            if producer is not None:
                producer.join()
        for f in range(nfolds):
            betas_all[it, :, f] = fold_betas(f)
        for lane, (a_i, p_i, f) in enumerate(where):
            train[it, a_i, p_i, f] = rt[lane]
            test[it, a_i, p_i, f] = re[lane]
        if it + 1 < iterations:
            prevM, prevU = counts_M.arrays() if pipelined else (counts_M, counts_U)
        if verbose > 0:
            _report(gen_pat, alphas, penalties, it, test[it], verbose)
    return {"train": train, "test": test, "betas": betas_all}


def _report(gen_pat, alphas, penalties, it, test, verbosity):
    """stderr lines of one iteration, in the reference's pass order (CV :153-161)."""
    level = pattern_level(gen_pat)
    for a_i, alpha in enumerate(alphas):
        for p_i, penalty in enumerate(penalties):
            if verbosity > 1:
                for lv in range(1, level + 1):
                    print(f'level {lv} of {level}', file=sys.stderr)
            roots = test[a_i, p_i]
            print(f'CV on k={len(gen_pat)} alpha={alpha} penalty={penalty} i={it} test_LL={_f64_sum(roots)}',
                  file=sys.stderr)
            if verbosity > 1:
                print(f'test LL for each fold: {roots}', file=sys.stderr)


def _f64_sum(values):
    """sum() of float32 scalars under the reference's pinned numpy<2 (float64 accumulation)."""
    acc = 0.0
    for v in values:
        acc += float(v)
    return acc


def _distributed_runner():
    """Under torch.distributed (one process per GPU, e.g. torchrun), each rank runs its
    chunk of the groups on GPU LOCAL_RANK and the root scalars are all-gathered
    (kmerpapa_amd.shard); otherwise every visible GPU of this process is used.  torch is
    not imported here: a caller that set up a process group has imported it already."""
    try:
        dist = sys.modules.get("torch.distributed")
        if dist is not None and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            import os
            from ..shard import sharded_run_groups, torch_all_gather
            # one GPU per rank; more ranks than GPUs (a rehearsal) share them round-robin
            local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, engine.device_count())
            return sharded_run_groups(engine.run_groups, dist.get_rank(), dist.get_world_size(),
                                      torch_all_gather(), devices=[local]), [local]
    except ImportError:
        pass
    return engine.run_groups, engine.visible_devices()


def pattern_partition_bottom_up(gen_pat, contextD, alphas, args, nmut, nunmut, penalties, index_mut=0):
    """Grid CV over (alpha, penalty); returns ``(best_alpha, best_penalty, best_test_loss)`` (CV :81-177)."""
    nf = args.nfolds
    nit = args.iterations
    verbosity = getattr(args, "verbosity", 0) or 0
    itype = _itype(nmut, nunmut)
    if index_mut != 0:
        contextD = {k: (v[index_mut], v[-1]) for k, v in contextD.items()}
    run_groups, devices = _distributed_runner()
    res = cv_roots(gen_pat, contextD, list(alphas), list(penalties), nf, args.seed, nit, itype,
                   devices=devices, verbose=verbosity, run_groups=run_groups)
    best_test_loss = 1e100
    best_values = (None, None)
    for a_i, alpha in enumerate(alphas):
        for p_i, penalty in enumerate(penalties):
            vals = [res["test"][it, a_i, p_i, f] for it in range(nit) for f in range(nf)]
            test = _f64_sum(vals) / nit
            if args.CVfile is not None:
                print(len(gen_pat), alpha, penalty, test, file=args.CVfile)
            if test < best_test_loss:
                best_values = (alpha, penalty)
                best_test_loss = test
    return best_values[0], best_values[1], best_test_loss

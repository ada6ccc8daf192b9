"""Penalized-likelihood pattern partition on all data, with backtrack -- drop-in for the
reference's ``kmerpapa.algorithms.bottum_up_array_w_numba`` (v0.2.4).

``pattern_partition_bottom_up(gen_pat, contextD, alpha_, beta_, penalty_, args, nmut,
nunmut, index_mut=0)`` returns ``(score, M, U, names)`` exactly as Fit :67-124: the
root's float32 score, the root's total counts (itype scalars) and the optimal partition
as IUPAC patterns in backtrack order (Fit :17-24).  The sweep and the backtrack run on
the GPU (one lane, fold = -1); names are decoded on the host.
"""
import sys

import numpy as np

from .. import engine
from ..pattern_utils import PatternEnumeration, generality, pattern_level


def _itype(nmut, nunmut):
    return np.uint64 if nmut + nunmut > np.iinfo(np.uint32).max else np.uint32


def fit_partition(gen_pat, contextD, alpha, beta, penalty, itype, index_mut=0, device=None, max_block=0):
    """Run the Fit DP; returns ``(score f32, M_root, U_root, leaf cell indices)``."""
    if hasattr(contextD, "letters") and index_mut == 0:  # io_utils.KmerCounts (native reader)
        contexts, M, U = contextD, contextD.M.astype(itype), contextD.U.astype(itype)
    else:
        contexts = list(contextD.keys())
        M = np.array([contextD[c][index_mut] for c in contexts], dtype=itype)
        U = np.array([contextD[c][-1] for c in contexts], dtype=itype)
    Mk, Uk = engine.counts_in_kmer_order(gen_pat, contexts, M, U, generality(gen_pat), itype)
    dev = engine.visible_devices()[0] if device is None else device
    plan = engine.get_plan(dev, gen_pat, max_block)
    plan.set_counts(Mk, Uk)
    plan.require_lanes(1)  # a clean KPError (KP_E_NOMEM) if one lane does not fit the GPU
    rt, _, _ = plan.run([(-1, alpha, beta, [penalty])])
    leaves = plan.leaves(0)
    Mroot = itype(Mk.sum(dtype=np.uint64))
    Uroot = itype(Uk.sum(dtype=np.uint64))
    return rt[0], Mroot, Uroot, leaves


def pattern_partition_bottom_up(gen_pat, contextD, alpha_, beta_, penalty_, args, nmut, nunmut, index_mut=0):
    """Optimal partition of all data for one (alpha, beta, penalty) (Fit :67-124)."""
    verbosity = getattr(args, "verbosity", 0) or 0
    if verbosity > 1:
        level = pattern_level(gen_pat)
        for lv in range(1, level + 1):
            print(f'level {lv} of {level}', file=sys.stderr)
    score, M, U, leaves = fit_partition(gen_pat, contextD, alpha_, beta_, penalty_, _itype(nmut, nunmut),
                                        index_mut=index_mut)
    PE = PatternEnumeration(gen_pat)
    names = [PE.num2pattern(int(x)) for x in leaves]
    return np.float32(score), M, U, names

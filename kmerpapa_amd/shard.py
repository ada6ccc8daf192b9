"""Sharding of the cross-validation grid over ranks (one process per GPU).

The (alpha, fold) groups of a CV sweep are independent DP passes: each
rank runs a contiguous, lane-balanced chunk of the group list on its own GPU and the
per-lane root scalars (a few floats per lane) are gathered on the host.  Nothing on the
data path is exchanged -- every rank rebuilds the fold tables from the same seed -- so the
only collective is an all-gather of root scalars, over whatever process group the caller
set up (gloo is enough; the payload is bytes).

The reference has no parallelism at all; its "distribution" is a shell loop over
``--CV_only`` runs (README.md:39-51).  This replaces that loop inside one job.
"""
import numpy as np


def chunk_bounds(lane_counts, parts):
    """Split a list of groups (given their lane counts) into ``parts`` contiguous chunks of
    roughly equal lanes.  Returns ``parts + 1`` boundaries."""
    total = sum(lane_counts)
    bounds, acc, d = [0], 0, 0
    for i, n in enumerate(lane_counts):
        acc += n
        if d < parts - 1 and acc >= total * (d + 1) / parts:
            bounds.append(i + 1)
            d += 1
    while len(bounds) < parts + 1:
        bounds.append(len(lane_counts))
    return bounds


def rank_groups(groups, rank, world):
    """This rank's share of ``groups`` (list of (fold, alpha, beta, penalties)), split at
    LANE granularity: the lanes (one penalty of one group) in group-major order are cut into
    ``world`` contiguous runs of equal length, and each run is regrouped by (fold, alpha).
    125 lanes of a 5x5x5 grid over 8 GPUs give every rank 15-16 lanes instead of 3-4
    whole groups.  Concatenating the ranks' lanes in rank order gives the original order."""
    lanes = [(g[0], g[1], g[2], c, gi) for gi, g in enumerate(groups) for c in g[3]]
    n = len(lanes)
    lo, hi = (n * rank) // world, (n * (rank + 1)) // world
    out = []
    for fold, alpha, beta, c, gi in lanes[lo:hi]:
        if out and out[-1][4] == gi:
            out[-1][3].append(c)
        else:
            out.append([fold, alpha, beta, [c], gi])
    return [(f, a, b, pens) for f, a, b, pens, _ in out]


def fold_order(nf):
    """Order of the folds inside each alpha when a CV grid is laid out as groups: fold 0
    last.  The fold split is drawn fold by fold and fold 0 is ready first (CV driver,
    CV_tools.fold_stream), so a rank can start once its lowest fold is drawn; with fold 0
    at the end of every alpha's run, the contiguous lane runs of rank_groups more often
    hold a fold-0 group (8 ranks over a 5x5x5 grid: every 16-lane share does).  The
    order of the groups does not change any result (lanes map back by (alpha, fold))."""
    return list(range(1, nf)) + [0] if nf > 1 else [0]


def sharded_run_groups(run_groups, rank, world, all_gather, devices=None):
    """Wrap a ``run_groups(gen_pat, M, U, groups, devices, max_block)`` callable so that
    each rank runs only its chunk and every rank returns the full lane arrays.

    ``all_gather(obj) -> list`` collects one picklable object per rank, in rank order
    (e.g. ``torch.distributed.all_gather_object``).
    """
    fixed = devices

    def prepare(gen_pat, groups, devices=None, max_block=0):
        inner = getattr(run_groups, "prepare", None)
        mine = rank_groups(groups, rank, world)
        if inner is not None and mine:
            inner(gen_pat, mine, devices=fixed if fixed is not None else devices, max_block=max_block)

    def run(gen_pat, M, U, groups, devices=None, max_block=0):
        mine = rank_groups(groups, rank, world)
        if mine:
            rt, re, nl = run_groups(gen_pat, M, U, mine, devices=fixed if fixed is not None else devices,
                                    max_block=max_block)
        else:
            rt, re, nl = np.zeros(0, np.float32), np.zeros(0, np.float32), np.zeros(0, np.uint64)
        parts = all_gather((np.asarray(rt), np.asarray(re), np.asarray(nl)))
        return tuple(np.concatenate([p[i] for p in parts]) for i in range(3))
    run.prepare = prepare
    run.fold_feed = getattr(run_groups, "fold_feed", False)
    return run


def torch_all_gather():
    """all_gather over the default torch.distributed process group (host objects)."""
    import torch.distributed as dist

    def gather(obj):
        out = [None] * dist.get_world_size()
        dist.all_gather_object(out, obj)
        return out
    return gather

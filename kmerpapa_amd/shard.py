"""Sharding of the cross-validation grid over ranks (one process per GPU).

The (alpha, fold) groups of a CV sweep are independent DP passes: each
rank runs a lane-balanced share of the group list on its own GPU (assign_lanes) and the
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


# lanes one sweep workgroup holds at 9-mer size with 32-bit counts
# (kp_plan_info.lanes_per_workgroup); callers pass the lattice's own width at its count
# width (engine.shard_width: 4 with 64-bit counts, fewer for lattices with larger blocks)
WG_LANES = 5


def assign_lanes(groups, world, width=WG_LANES):
    """Every rank's lanes, as lists of group-major lane numbers of ``groups`` (list of
    (fold, alpha, beta, penalties); a lane = one penalty of one group).

    Groups that each fit one sweep workgroup (every group the same size, <= ``width``
    lanes: the 5x5x5 headline grid) are dealt WHOLE: a group split over ranks costs every
    rank that gets a piece a device group's fixed work (9-mer: a 1-lane pass 109 ms against
    74 ms per lane inside a 5-lane group).  G groups over N ranks: G // N whole groups per
    rank, in fold order round-robin (so the fold-0 groups, drawn first, go to the first
    ranks), and the G % N leftover groups -- those of the highest folds, drawn last -- cut
    into single lanes dealt to ranks 0, 1, ... (the ranks holding fold-0 groups): every
    16-lane share of the 5x5x5 grid over 8 ranks is then 3 whole groups + 1 lane of a fold
    drawn last, which packs beside one of them in one pass ([5, 5, 5 + 1]) and starts when
    fold 0 is drawn.  Other grids (groups wider than a workgroup, or of mixed sizes) are cut
    into ``world`` contiguous, equal runs of lanes in group-major order, so that the fold
    pieces of a rank's share stay full (the 7x7x10 11-mer grid)."""
    counts = [len(g[3]) for g in groups]
    start = np.cumsum([0] + counts)
    n = int(start[-1])
    world = max(1, int(world))
    uniform = bool(counts) and len(set(counts)) == 1 and counts[0] <= width and len(groups) >= world
    if world == 1 or not uniform:
        return [list(range((n * r) // world, (n * (r + 1)) // world)) for r in range(world)]
    G = len(groups)
    q, r = divmod(G, world)
    by_fold = sorted(range(G), key=lambda i: (groups[i][0], i))  # fold ascending (fold 0 is drawn first)
    left = set(by_fold[G - r:])                                  # the highest folds: drawn last
    per = [[] for _ in range(world)]
    for k, gi in enumerate([i for i in by_fold if i not in left]):
        per[k % world].extend(range(start[gi], start[gi + 1]))
    for k, lid in enumerate([lid for gi in sorted(left) for lid in range(start[gi], start[gi + 1])]):
        per[k % world].append(lid)
    return [[int(x) for x in p] for p in per]


def _regroup(groups, lane_ids):
    gof = np.repeat(np.arange(len(groups)), [len(g[3]) for g in groups])
    start = np.cumsum([0] + [len(g[3]) for g in groups])
    out = []
    for lid in lane_ids:
        gi = int(gof[lid])
        c = groups[gi][3][lid - start[gi]]
        if out and out[-1][4] == gi:
            out[-1][3].append(c)
        else:
            f, a, b = groups[gi][:3]
            out.append([f, a, b, [c], gi])
    return [(f, a, b, pens) for f, a, b, pens, _ in out]


def rank_groups(groups, rank, world, width=WG_LANES):
    """This rank's share of ``groups`` (assign_lanes), regrouped by (fold, alpha): a list of
    (fold, alpha, beta, penalties) whose group-major lanes are ``rank_lane_ids``."""
    return _regroup(groups, assign_lanes(groups, world, width)[rank])


def rank_lane_ids(groups, rank, world, width=WG_LANES):
    """Group-major lane numbers (in ``groups``) of the lanes of ``rank_groups``, in its
    group-major order: results of the ranks concatenated in rank order go back to the
    original lane order by ``out[concatenated ids] = concatenated results``."""
    return assign_lanes(groups, world, width)[rank]


def unshard(groups, world, parts, width=WG_LANES):
    """The ranks' result arrays (``parts``, rank order, each in its rank_groups order) as
    one array in the original group-major lane order."""
    ids = np.concatenate([np.asarray(p, np.int64) for p in assign_lanes(groups, world, width)] or
                         [np.zeros(0, np.int64)])
    cat = np.concatenate(parts) if parts else np.zeros(0)
    out = np.empty_like(cat)
    out[ids] = cat
    return out


def fold_order(nf):
    """Order of the folds inside each alpha when a CV grid is laid out as groups: fold 0
    last.  The fold split is drawn fold by fold and fold 0 is ready first (CV driver,
    CV_tools.fold_stream), so a rank can start once its lowest fold is drawn; with fold 0
    at the end of every alpha's run, the contiguous lane runs of rank_groups more often
    hold a fold-0 group (8 ranks over a 5x5x5 grid: every 16-lane share does).  The
    order of the groups does not change any result (lanes map back by (alpha, fold))."""
    return list(range(1, nf)) + [0] if nf > 1 else [0]


def sharded_run_groups(run_groups, rank, world, all_gather, devices=None, width=None):
    """Wrap a ``run_groups(gen_pat, M, U, groups, devices, max_block)`` callable so that
    each rank runs only its chunk and every rank returns the full lane arrays.

    ``all_gather(obj) -> list`` collects one picklable object per rank, in rank order
    (e.g. ``torch.distributed.all_gather_object``).  ``width`` = the group size dealt whole
    (assign_lanes); None = the lattice's sweep-workgroup width at the counts' width
    (engine.shard_width, the same on every rank).
    """
    fixed = devices

    def _width(gen_pat, itype, max_block):
        if width is not None:
            return width
        from . import engine
        return engine.shard_width(gen_pat, itype, max_block)

    def prepare(gen_pat, groups, devices=None, max_block=0, itype=np.uint32):
        inner = getattr(run_groups, "prepare", None)
        mine = rank_groups(groups, rank, world, _width(gen_pat, itype, max_block))
        if inner is not None and mine:
            inner(gen_pat, mine, devices=fixed if fixed is not None else devices, max_block=max_block, itype=itype)

    def run(gen_pat, M, U, groups, devices=None, max_block=0):
        from . import engine
        w = _width(gen_pat, engine.counts_itype(M), max_block)
        mine = rank_groups(groups, rank, world, w)
        if mine:
            rt, re, nl = run_groups(gen_pat, M, U, mine, devices=fixed if fixed is not None else devices,
                                    max_block=max_block)
        else:
            rt, re, nl = np.zeros(0, np.float32), np.zeros(0, np.float32), np.zeros(0, np.uint64)
        parts = all_gather((np.asarray(rt), np.asarray(re), np.asarray(nl)))
        return tuple(unshard(groups, world, [p[i] for p in parts], w) for i in range(3))
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

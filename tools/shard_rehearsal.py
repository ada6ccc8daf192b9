"""Rehearsal of the multi-GPU CV driver under torchrun (tool): every rank runs the drop-in
CV driver on the reference's 7-mer test data, 3x3 grid, 5 folds (config 3); the driver
shards the (alpha, fold, penalty) lanes over the ranks and all-gathers the root scalars
(gloo).  Rank 0 checks the CVfile text and best point against the reference's own
(tests/golden/cv7.json) and prints one JSON line.  With more ranks than GPUs the ranks
share them (a rehearsal of the code path, not of scaling).
usage: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
           --master-port 29511 tools/shard_rehearsal.py"""
import io
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch.distributed as dist  # noqa: E402

from kmerpapa_amd.algorithms import bottum_up_array_penalty_plus_pseudo_CV as cvm  # noqa: E402
from tests.fixtures import context_table, golden_json  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    ctx, gp, nm, nu = context_table(7)
    g = golden_json("cv7.json")
    buf = io.StringIO()

    class A:
        nfolds = 5
        iterations = 1
        seed = 1
        verbosity = 0
        CVfile = buf
    t0 = time.time()
    best = cvm.pattern_partition_bottom_up(gp, ctx, g["alphas"], A, nm, nu, g["penalties"])
    wall = time.time() - t0
    ok = buf.getvalue() == g["cvfile"] and [best[0], best[1], best[2]] == g["best"]
    oks = [None] * world
    dist.all_gather_object(oks, ok)
    if rank == 0:
        print(json.dumps({"ranks": world, "gen_pat": gp, "cv_wall_s": round(wall, 3), "all_ranks_match_reference": all(oks),
                          "best": list(best)}), flush=True)
    dist.destroy_process_group()
    sys.exit(0 if all(oks) else 1)


if __name__ == "__main__":
    main()

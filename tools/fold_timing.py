"""Host time of the CV fold split on the 9-mer counts (tool): fold 0's draw (what every
pass of a CV job waits for) and the whole 5-fold split, best of REPS, in this process.
Run twice, with and without KP_FOLDS_SCALAR=1, to compare kp_folds.h's two paths."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from kmerpapa_amd import engine  # noqa: E402
from kmerpapa_amd.CV_tools import _colors  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
kmers, M, U = bench.synthetic_counts("NNNNMNNNN", seed=9)
_, colors = _colors(bench.kmer_table(kmers, M, U), np.uint32)
col = colors.astype(np.uint64)
n = int(col.sum())
f0, full = [], []
for _ in range(reps):
    t = time.perf_counter()
    engine.fold_sample(col, n // 5, np.random.RandomState(1))
    f0.append(time.perf_counter() - t)
    t = time.perf_counter()
    engine.fold_split(col, 5, np.random.RandomState(1))
    full.append(time.perf_counter() - t)
print(json.dumps({"scalar": bool(os.environ.get("KP_FOLDS_SCALAR")), "colours": int(col.size),
                  "fold0_ms": round(min(f0) * 1e3, 2), "fold0_ms_median": round(sorted(f0)[len(f0) // 2] * 1e3, 2),
                  "split_ms": round(min(full) * 1e3, 2)}))

"""Time the CLI's output writer (cli.write_partition, cli.py:301-316) at 9-mer scale on the
host (tool): the synthetic 9-mer table (bench.synthetic_counts) and partitions of 512 and
8,192 patterns covering all 131,072 k-mers, short and long (-l) output.  Prints one JSON line
per case with the seconds and the output's md5 (to compare writers)."""
import hashlib
import io
import itertools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from kmerpapa_amd.cli import write_partition  # noqa: E402

kmers, M, U = bench.synthetic_counts("NNNNMNNNN")
table = bench.kmer_table(kmers, M, U)
nm, nu = int(M.sum()), int(U.sum())
my = nm / (nm + nu)
alpha = 2.0
beta = (alpha * (1.0 - my)) / my
parts = {
    512: ["".join(a) + "NNNNM"[4:] + "NNN" + b for a in itertools.product("ACGT", repeat=4) for b in "RY"],
    4096: ["".join(a) + "M" + "".join(c) + "NN" for a in itertools.product("ACGT", repeat=4)
           for c in itertools.product("ACGT", repeat=2)] ,
}
for n, names in parts.items():
    names = [x if len(x) == 9 else x for x in names]
    counts = table.pattern_counts(names)
    assert sum(c[0] for c in counts) == nm and sum(c[1] for c in counts) == nu
    for long_output in (False, True):
        buf = io.StringIO()
        t0 = time.perf_counter()
        write_partition(buf, names, counts, table, alpha, beta, long_output)
        dt = time.perf_counter() - t0
        text = buf.getvalue()
        print(json.dumps({"patterns": len(names), "long": long_output, "rows": text.count("\n") - 1,
                          "seconds": round(dt, 4), "md5": hashlib.md5(text.encode()).hexdigest()}), flush=True)

"""End-to-end CLI run at 11-mer input scale (BASELINE configs[4], super-pattern form):
synthetic counts for every 11-mer of NNNNNMNNNNN (2,097,152 lines per file, the bench's
generator), then `python -m kmerpapa_amd -s ANNNNMNNNNA` with the 7x7 grid and 10 folds,
exactly as a user would run it (native parse + super-pattern filter, CV on the
7.69e9-cell lattice, final fit, output).  Prints one JSON line."""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else tempfile.mkdtemp(prefix="kp_cli_")  # large inputs: not under gpurun_out
os.makedirs(out, exist_ok=True)
t0 = time.time()
kmers, M, U = bench.synthetic_counts("NNNNNMNNNNN")
with open(os.path.join(out, "pos.txt"), "w") as f:
    f.writelines(f"{k} {m}\n" for k, m in zip(kmers, M.tolist()))
with open(os.path.join(out, "bg.txt"), "w") as f:
    f.writelines(f"{k} {b}\n" for k, b in zip(kmers, (M + U).tolist()))
gen_s = time.time() - t0
import types  # noqa: E402
from kmerpapa_amd import io_utils  # noqa: E402
from kmerpapa_amd.papa import Pattern  # noqa: E402
cfg = bench.CONFIGS["11mer"]
t0 = time.time()
table, _, _ = io_utils.read_input_table(types.SimpleNamespace(
    positive=open(os.path.join(out, "pos.txt")), background=open(os.path.join(out, "bg.txt")), negative=None,
    joint_context_counts=None), Pattern(cfg["gen_pat"]))
parse_s = time.time() - t0
cmd = [sys.executable, "-m", "kmerpapa_amd", "-p", os.path.join(out, "pos.txt"), "-b", os.path.join(out, "bg.txt"),
       "-s", cfg["gen_pat"], "-c"] + [str(c) for c in cfg["penalties"]] + ["-a"] + [str(a) for a in cfg["alphas"]] + \
      ["--nfolds", str(cfg["nfolds"]), "--seed", "1", "-o", os.path.join(out, "partition.txt"),
       "-f", os.path.join(out, "cv.txt")]
t0 = time.time()
r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True)
wall = time.time() - t0
lines = open(os.path.join(out, "partition.txt")).read().splitlines() if r.returncode == 0 else []
print(json.dumps({"cmd": " ".join(cmd[1:]), "rc": r.returncode, "wall_s": wall, "input_lines_per_file": len(kmers),
                  "input_write_s": gen_s, "native_parse_s": parse_s, "kmers_kept": len(table), "patterns": max(0, len(lines) - 1), "stderr_tail": r.stderr[-1200:]}))

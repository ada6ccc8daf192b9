"""End-to-end CLI run on the benchmark's synthetic 9-mer counts (BASELINE configs[3]):
writes positive/background count files, then times `python -m kmerpapa_amd` exactly as a
user would run it (grid CV + final fit + output table).  Prints one JSON line.
usage: cli_9mer.py [OUTDIR [CLI ARGS...]]: CLI ARGS replace the default grid CV arguments
(e.g. "-c 5 -a 2 -l": one fit with the long output)."""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else tempfile.mkdtemp(prefix="kp_cli_")  # large inputs: not under gpurun_out
os.makedirs(out, exist_ok=True)
kmers, M, U = bench.synthetic_counts("NNNNMNNNN")
with open(os.path.join(out, "pos.txt"), "w") as f:
    f.writelines(f"{k} {m}\n" for k, m in zip(kmers, M))
with open(os.path.join(out, "bg.txt"), "w") as f:
    f.writelines(f"{k} {m + u}\n" for k, m, u in zip(kmers, M, U))
grid = sys.argv[2:] or ["-c", "3", "4", "5", "6", "7", "-a", "0.5", "1", "2", "5", "10", "--nfolds", "5", "--seed", "1",
                        "-f", os.path.join(out, "cv.txt")]
cmd = [sys.executable, "-m", "kmerpapa_amd", "-p", os.path.join(out, "pos.txt"), "-b", os.path.join(out, "bg.txt"),
       "-o", os.path.join(out, "partition.txt")] + grid
metrics = os.path.join(out, "metrics.jsonl")
if os.path.exists(metrics):
    os.remove(metrics)
t0 = time.time()
r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, env=dict(os.environ, KMERPAPA_METRICS=metrics))
wall = time.time() - t0
phases = json.loads(open(metrics).read().splitlines()[-1]) if os.path.exists(metrics) else None
lines = open(os.path.join(out, "partition.txt")).read().splitlines() if r.returncode == 0 else []
print(json.dumps({"cmd": " ".join(cmd[1:]), "rc": r.returncode, "wall_s": wall, "patterns": max(0, len(lines) - 1),
                  "in_process": phases, "stderr_tail": r.stderr[-600:]}))

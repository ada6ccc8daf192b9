"""Scratch: time 9-mer passes under env variants (KP_DEBUG_SKIP ablates phases -> wrong
results, timing only; KP_LANES_PER_WG changes lanes per workgroup)."""
import json, os, subprocess, sys
variants = [v.split(",") for v in sys.argv[1:]] or [["KP_DEBUG_SKIP=0"]]
for var in variants:
    env = dict(os.environ)
    for kv in var:
        k, v = kv.split("=")
        env[k] = v
    out = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"],
                         env=env, capture_output=True, text=True)
    try:
        d = json.loads(out.stdout.strip().splitlines()[-1])
        print(var, "dp_ms %.1f bt_ms %.1f step_ms %.1f" % (d["dp_kernel_ms_per_step"], d["backtrack_ms_per_step"],
                                                           d["ms_per_step"]), flush=True)
    except Exception:
        print(var, "failed", out.stderr[-800:], flush=True)

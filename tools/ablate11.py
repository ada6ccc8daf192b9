import json, os, subprocess, sys
for var in [v.split(",") for v in sys.argv[1:]]:
    env = dict(os.environ)
    for kv in var:
        k, v = kv.split("="); env[k] = v
    out = subprocess.run([sys.executable, "bench.py", "--config", "11mer", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-full-cv"], env=env, capture_output=True, text=True)
    try:
        d = json.loads(out.stdout.strip().splitlines()[-1]); print(var, "dp_ms %.1f" % d["dp_kernel_ms_per_step"], flush=True)
    except Exception:
        print(var, "failed", out.stderr[-500:], flush=True)

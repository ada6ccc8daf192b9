"""Plan construction time (tool; one GPU): engine.Plan for the 9-mer lattice, three times
(host tables, uploads, the pair-delta table)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kmerpapa_amd import engine  # noqa: E402

dev = engine.get_device(0)
for _ in range(4):
    t0 = time.perf_counter()
    p = engine.Plan(dev, "NNNNMNNNN", 0)
    t1 = time.perf_counter()
    p.close()
    print(f"Plan(): {1e3 * (t1 - t0):.2f} ms", flush=True)

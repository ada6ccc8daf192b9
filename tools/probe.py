"""Scratch timing probe (not part of the product): one CV pass on a fixture lattice."""
import sys, time
sys.path.insert(0, '.')
import numpy as np
from kmerpapa_amd import engine
from kmerpapa_amd.CV_tools import fold_tables
from kmerpapa_amd.pattern_utils import generality
from tests.fixtures import context_table

k = int(sys.argv[1]) if len(sys.argv) > 1 else 7
lanes_per_group = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ctx, gp, nm, nu = context_table(k)
t0 = time.time()
contexts, Mf, Uf = fold_tables(ctx, 5, np.random.RandomState(1), np.uint32)
t1 = time.time()
Mk, Uk = engine.counts_in_kmer_order(gp, contexts, Mf, Uf, generality(gp), np.uint32)
dev = engine.get_device(0)
plan = engine.Plan(dev, gp)
t2 = time.time()
plan.set_counts(Mk, Uk)
t3 = time.time()
print("plan", plan.info, "sample %.2fs plan %.2fs counts %.3fs" % (t1 - t0, t2 - t1, t3 - t2), flush=True)
pens = [3.0, 5.0, 7.0][:lanes_per_group]
groups = [(f, a, 1000.0, pens) for a in (0.5, 1.0, 10.0) for f in range(5)]
for rep in range(3):
    rt, re, nl = plan.run(groups)
    s = plan.stats()
    units = s["units"]
    print("rep", rep, "dp_ms %.2f bt_ms %.2f total_ms %.2f units %d -> %.3e units/s, alg %.2f TB/s, gather-model %.2f TB/s"
          % (s["dp_ms"], s["backtrack_ms"], s["total_ms"], units, units / (s["dp_ms"] / 1e3),
             s["alg_bytes"] / (s["dp_ms"] / 1e3) / 1e12, s["gather_bytes"] / (s["dp_ms"] / 1e3) / 1e12), flush=True)
print("leaves", nl[:6])

"""Model (tool, CPU only): how often a cheap lower bound on the single-pattern term proves it
cannot win, so that a cell could skip its two float64 logs -- per cell, and per wave of 64
cells as the sweep runs them (a wave pays for the logs if any of its lanes needs them).

Bound (no float64 log): s = c + (-2M) ln p + (-2U) ln(1-p) >= c + 2M (-ln2 log2f(p_up) - err)
+ 2U (p + p^2/2), with p_up = float32(p) rounded up and err bounding the hardware log2's
error; the cell's logs are skippable when that bound >= the best split.  A copy of
oracle/kp_oracle.c's kpo_cv_lane is patched (in /tmp, never the repo's oracle) to flag such
cells; waves are the 64-cell runs of each block's low levels in ascending index order.
usage: python tools/logskip_model.py [GEN_PAT SUB]   (default NNNNMNNNN ANNNMNNNA)"""
import ctypes
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

src = open(os.path.join(ROOT, "oracle", "kp_oracle.c")).read()
hook = "                    double s = penalty;                                                                \\\n"
assert hook in src
patch = ("                    { float pu = (float)p; if ((double)pu < p) pu = nextafterf(pu, 2.0f);              \\\n"
         "                      double l2 = (double)log2f(pu); l2 = l2 + fabs(l2) * 4.8e-7;                      \\\n"
         "                      double t1 = -0.6931471805599453 * l2; if (t1 < 0) t1 = 0;                       \\\n"
         "                      double slo = penalty + 2.0 * (double)trm * t1 * (1 - 1e-9)                      \\\n"
         "                                 + 2.0 * (double)tru * (p + 0.5 * p * p) * (1 - 1e-9);                \\\n"
         "                      if (g_flags && slo >= (double)rs) g_flags[n] = 1; }                             \\\n")
src = src.replace(hook, patch + hook, 1)
src = src.replace("#define KPO_LANE_BODY(CT)", "unsigned char *g_flags = 0;\nvoid kpo_set_flags(unsigned char *f) "
                  "{ g_flags = f; }\n#define KPO_LANE_BODY(CT)", 1)
tmp = tempfile.mkdtemp()
with open(os.path.join(tmp, "lb.c"), "w") as fh:
    fh.write(src)
lib_path = os.path.join(tmp, "liblb.so")
subprocess.run(["gcc", "-O2", "-fPIC", "-std=c11", "-ffp-contract=off", "-fno-fast-math", "-fopenmp", "-shared",
                "-o", lib_path, os.path.join(tmp, "lb.c"), "-lm"], check=True)

import oracle.oracle as OO  # noqa: E402
OO._LIB_PATH, OO._lib = lib_path, None
from oracle import oracle as O  # noqa: E402
from oracle import treecheck as T  # noqa: E402
import bench  # noqa: E402

gp, sub = (sys.argv[1], sys.argv[2]) if len(sys.argv) > 2 else ("NNNNMNNNN", "ANNNMNNNA")
lib = O.lib()
kmers, M, U = bench.synthetic_counts(gp, seed=9)
keep = np.array([all(k[j] in T.IUPAC[ch] for j, ch in enumerate(sub)) for k in kmers])
kc = np.array([O.cell_index(sub, k) for k, x in zip(kmers, keep) if x], np.uint64)
my = M.sum() / (M.sum() + U.sum())
lat = T.Lattice(sub)
npat = O.npat(sub)
B = lat.radix[0] * lat.radix[1] * lat.radix[2]
x = np.arange(npat, dtype=np.int64)
lev = np.zeros(npat, np.int8)
lolev = np.zeros(B, np.int8)
for i, g in enumerate(sub):
    lv = np.array([len(T.IUPAC[c]) - 1 for c in O._PERM[g]])
    lev += lv[(x // lat.cw[i]) % lat.radix[i]].astype(np.int8)
    if i < 3:
        lolev += lv[(np.arange(B) // lat.cw[i]) % lat.radix[i]].astype(np.int8)
lo, h = x % B, x // B
order = np.lexsort((lo, lolev[lo], h))
key = (h * 16 + lolev[lo])[order]
starts = np.r_[0, np.nonzero(np.diff(key))[0] + 1]
rank = np.arange(key.size) - np.repeat(starts, np.diff(np.r_[starts, key.size]))
wave = key * 1000 + rank // 64
valid = lev[order] > 0
for a, c in [(0.5, 3.0), (2.0, 5.0), (10.0, 7.0)]:
    f = np.zeros(npat, np.uint8)
    lib.kpo_set_flags(f.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)))
    O.cv_lane(sub, kc, M[keep], U[keep], a, a * (1 - my) / my, c, 32, threads=os.cpu_count() or 1)
    lib.kpo_set_flags(None)
    fv = f[order][valid]
    _, inv = np.unique(wave[valid], return_inverse=True)
    allskip = np.bincount(inv, weights=1 - fv) == 0
    print(f"{sub} alpha {a} c {c}: cells whose logs are skippable {fv.mean():.3f}, "
          f"cells in waves where every lane is {allskip[inv].mean():.3f}", flush=True)

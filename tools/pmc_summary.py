"""Sum rocprofv3 PMC counter_collection.csv files per kernel (one dir per pass)."""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
tot = defaultdict(float)
dur = defaultdict(float)
for fn in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
    seen = set()
    for r in csv.DictReader(open(fn)):
        k = r["Kernel_Name"].split("(")[0][:40]
        tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        key = (fn, r["Dispatch_Id"])
        if key not in seen and "sq1" in fn:
            seen.add(key)
            dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for (k, c), v in sorted(tot.items()):
    if "dp_kernel" in k or len(sys.argv) > 2:
        print(f"{k:42s} {c:24s} {v:.4e}")
for k, v in dur.items():
    if "dp_kernel" in k:
        print(k, "ms (sq1 pass)", round(v, 1))

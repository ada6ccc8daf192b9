"""Sum the SQ counters of tools/pmc_phases.sh per KP_DEBUG_SKIP value (tool): kp_dp_kernel
dispatches of the run, divided by the 3 passes tools/ablate.py times, per 9-mer cell-lane."""
import csv
import glob
import os
import sys

d = sys.argv[1]
cells_lanes = 7688671875 * int(os.environ.get("ABLATE_LANES", "5"))
print("skip  " + "  ".join(f"{c:>22}" for c in ("SQ_INSTS_VALU/unit", "SQ_INSTS_LDS/unit", "SQ_ACTIVE_INST_VALU",
                                                   "LDS_BANK_CONFLICT", "LDS_IDX_ACTIVE")))
for sub in sorted(glob.glob(os.path.join(d, "s*"))):
    if not os.path.isdir(sub):
        continue
    tot = {}
    for fn in glob.glob(os.path.join(sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            if "kp_dp_kernel" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    per = {k: v / 3 for k, v in tot.items()}  # 3 passes per skip value
    skip = os.path.basename(sub)[1:]
    print(f"{skip:>4}  " + "  ".join(f"{x:>22.4g}" for x in (
        per.get("SQ_INSTS_VALU", 0) * 64 / cells_lanes, per.get("SQ_INSTS_LDS", 0) * 64 / cells_lanes,
        per.get("SQ_ACTIVE_INST_VALU", 0), per.get("SQ_LDS_BANK_CONFLICT", 0), per.get("SQ_LDS_IDX_ACTIVE", 0))))

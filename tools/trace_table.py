"""Per-launch table from tools/trace_ablate.sh output: full vs levels-only vs gather-only."""
import csv
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"


def durs(v):
    rows = [r for r in csv.DictReader(open(f"{root}/tr{v}/run_kernel_trace.csv")) if "kp_dp_kernel" in r["Kernel_Name"]]
    return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows][-17:]


a, l, g = durs(0), durs(1), durs(2)
for H in range(len(a)):
    print("%2d full %6.1f  levels-only %6.1f  gather-only %6.1f  loss %5.1f" % (H, a[H], l[H], g[H], a[H] - max(l[H], g[H])))
print("sum full %.1f  sum max(l,g) %.1f  sum l %.1f  sum g %.1f" % (sum(a), sum(max(x, y) for x, y in zip(l, g)), sum(l), sum(g)))

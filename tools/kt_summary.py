"""Top kernels of a rocprofv3 --kernel-trace --stats run: usage kt_summary.py <dir> [n]."""
import csv
import glob
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
f = sorted(glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True))
if not f:
    sys.exit(f"no kernel_stats.csv under {d}")
rows = list(csv.DictReader(open(f[0])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print(f"{'total ms':>10} {'calls':>6} {'avg us':>10} {'min us':>10} {'max us':>10}  kernel")
for r in rows[:n]:
    print(f'{float(r["TotalDurationNs"]) / 1e6:10.3f} {int(r["Calls"]):6d} {float(r["AverageNs"]) / 1e3:10.1f} '
          f'{float(r["MinNs"]) / 1e3:10.1f} {float(r["MaxNs"]) / 1e3:10.1f}  {r["Name"][:150]}')

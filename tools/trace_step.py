"""Print the kernel timeline of the last step of a rocprofv3 --kernel-trace run (dev tool).

usage: python tools/trace_step.py <trace dir>   (a step starts at each k_fingerprint, or k_bbox, dispatch)"""
import csv, glob, sys

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# a step starts at its first kernel: k_fingerprint for a slab-culled call (the cull map's key), else k_bbox
mark = "k_fingerprint(" if any("k_fingerprint(" in r["Kernel_Name"] for r in rows) else "k_bbox("
starts = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
step = rows[starts[-2]:starts[-1]] if len(starts) > 1 else rows
t0 = int(step[0]["Start_Timestamp"])
for r in step:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    g = r.get("Grid_Size", r.get("Grid_Size_X", ""))
    print(f"{s / 1e6:8.3f} {e / 1e6:8.3f} {(e - s) / 1e6:7.3f} ms  q{r.get('Queue_Id', '?'):>3s} grid {g:>10s}  {r['Kernel_Name'][:70]}")

"""Summarise rocprofv3 counter_collection / kernel_stats CSVs per kernel (dev tool)."""
import csv, collections, glob, sys
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for f in sorted(glob.glob(f"{root}/**/*kernel_stats.csv", recursive=True)):
    print(f)
    for r in csv.DictReader(open(f)):
        print(f"  {r['Name'][:60]:60s} calls {r['Calls']:>4s} avg_ms {float(r['AverageNs'])/1e6:9.3f} tot% {float(r['Percentage']):6.2f}")
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    print(f)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        key = "knn" if "knn_interp" in name else name[:40]
        g = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)))
        if key == "knn":
            key = f"knn(grid={g})"
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[key].add(r["Dispatch_Id"])
    for key, d in agg.items():
        if "knn" not in key:
            continue
        n = len(cnt[key])
        print(f"  {key}  dispatches={n}")
        for c, v in sorted(d.items()):
            print(f"     {c:28s} {v / n:.4g}")

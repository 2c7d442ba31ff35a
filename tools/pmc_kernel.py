"""Per-dispatch averages of rocprofv3 counter CSVs for the kernels whose name contains a
substring, plus derived shares (dev tool).  usage: pmc_kernel.py DIR SUBSTR"""
import collections, csv, glob, sys

root, sub = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sub not in r["Kernel_Name"]:
            continue
        key = r["Kernel_Name"][:60]
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(key, r["Counter_Name"])].add((f, r["Dispatch_Id"]))
for key, d in agg.items():
    print(key)
    avg = {c: v / max(1, len(disp[(key, c)])) for c, v in d.items()}
    for c in sorted(avg):
        print(f"   {c:26s} {avg[c]:.4g}")
    w = avg.get("SQ_WAVES", 0)
    if w:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_LDS_BANK_CONFLICT"):
            if c in avg:
                print(f"   per wave {c:22s} {avg[c] / w:.1f}")
    wc = avg.get("SQ_WAVE_CYCLES", 0)
    if wc:
        for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                  "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA"):
            if c in avg:
                print(f"   share of wave cycles {c:20s} {avg[c] / wc:.3f}")

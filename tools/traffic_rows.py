"""HBM bytes per launch of the §8(f) row kernels from separate rocprofv3 --pmc passes.

usage: python3 tools/traffic_rows.py <pmc root> <round>
  <pmc root>/<row>_fetch and <row>_write for row in filter, mask, div (tools/gpu_pmc_rows.sh)
Writes profiles/traffic_rows_<round>.json: {kernel name prefix: {read_bytes, write_bytes,
hbm_bytes, dispatches}} averaged over dispatches; read = 2 x FETCH_SIZE x 1 KiB (gfx950
half-count of coalesced streams, MI355X_MICROARCH.md), write = WRITE_SIZE x 1 KiB.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"filter": ["k_knn_interp", "k_slot_speed"], "mask": ["k_mask_sample_sep", "k_boundary_count16",
                                                                   "k_boundary_emit16"],
           "div": ["k_divergence"]}


def per_kernel(d, name):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                acc[r["Kernel_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return acc


def main(root, rnd):
    out = {"round": rnd, "units": "bytes per launch (average over dispatches)",
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes; read = 2*FETCH_SIZE*1024, "
                     "write = WRITE_SIZE*1024"}
    for row, names in KERNELS.items():
        fe = per_kernel(os.path.join(root, f"{row}_fetch"), "FETCH_SIZE")
        wr = per_kernel(os.path.join(root, f"{row}_write"), "WRITE_SIZE")
        for nm in names:
            fk = [v for k, d in fe.items() if nm in k for v in d.values()]
            wk = [v for k, d in wr.items() if nm in k for v in d.values()]
            if nm == "k_knn_interp":  # the filter's slot-mode launch: the largest-fetch dispatches
                fk = sorted(fk)[len(fk) // 2:]
                wk = sorted(wk)[len(wk) // 2:]
            if not fk or not wk:
                continue
            rd = 2 * 1024 * sum(fk) / len(fk)
            wb = 1024 * sum(wk) / len(wk)
            out[f"{row}:{nm}"] = {"read_bytes": rd, "write_bytes": wb, "hbm_bytes": rd + wb, "dispatches": len(fk)}
    path = os.path.join(ROOT, "profiles", f"traffic_rows_{rnd}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])

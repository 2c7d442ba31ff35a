"""Summarise a tools/collect_profiles.sh run into profiles/ (committed evidence).

Writes
  profiles/<round>_kernel_stats.csv   rocprofv3 --stats per-kernel summary (copied)
  profiles/<round>_summary.txt        readable per-kernel average durations
  profiles/traffic_<round>.json       HBM bytes per k-NN launch from the PMC passes

HBM bytes follow MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE and WRITE_SIZE are
KiB per dispatch, collected in separate passes; on gfx950 FETCH_SIZE reports half
the bytes of a coalesced stream, so read bytes = 2 x FETCH_SIZE x 1024.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(d, name):
    per = collections.defaultdict(dict)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != name:
                continue
            g = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)))
            key = (r["Kernel_Name"], r["Dispatch_Id"], g)
            per[key][name] = per[key].get(name, 0.0) + float(r["Counter_Value"])
    return per


def main(out, rnd):
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(f"{out}/stats/**/*kernel_stats.csv", recursive=True)
    lines = []
    knn_avg_ms = None
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{rnd}_kernel_stats.csv"))
        for r in csv.DictReader(open(stats[0])):
            avg = float(r["AverageNs"]) / 1e6
            lines.append(f"{r['Name'][:90]:90s} calls {int(r['Calls']):5d} avg_ms {avg:9.3f} "
                         f"min_ms {float(r['MinNs']) / 1e6:9.3f} max_ms {float(r['MaxNs']) / 1e6:9.3f} "
                         f"pct {float(r['Percentage']):6.2f}")
    # per-dispatch durations of the main k-NN launch (largest grid) from the kernel trace
    trace = glob.glob(f"{out}/stats/**/*kernel_trace.csv", recursive=True)
    if trace:
        durs = collections.defaultdict(list)
        for r in csv.DictReader(open(trace[0])):
            if "k_knn_interp" in r["Kernel_Name"]:
                g = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)))
                durs[g].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        if durs:
            gmax = max(durs)
            knn_avg_ms = sum(durs[gmax]) / len(durs[gmax])
            lines.append(f"main k_knn_interp launch (grid {gmax}): {len(durs[gmax])} dispatches, "
                         f"avg {knn_avg_ms:.3f} ms")
            for g in sorted(durs):
                if g != gmax:
                    lines.append(f"  lattice-level k_knn_interp (grid {g}): avg {sum(durs[g]) / len(durs[g]):.3f} ms")
    fetch = counters(f"{out}/fetch", "FETCH_SIZE")
    write = counters(f"{out}/write", "WRITE_SIZE")

    def main_launch(per, name):
        # the main launch = the k_knn_interp dispatches with the largest grid (the lattice
        # levels run the same template over far fewer waves)
        ks = [(k, v[name]) for k, v in per.items() if "k_knn_interp" in k[0]]
        if not ks:
            return []
        gmax = max(k[2] for k, _ in ks)
        return [v for k, v in ks if k[2] == gmax]

    import hashlib

    lib = os.path.join(ROOT, "ptv_interpolation_amd", "libptv_amd.so")
    sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16] if os.path.exists(lib) else None
    res = {"round": rnd, "kernel": "k_knn_interp<8> (main launch)", "units": "bytes per launch",
           "lib_sha256": sha,  # the library these counters were collected with (bench.py compares)
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                     "read = 2*FETCH_SIZE*1024 (gfx950 half-count of coalesced streams; the "
                     "k-NN gathers are 32-B double4 loads, uncalibrated), write = WRITE_SIZE*1024"}
    f_main = main_launch(fetch, "FETCH_SIZE")
    w_main = main_launch(write, "WRITE_SIZE")
    if f_main and w_main:
        rb = 2 * 1024 * sum(f_main) / len(f_main)
        wb = 1024 * sum(w_main) / len(w_main)
        res.update({"read_bytes_per_launch": rb, "write_bytes_per_launch": wb,
                    "hbm_bytes_per_launch": rb + wb, "dispatches_averaged": len(f_main)})
        lines.append(f"HBM traffic per main launch: read {rb / 1e9:.3f} GB write {wb / 1e9:.3f} GB")
    if knn_avg_ms is not None:
        res["kernel_avg_ms_trace"] = knn_avg_ms
    with open(os.path.join(prof, f"traffic_{rnd}.json"), "w") as f:
        json.dump(res, f, indent=1)
    with open(os.path.join(prof, f"{rnd}_summary.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "r01")

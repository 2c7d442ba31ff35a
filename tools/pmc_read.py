#!/usr/bin/env python3
"""Per-dispatch PMC counter values from rocprofv3 rocpd databases.

    pmc_read.py DB [DB ...] [--kernel SUBSTR] [--min-grid N]
"""
import argparse
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("dbs", nargs="+")
ap.add_argument("--kernel", default=None)
ap.add_argument("--min-grid", type=int, default=0)
a = ap.parse_args()
rows = defaultdict(dict)
for p in a.dbs:
    c = sqlite3.connect(p)
    q = ("select dispatch_id, kernel_name, grid_size, duration, counter_name, sum(value) from counters_collection "
         "group by dispatch_id, kernel_name, counter_name")
    for did, kn, gs, dur, cn, v in c.execute(q):
        if a.kernel and a.kernel not in kn:
            continue
        if gs < a.min_grid:
            continue
        key = (p, did)
        rows[key].update({"kernel": kn[:40], "grid": gs, "ns": dur, cn: v})
for (p, did), r in sorted(rows.items()):
    ctr = {k: v for k, v in r.items() if k not in ("kernel", "grid", "ns")}
    print(f"{r['kernel']:40s} grid={r['grid']:>10d} ns={r['ns']:>10.0f} " +
          " ".join(f"{k}={v:.4g}" for k, v in sorted(ctr.items())))

#!/usr/bin/env python3
"""Print per-kernel PMC counter sums from rocprofv3 rocpd databases: pmc_read.py DB [DB ...] [--kernel SUBSTR]"""
import sqlite3
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
ksub = None
if "--kernel" in sys.argv:
    ksub = sys.argv[sys.argv.index("--kernel") + 1]
    args = [a for a in args if a != ksub]
for p in args:
    c = sqlite3.connect(p)
    q = ("select kernel_name, counter_name, sum(value), count(distinct dispatch_id), avg(duration) "
         "from counters_collection group by kernel_name, counter_name order by kernel_name")
    for kn, cn, v, nd, dur in c.execute(q):
        if ksub and ksub not in kn:
            continue
        print(f"{kn[:48]:48s} {cn:28s} {v:16.4g}  dispatches={nd} avg_ns={dur:.0f}")

"""Per-dispatch averages of rocprofv3 counters from its sqlite output (rocpd *.db, the default
format of rocprofv3 --pmc without --output-format csv), for kernels whose name contains a
substring, plus the derived per-wave / share-of-cycles figures (dev tool).

usage: pmc_db.py SUBSTR DB_OR_DIR [DB_OR_DIR ...]
"""
import collections
import glob
import os
import sqlite3
import sys


def rows(db, sub):
    c = sqlite3.connect(db)
    q = ("select kernel_name, dispatch_id, counter_name, value, grid_size, vgpr_count, accum_vgpr_count, "
         "scratch_size, lds_block_size from counters_collection")
    for r in c.execute(q):
        if sub in r[0]:
            yield r


def main():
    sub = sys.argv[1]
    dbs = []
    for a in sys.argv[2:]:
        dbs += [a] if a.endswith(".db") else glob.glob(os.path.join(a, "**", "*.db"), recursive=True)
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    info = {}
    for db in dbs:
        for name, did, cn, v, grid, vg, ag, scr, lds in rows(db, sub):
            key = (name.split("(")[0][:80], grid)
            tot[key][cn] += v
            disp[key][cn].add((db, did))
            info[key] = (vg, ag, scr, lds)
    for key, d in sorted(tot.items(), key=lambda kv: -kv[0][1]):
        vg, ag, scr, lds = info[key]
        print(f"{key[0]}  grid={key[1]}  vgpr={vg} agpr={ag} scratch={scr} lds={lds}")
        avg = {c: v / max(1, len(disp[key][c])) for c, v in d.items()}
        for c in sorted(avg):
            print(f"   {c:26s} {avg[c]:.4g}   ({len(disp[key][c])} dispatches)")
        w = avg.get("SQ_WAVES", 0)
        if w:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                      "SQ_INSTS_SMEM"):
                if c in avg:
                    print(f"   per wave {c:22s} {avg[c] / w:.1f}")
        wc = avg.get("SQ_WAVE_CYCLES", 0)
        if wc:
            for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_WAIT_INST_ANY",
                      "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA"):
                if c in avg:
                    print(f"   share of wave cycles {c:20s} {avg[c] / wc:.3f}")
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            if c in avg:
                print(f"   {c} per dispatch: {avg[c] * 1024 / 1e9:.3f} GB (counter unit KB)")


if __name__ == "__main__":
    main()

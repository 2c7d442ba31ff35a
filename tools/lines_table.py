"""Markdown table of one round's bench lines (profiles/<tag>_lines/*.json + the kernel-trace
summaries *.kt.txt next to them), for DESIGN.md §5.

usage: python tools/lines_table.py r05
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORDER = [
    ("headline", "512³ / 5M IDW k=8 (BASELINE metric)"),
    ("nearest", "512³ / 5M nearest (k=1)"),
    ("sibson", "512³ / 5M Sibson k=30"),
    ("sibson_k50", "512³ / 5M Sibson k=50"),
    ("idw_k50", "512³ / 5M IDW k=50 (reference default k)"),
    ("c2", "C2 256³ / 1M IDW k=8"),
    ("c2r", "C2 256³ / 1M IDW radius r=3 (extension)"),
    ("c3", "C3 512³ / 5M local Gaussian RBF 32×32"),
    ("rbf_tps20", "512³ / 5M local TPS RBF k=20 (degree 1)"),
    ("rbf_tps32", "512³ / 5M local TPS RBF k=32 (degree 1)"),
    ("c4", "C4 1024³ / 10M masked IDW (whole grid, 1 GPU)"),
    ("c5", "C5 2048³ / 50M IDW f32 + divergence (whole grid, 1 GPU)"),
    ("linear", "linear 256³ / 1M"),
    ("filter", "outlier filter 5M particles k=25"),
    ("mask", "mask sample + boundary 512³"),
    ("div_f64", "divergence 512³ f64"),
    ("div_f32", "divergence 512³ f32"),
]


def main(tag):
    d0 = os.path.join(ROOT, "profiles", f"{tag}_lines")
    print("| Line | Value | Step | Dominant kernel (hipEvent, per step) | rocprofv3 (per step) | Roofline frac (kernel / step) | CPU baseline |")
    print("|---|---|---|---|---|---|---|")
    libs = set()
    for name, label in ORDER:
        f = os.path.join(d0, name + ".json")
        if not os.path.exists(f):
            continue
        d = json.loads(open(f).read().strip().splitlines()[-1])
        r = d.get("roofline", {})
        cb = d.get("cpu_baseline") or {}
        libs.add(d.get("lib_sha256"))
        kt = ""
        ktf = os.path.join(d0, name + ".kt.txt")
        if os.path.exists(ktf):
            # the same command under rocprofv3 --kernel-trace: the dominant kernel's total over the
            # run's warmup + timed steps, per step (chunked launches, e.g. the RBF solve, summed)
            row = open(ktf).read().splitlines()[1].split()
            kt = f"{float(row[0]) / (d['steps'] + d['warmup']):.3f} ms"
        fs = r.get("frac_step")
        frac = f"{r.get('frac')}" + (f" / {fs}" if fs is not None else "") + f" ({r.get('bound')})"
        kern = str(r.get("kernel", "?")).split(" (")[0]
        extra = f", pivoted {r['n_rbf_pivoted']}" if r.get("n_rbf_pivoted") is not None else ""
        unit = d["unit"].split()[0]
        print(f"| {label} | {d['value']} {unit} | {d['ms_per_step']} ms | {kern} {r.get('kernel_ms')} ms{extra} | {kt} | "
              f"{frac} | {cb.get('value')} {cb.get('unit', '')} ({cb.get('cores')} cores, {cb.get('kind')}) |")
    print(f"\nlibraries: {sorted(x for x in libs if x)}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r05")

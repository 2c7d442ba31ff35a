"""One-GPU rehearsal of the N-rank strong split with the warmup re-cut (bench.py's rebalance):
every share of the even cut is timed (bench.py --share r/N), the cut is re-made from the measured
step times (zslab.balanced_bounds), twice, and the shares of the final cut are timed again.  The
N-GPU step is predicted as the slowest share (the ranks run concurrently, no collective in the step).
usage (GPU box): python tools/share_balance.py N [out_dir] [extra bench args...]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ptv_interpolation_amd import zslab  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
out = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/share_balance"
extra = sys.argv[3:]
os.makedirs(out, exist_ok=True)
nz = 512
for i, a in enumerate(extra):
    if a == "--grid":
        nz = int(extra[i + 1])
bounds = [0] + [zslab.rank_slab(nz, N, r)[1] for r in range(N)]


def run_all(tag, bounds):
    lines = []
    for r in range(N):
        cmd = [sys.executable, "-u", "bench.py", "--share", f"{r}/{N}", "--no-cpu-baseline", "--slabs",
               ",".join(str(b) for b in bounds)] + extra
        p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
        if p.returncode != 0:
            sys.exit(f"share {r}/{N} failed:\n{p.stderr[-3000:]}")
        line = json.loads(p.stdout.strip().splitlines()[-1])
        with open(os.path.join(out, f"{tag}_share_{r}of{N}.json"), "w") as f:
            f.write(json.dumps(line) + "\n")
        lines.append(line)
    t = [l["ms_per_step"] for l in lines]
    print(f"{tag}: bounds {bounds} step ms {t} worst {max(t):.3f}", flush=True)
    return t, lines


t, _ = run_all("even", bounds)
for it in range(2):
    bounds = zslab.balanced_bounds(bounds, t)
    t, lines = run_all(f"cut{it + 1}", bounds)
summary = {"n": N, "bounds": bounds, "step_ms": t, "worst_ms": max(t)}
with open(os.path.join(out, "summary.json"), "w") as f:
    f.write(json.dumps(summary) + "\n")
print(json.dumps(summary))

#!/bin/bash
# One-GPU rehearsal of the N-rank strong z-slab step (bench.py --share R/N) for the headline:
# the end slab and a middle slab of N = 8, 4, 2, with breakdown_ms (cull, bin, lattice, knn).
# usage: gpurun -- bash tools/gpu_r04_share.sh tag
set -o pipefail
tag=${1:-r04_share}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/$tag
mkdir -p "$out"
for s in 0/8 3/8 7/8 0/4 1/4 0/2; do
  n=${s/\//of}
  timeout -k 10 300 python -u bench.py --share $s --no-cpu-baseline > "$out/share_$n.json" 2> "$out/share_$n.err" || { echo "FAILED $s"; tail -20 "$out/share_$n.err"; exit 1; }
  python - "$out/share_$n.json" <<'PY'
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "ms_per_step", l["ms_per_step"], "breakdown", l.get("breakdown_ms"), "binned", l.get("config", {}).get("particles_binned", l.get("n_binned")))
PY
done

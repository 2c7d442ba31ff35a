#!/bin/bash
# All eight shares of the N = 8 strong z-slab step (bench.py --share r/8) plus r/4 and r/2, one
# GPU rehearsal each, with the breakdown (cull, bin, lattice, knn).  usage: gpurun -- bash tools/gpu_r04_share8.sh tag
set -o pipefail
tag=${1:-r04_share8}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/$tag
mkdir -p "$out"
for s in 0/8 1/8 2/8 3/8 4/8 5/8 6/8 7/8 0/4 1/4 2/4 3/4 0/2 1/2; do
  n=${s/\//of}
  timeout -k 10 300 python -u bench.py --share $s --no-cpu-baseline > "$out/share_$n.json" 2> "$out/share_$n.err" || { echo "FAILED $s"; tail -20 "$out/share_$n.err"; exit 1; }
  python - "$out/share_$n.json" <<'PY'
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "ms_per_step", l["ms_per_step"], "breakdown", l.get("breakdown_ms"))
PY
done

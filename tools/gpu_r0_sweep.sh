#!/bin/bash
# Dev sweep of the first search radius scale (lattice levels are unseeded) on the headline bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
for r in 1.0 1.25 1.5 2.0 1.0; do
  timeout -k 10 200 python bench.py --r0-scale $r --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r0.log 2>&1 || { tail -5 gpurun_out/r0.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/r0.log').read().strip().splitlines()[-1]);print(sys.argv[1], d['breakdown_ms'], d['ms_per_step'])" $r
done

#!/bin/bash
# Masked geometry bench lines: 512^3/5M and the C4 per-GPU workload 1024^3/10M (sphere-pack mask fused)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --mask --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r01_mask512_bench.json 2> gpurun_out/m512.err || { tail gpurun_out/m512.err; exit 1; }
timeout -k 10 500 python -u bench.py --mask --grid 1024 --particles 10000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r01_c4_1024_bench.json 2> gpurun_out/c4.err || { tail gpurun_out/c4.err; exit 1; }
for f in r01_mask512_bench r01_c4_1024_bench; do python3 -c "import json;d=json.loads(open('gpurun_out/$f.json').read().strip().splitlines()[-1]);print('$f', d['value'], d.get('fluid_mvoxels_per_s'), d['ms_per_step'], d['breakdown_ms'], d['roofline']['frac'])"; done

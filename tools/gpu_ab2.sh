#!/bin/bash
# Same-box A/B over several env settings of the headline bench: tools/gpu_ab2.sh "A=1 B=2" "A=0" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
for r in $(seq ${AB_ROUNDS:-1}); do
  for cfg in "$@"; do
    env $cfg timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e $AB_ARGS > gpurun_out/ab2.log 2>&1 || { tail -5 gpurun_out/ab2.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab2.log').read().strip().splitlines()[-1]);print(sys.argv[1], d['breakdown_ms'], d['ms_per_step'])" "$cfg"
  done
done

#!/bin/bash
# A/B a dev environment knob on the headline bench: tools/ab_env.sh VAR v1 v2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
var=$1; shift
for v in "$@"; do
  env "$var=$v" timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > "gpurun_out/ab_$v.log" 2>&1 || { tail -5 "gpurun_out/ab_$v.log"; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], d['breakdown_ms'], d['ms_per_step'])" "gpurun_out/ab_$v.log" "$var=$v"
done

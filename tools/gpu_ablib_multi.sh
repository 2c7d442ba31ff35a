#!/bin/bash
# Same-box A/B of library builds over several bench configurations (one line each):
# tools/gpu_ablib_multi.sh "bench args 1" "bench args 2" ... -- libA.so libB.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
cfgs=(); while [ "$1" != "--" ]; do cfgs+=("$1"); shift; done; shift
for cfg in "${cfgs[@]}"; do
  for L in "$@"; do
    PTV_LIB=$(realpath "$L") timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e $cfg > gpurun_out/abm.log 2>&1 || { tail -5 gpurun_out/abm.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/abm.log').read().strip().splitlines()[-1]);print(sys.argv[1], '|', sys.argv[2], d.get('breakdown_ms'), d['ms_per_step'])" "$cfg" "$L"
  done
done

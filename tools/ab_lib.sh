#!/bin/bash
# Same-box A/B of library builds on the headline bench: tools/ab_lib.sh libA.so libB.so [libC.so ...]
# (AB_ROUNDS rounds, default 2; extra bench args in AB_ARGS)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
for r in $(seq ${AB_ROUNDS:-2}); do
  for L in "$@"; do
    PTV_LIB=$(realpath "$L") timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e $AB_ARGS > gpurun_out/ab_lib.log 2>&1 || { tail -5 gpurun_out/ab_lib.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab_lib.log').read().strip().splitlines()[-1]);print(sys.argv[1], d['breakdown_ms'], d['ms_per_step'])" "$L"
  done
done

#!/bin/bash
# A/B library builds on the headline bench in one process sequence: tools/ab_lib.sh libA.so libB.so [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
a=$1; b=$2; n=${3:-2}
for r in $(seq $n); do
  for L in "$a" "$b"; do
    PTV_LIB=$(realpath "$L") timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_lib.log 2>&1 || { tail -5 gpurun_out/ab_lib.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab_lib.log').read().strip().splitlines()[-1]);print(sys.argv[1], d['breakdown_ms'], d['ms_per_step'])" "$L"
  done
done

#!/bin/bash
# Same-box A/B of two library builds on any bench line: tools/ab_args.sh libA.so libB.so "bench args" [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
a=$1; b=$2; args=$3; n=${4:-2}
for r in $(seq $n); do
  for L in "$a" "$b"; do
    PTV_LIB=$(realpath "$L") timeout -k 10 300 python bench.py $args --no-cpu-baseline --no-e2e > gpurun_out/ab_args.log 2>&1 || { tail -5 gpurun_out/ab_args.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab_args.log').read().strip().splitlines()[-1]);print(sys.argv[1], sys.argv[2], d.get('breakdown_ms'), d['ms_per_step'])" "$L" "$args"
  done
done

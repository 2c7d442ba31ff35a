#!/bin/bash
# A/B two library builds on the local-RBF Gaussian k=32 bench: tools/ab_rbf.sh libA.so libB.so [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
a=$1; b=$2; n=${3:-2}
for r in $(seq $n); do
  for L in "$a" "$b"; do
    PTV_LIB=$(realpath "$L") timeout -k 10 200 python bench.py --method rbf --k 32 --rbf-kernel gaussian --epsilon 0.3 --degree -1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_rbf.log 2>&1 || { tail -5 gpurun_out/ab_rbf.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab_rbf.log').read().strip().splitlines()[-1]);print(sys.argv[1], d['breakdown_ms'], d['ms_per_step'])" "$L"
  done
done

#!/bin/bash
# Same-box A/B of one bench line over dev-knob settings of one dev library: each setting run
# twice, alternating.  Output: gpurun_out/<tag>_envab/<i>_<n>.json
# usage: gpurun -- bash tools/gpu_envab.sh TAG LIB "bench args" "VAR=a VAR2=b; VAR=c; -"   ("-" = none)
set -o pipefail
tag=$1; lib=$2; args=$3; sets=$4
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/${tag}_envab
mkdir -p "$out"
IFS=';' read -ra SS <<< "$sets"
for i in 1 2; do
  n=0
  for st in "${SS[@]}"; do
    n=$((n + 1))
    envs=(); [ "$(echo $st)" != "-" ] && read -ra envs <<< "$st"
    env "${envs[@]}" PTV_LIB=$(realpath "$lib") timeout -k 10 300 python -u bench.py $args --no-cpu-baseline --no-e2e \
      > "$out/${i}_$n.json" 2> "$out/${i}_$n.err" || { echo "FAILED $st"; tail -5 "$out/${i}_$n.err"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$out/${i}_$n.json').read().strip().splitlines()[-1])
print('$i', '[$st]', d['ms_per_step'], d.get('breakdown_ms'))"
  done
done

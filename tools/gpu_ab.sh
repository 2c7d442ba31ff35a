#!/bin/bash
# Same-box A/B of bench lines over dev libraries: each (library, bench args) pair run twice,
# alternating, every run under its own time limit.  Output: gpurun_out/<tag>_ab/<lib>_<n>_<i>.json
# usage: gpurun -- bash tools/gpu_ab.sh TAG "lib1 lib2 ..." "args1; args2; ..."   (lib "-" = shipped)
set -o pipefail
tag=$1; libs=$2; specs=$3
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/${tag}_ab
mkdir -p "$out"
IFS=';' read -ra SP <<< "$specs"
for i in 1 2; do
  n=0
  for spec in "${SP[@]}"; do
    n=$((n + 1))
    for lib in $libs; do
      name=$(basename "$lib" .so)_${n}_$i
      if [ "$lib" = "-" ]; then name=shipped_${n}_$i; unset PTV_LIB; else export PTV_LIB=$(realpath "$lib"); fi
      timeout -k 10 300 python -u bench.py $spec --no-cpu-baseline --no-e2e > "$out/$name.json" 2> "$out/$name.err" || { echo "FAILED $name"; tail -5 "$out/$name.err"; exit 1; }
      python3 -c "
import json,sys; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1])
print('$name', '$spec', d['ms_per_step'], d.get('breakdown_ms'))"
    done
  done
done

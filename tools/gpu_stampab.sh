#!/bin/bash
# Per-wave stamps of the main k-NN launch under several dev builds (A/B of kernel variants).
# usage: gpurun -- bash tools/gpu_stampab.sh TAG "lib1 lib2 ..." "k method; k method; ..."
set -o pipefail
tag=$1; libs=$2; specs=$3
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
out=gpurun_out/${tag}_stamps.txt
: > $out
IFS=';' read -ra SP <<< "$specs"
for lib in $libs; do
  for spec in "${SP[@]}"; do
    echo "== $lib: $spec" >> $out
    PTV_LIB=$(realpath $lib) timeout -k 10 300 python -u tools/stamp_k.py 512 5000000 $spec >> $out 2>&1 || { cat $out; exit 1; }
  done
done
cat $out

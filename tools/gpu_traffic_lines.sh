#!/bin/bash
# HBM traffic (rocprofv3 FETCH_SIZE and WRITE_SIZE, one pass each) of the k-NN main launch of
# some bench lines: gpurun_out/traffic_<tag>/<name>/{fetch,write}; summarise with
# python tools/pmc_kernel.py gpurun_out/traffic_<tag>/<name> "k_knn_interp<".
# usage: gpurun -- bash tools/gpu_traffic_lines.sh TAG "name:bench args; name:bench args"
set -o pipefail
tag=$1; specs=$2
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
IFS=';' read -ra SP <<< "$specs"
for sp in "${SP[@]}"; do
  sp=$(echo $sp)
  name=${sp%%:*}; args=${sp#*:}
  out=gpurun_out/traffic_$tag/$name
  rm -rf "$out"; mkdir -p "$out"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$out/$c" -- python3 bench.py $args --steps 2 --warmup 1 \
      --no-cpu-baseline --no-e2e > "$out/$c.log" 2>&1 || { echo "FAILED $name $c"; tail -5 "$out/$c.log"; exit 1; }
  done
  echo "== $name done"
done

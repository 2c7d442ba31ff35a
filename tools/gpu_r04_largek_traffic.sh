#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the large-k main launches: IDW k = 50
# and Sibson k = 30 / 50 (spill traffic shows in WRITE_SIZE).  usage: gpurun -- bash tools/gpu_r04_largek_traffic.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
out=gpurun_out/largek_traffic
rm -rf "$out"; mkdir -p "$out"
for cfg in "idw 50" "sibson 30" "sibson 50"; do
  set -- $cfg
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$out/$1$2_$c" -- python3 bench.py --method $1 --k $2 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > "$out/$1$2_$c.log" 2>&1 || { echo "pass failed $cfg $c"; tail -5 "$out/$1$2_$c.log"; exit 1; }
  done
  python3 tools/pmc_kernel.py "$out" "k_knn_interp<" | grep -v "^ *SQ" > "$out/summary_$1$2.txt"
  rm -rf "$out"/*_FETCH_SIZE "$out"/*_WRITE_SIZE
  echo "== $cfg"; cat "$out/summary_$1$2.txt"
done

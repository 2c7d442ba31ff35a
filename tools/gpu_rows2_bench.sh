#!/bin/bash
# Bench lines + rocprofv3 kernel stats for the pore-mask path and the outlier filter.
# usage: tools/gpu_rows2_bench.sh r01
set -o pipefail
R=${1:-r01}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --method filter --steps 5 --warmup 2 > gpurun_out/${R}_filter_bench.json 2> gpurun_out/${R}_filter_bench.err || { tail -20 gpurun_out/${R}_filter_bench.err; exit 1; }
cat gpurun_out/${R}_filter_bench.json
timeout -k 10 300 python -u bench.py --method mask --steps 10 --warmup 3 > gpurun_out/${R}_mask_bench.json 2> gpurun_out/${R}_mask_bench.err || { tail -20 gpurun_out/${R}_mask_bench.err; exit 1; }
cat gpurun_out/${R}_mask_bench.json
for M in filter mask; do
  OUT=gpurun_out/prof_${R}_${M}; rm -rf "$OUT"; mkdir -p "$OUT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -- python3 bench.py --method $M --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/stats.log" 2>&1 || { tail -20 "$OUT/stats.log"; exit 1; }
done
find gpurun_out/prof_${R}_filter gpurun_out/prof_${R}_mask -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-5 "$f" | head -12; done

#!/bin/bash
# End-of-round evidence: PMC passes for the row kernels, filter bench + stats, headline bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
bash tools/gpu_pmc_rows.sh > /dev/null || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof_r01_filter; rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -- python3 bench.py --method filter --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/stats.log" 2>&1 || { tail -5 "$OUT/stats.log"; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/r01_bench.json 2> gpurun_out/r01_bench.err || { tail gpurun_out/r01_bench.err; exit 1; }
cat gpurun_out/r01_bench.json

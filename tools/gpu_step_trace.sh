#!/bin/bash
# Kernel timeline of the last full step of one bench line: tools/gpu_step_trace.sh <tag> "bench args" [ENV=val ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
tag=$1; cfg=$2; shift 2
out=gpurun_out/trace_$tag
rm -rf "$out"; mkdir -p "$out"
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$out" -- python3 bench.py --steps 3 --warmup 5 --no-cpu-baseline --no-e2e $cfg > "$out/bench.log" 2>&1 || { tail -5 "$out/bench.log"; exit 1; }
echo "== $tag: $cfg $*"; python3 tools/trace_step.py "$out" | tee "$out/step.txt"
find "$out" -name "*kernel_trace.csv" -delete

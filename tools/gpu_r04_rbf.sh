#!/bin/bash
# Round 4: local-RBF null-space kernel -- GPU tests, then TPS k=20 / k=32 bench lines at 512^3/5M
# (no CPU leg) with a rocprofv3 kernel-stats pass.  usage: gpurun -- bash tools/gpu_r04_rbf.sh tag
set -o pipefail
tag=${1:-r04a}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rbf.py -x -v -s --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { echo "TESTS FAILED"; tail -30 "$out/tests.log"; exit 1; }
tail -3 "$out/tests.log"
for kk in 20 32; do
  timeout -k 10 300 python -u bench.py --method rbf --k $kk --steps 3 --warmup 1 --no-cpu-baseline > "$out/tps$kk.json" 2> "$out/tps$kk.err" || { echo "BENCH FAILED k=$kk"; tail -20 "$out/tps$kk.err"; exit 1; }
  tail -c 600 "$out/tps$kk.json"; echo
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python -u bench.py --method rbf --k 20 --steps 2 --warmup 1 --no-cpu-baseline > "$out/prof.log" 2>&1 || { echo "PROF FAILED"; tail -20 "$out/prof.log"; exit 1; }
find "$out/prof" -name "*kernel_stats.csv" -exec head -12 {} \;

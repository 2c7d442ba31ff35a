#!/bin/bash
# Round evidence on the GPU box: profiles (stats + FETCH/WRITE passes), the default bench line
# with its CPU baseline, the fluid/solid split, and a local-RBF stats profile.
# usage: (locally) rm -rf gpurun_out/prof_r01* ; gpurun -- tools/round_evidence.sh r01
#        then (locally) python3 tools/traffic.py gpurun_out/prof_r01 r01 and copy the
#        gpurun_out/r01_* files into profiles/ (only gpurun_out/ comes back from the box)
set -o pipefail
R=${1:-r01}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
bash tools/collect_profiles.sh "$R" || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit 1
timeout -k 10 300 python tools/split_time.py 512 5000000 8 --stamps > gpurun_out/${R}_split.txt 2>&1 || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof_${R}_rbf; rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -- python3 bench.py --method rbf --k 32 --rbf-kernel gaussian --epsilon 0.3 --degree -1 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/stats.log" 2>&1 || exit 1

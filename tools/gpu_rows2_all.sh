#!/bin/bash
# parity (new rows) then bench lines + rocprof stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
bash tools/gpu_rows2.sh && bash tools/gpu_rows2_bench.sh ${1:-r01}

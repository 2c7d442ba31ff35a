#!/bin/bash
# Round-4 final evidence, part B: every bench line and every --share r/N rehearsal on the same
# build (after part A's traffic file is in profiles/).  usage: gpurun -- bash tools/gpu_r04_finalB.sh tag
set -o pipefail
tag=${1:-r04b}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
bash tools/gpu_lines.sh ${tag} > gpurun_out/${tag}_lines.log 2>&1 || { tail -20 gpurun_out/${tag}_lines.log; exit 1; }
bash tools/gpu_r04_share8.sh ${tag}_share > gpurun_out/${tag}_share.log 2>&1 || { tail -20 gpurun_out/${tag}_share.log; exit 1; }
echo done

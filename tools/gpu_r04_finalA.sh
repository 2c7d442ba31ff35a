#!/bin/bash
# Round-4 final evidence, part A: the whole -m gpu suite + smoke, rocprofv3 kernel-trace stats and
# FETCH/WRITE passes of the default bench (tools/collect_profiles.sh), SQ counters of the headline
# k-NN kernel and of the TPS k = 20 null-space kernel.  usage: gpurun -- bash tools/gpu_r04_finalA.sh tag
set -o pipefail
tag=${1:-r04b}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
SKIP_LINES=1 bash tools/gpu_r04_final.sh ${tag} || exit 1
bash tools/pmc_any.sh gpurun_out/pmc_${tag}_knn8 "k_knn_interp<8" --steps 3 --warmup 1 > /dev/null || exit 1
bash tools/pmc_any.sh gpurun_out/pmc_${tag}_ns20 k_rbf_ns --method rbf --k 20 --steps 1 --warmup 0 > /dev/null || exit 1
bash tools/pmc_any.sh gpurun_out/pmc_${tag}_spd32 k_rbf_spd16 --config c3 --steps 1 --warmup 0 > /dev/null || exit 1
echo done

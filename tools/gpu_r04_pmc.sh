#!/bin/bash
# Round-4 SQ counters: the headline k_knn_interp<8> and the TPS k = 20 null-space kernel.
# usage: gpurun -- bash tools/gpu_r04_pmc.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
bash tools/pmc_any.sh gpurun_out/pmc_r04_knn8 "k_knn_interp<8" --steps 3 --warmup 1 || exit 1
bash tools/pmc_any.sh gpurun_out/pmc_r04_ns20 k_rbf_ns --method rbf --k 20 --steps 1 --warmup 0 || exit 1

#!/bin/bash
# Round evidence in one GPU call: rocprofv3 stats + FETCH/WRITE passes, default bench line,
# fluid/solid split with stamps, local-RBF stats, SQ counter passes on the main k-NN launch.
# usage: gpurun -- bash tools/gpu_evidence.sh r02   (then tools/traffic.py locally)
set -o pipefail
R=${1:-r02}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
bash tools/round_evidence.sh "$R" || exit 1
bash tools/gpu_pmc.sh || exit 1
mkdir -p gpurun_out/pmc_$R && mv gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc_summary.txt gpurun_out/pmc_$R/

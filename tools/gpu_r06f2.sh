#!/bin/bash
# Round-6 final evidence (library with the half-block epilogue), second call: the remaining bench lines, the 8-share rehearsal and SQ
# counters of the headline, nearest and filter kernels on the shipped library.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
KT=1 LINES="idw_k50 sibson_k50 rbf_tps20 rbf_tps32 c3 c5 linear mask div_f64 div_f32" bash tools/gpu_lines.sh r06f || exit 1
timeout -k 10 600 python -u tools/share_balance.py 8 gpurun_out/r06f_balance > gpurun_out/r06f_balance.log 2>&1 || exit 1
tail -4 gpurun_out/r06f_balance.log
bash tools/pmc_any.sh gpurun_out/pmc_r06f/knn8 "k_knn_interp<8, false, 0" --steps 3 --warmup 1 || exit 1
bash tools/pmc_any.sh gpurun_out/pmc_r06f/knn1 "k_knn_interp<1, false, 0" --method nearest --steps 3 --warmup 1 || exit 1
bash tools/pmc_any.sh gpurun_out/pmc_r06f/filter "k_knn_interp<32, false, 4" --method filter --steps 3 --warmup 1 || exit 1

#!/bin/bash
# GPU round trip for the pore-mask path and the outlier filter.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_mask_filter.py tests/test_host.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_rows2.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_rows2.log; exit $rc

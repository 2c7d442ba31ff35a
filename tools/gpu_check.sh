#!/bin/bash
# GPU round trip: parity tests (all gpu-marked), headline bench, stamps split.
# usage: tools/gpu_check.sh [quick]   (quick: skip the full-size sampled tests)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
kexpr=""
[ "$1" = "quick" ] && kexpr="not full_size"
timeout -k 10 600 python -u -m pytest tests -m gpu ${kexpr:+-k "$kexpr"} -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print('value',d['value'],'ms',d['ms_per_step'],'frac',d['roofline']['frac'],'knn',d['breakdown_ms'])"

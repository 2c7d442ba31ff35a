#!/bin/bash
# RBF parity tests with the current build, then the TPS k=32 (M=36 -> 40) bench for two builds
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rbf.py tests/test_gpu_launcher.py -x -q --timeout 200 --timeout-method thread > gpurun_out/rbf_t.log 2>&1 || { tail -20 gpurun_out/rbf_t.log; exit 1; }
tail -1 gpurun_out/rbf_t.log
for L in "$1" "$2"; do
  PTV_LIB=$(realpath "$L") timeout -k 10 300 python bench.py --method rbf --k 32 --rbf-kernel thin_plate_spline --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/ab_tps.log 2>&1 || { tail -5 gpurun_out/ab_tps.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab_tps.log').read().strip().splitlines()[-1]);print(sys.argv[1], d['breakdown_ms'], d['ms_per_step'])" "$L"
done
bash tools/ab_rbf.sh "$1" "$2" 1

#!/bin/bash
# Half-block epilogue check: key-list tests on the shipped build, Sibson k = 30 HBM traffic with and
# without the half blocks, and timing A/B of the affected list lengths.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_keys.py tests/test_gpu_out_f32.py tests/test_gpu_bigk.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06z2_tests.log 2>&1; tail -2 gpurun_out/r06z2_tests.log
grep -q " passed" gpurun_out/r06z2_tests.log && ! grep -q "failed" gpurun_out/r06z2_tests.log || exit 1
for l in nohalf half32; do
  PTV_LIB=$PWD/abr6/libptv_$l.so bash tools/gpu_traffic_lines.sh r06z_$l "sibson30:--method sibson --k 30" || exit 1
  python3 tools/pmc_kernel.py gpurun_out/traffic_r06z_$l/sibson30 "k_knn_interp<32" > gpurun_out/traffic_r06z_$l/summary.txt 2>&1
  tail -6 gpurun_out/traffic_r06z_$l/summary.txt
done
bash tools/gpu_ab.sh r06z2 "abr6/libptv_nohalf.so abr6/libptv_half32.so" "--method idw --k 24 --steps 5 --warmup 1 --no-e2e; --method idw --k 50 --steps 5 --warmup 1 --no-e2e; --method sibson --k 30 --steps 10 --warmup 2 --no-e2e"

# value-pass split (u, v then w) and the filter's neighbour-blob seeds: tests, then A/B against the
# previous library (abr6/libptv_prev.so) on the key-list and filter lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_keys.py tests/test_gpu_parity.py tests/test_gpu_mask_filter.py tests/test_gpu_bigk.py > gpurun_out/r06i_tests.log 2>&1 || { tail -30 gpurun_out/r06i_tests.log; exit 2; }
tail -2 gpurun_out/r06i_tests.log
bash tools/gpu_ab.sh r06j "- abr6/libptv_prev.so abr6/libptv_fseeded.so" "--method filter --steps 10 --warmup 2"
bash tools/gpu_ab.sh r06i "- abr6/libptv_prev.so" "--method sibson --k 30 --steps 6 --warmup 2; --method idw --k 50 --steps 4 --warmup 1; --method idw --k 16 --steps 6 --warmup 2; --method sibson --k 50 --steps 4 --warmup 1"

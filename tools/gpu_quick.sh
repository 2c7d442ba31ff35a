# quick GPU check: GPU tests (no full size) + headline timing + fluid/solid split
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "not full_size" > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python tools/quick_time.py 512 5000000 8 0 ${STAMPS:-} > gpurun_out/qt512.log 2>&1 || { cat gpurun_out/qt512.log; exit 1; }
cat gpurun_out/qt512.log
if [ -n "$SPLIT" ]; then timeout -k 10 300 python tools/split_time.py 512 5000000 8 > gpurun_out/split512.log 2>&1 && cat gpurun_out/split512.log; fi

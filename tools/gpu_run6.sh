cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "not full_size" > gpurun_out/pytest_gpu.log 2>&1 ; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 200 python tools/quick_time.py 512 5000000 8 0 --stamps > gpurun_out/qt512.log 2>&1 || exit 1
timeout -k 10 300 python tools/split_time.py 512 5000000 8 > gpurun_out/split512.log 2>&1 || exit 1

cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -k "not full_size" > gpurun_out/pytest_gpu.log 2>&1 ; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
for occ in 1 2 3 6; do timeout -k 10 120 python tools/quick_time.py 512 5000000 8 $occ --counters >> gpurun_out/qt512.log 2>&1 || exit 1; done
timeout -k 10 120 python tools/quick_time.py 64 10000 8 0 --counters > gpurun_out/qt64.log 2>&1
timeout -k 10 120 python tools/quick_time.py 256 1000000 8 0 --counters > gpurun_out/qt256.log 2>&1

cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
timeout -k 10 300 python tools/split_time.py 512 5000000 8 > gpurun_out/split512.log 2>&1

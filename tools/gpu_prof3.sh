cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof1; mkdir -p gpurun_out/prof1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof1 -- python tools/quick_time.py 512 5000000 8 > gpurun_out/prof1.log 2>&1

set -o pipefail
mkdir -p gpurun_out
export PTV_LIB=$(realpath ab/libptv_stamp.so)
timeout -k 10 120 python -u tools/stamp_k.py 512 5000000 8 idw > gpurun_out/r03b_stamps.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/stamp_k.py 512 5000000 30 sibson >> gpurun_out/r03b_stamps.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/stamp_k.py 512 5000000 50 idw >> gpurun_out/r03b_stamps.txt 2>&1 || exit $?
cat gpurun_out/r03b_stamps.txt
unset PTV_LIB
timeout -k 10 120 python -u tools/xfer_bench.py 1 > gpurun_out/r03b_xfer.txt 2>&1 || exit $?
cat gpurun_out/r03b_xfer.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_main_pipeline.py -x -q --timeout 300 --timeout-method thread -s > gpurun_out/r03b_tests.log 2>&1; rc=$?
grep -E "normwise|ties|passed|failed" gpurun_out/r03b_tests.log | tail -60
exit $rc

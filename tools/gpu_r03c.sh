set -o pipefail
mkdir -p gpurun_out
cat /sys/kernel/mm/transparent_hugepage/enabled > gpurun_out/r03c_thp.txt 2>&1
timeout -k 10 300 python -u tools/e2e_profile.py 512 5000000 8 dense > gpurun_out/r03c_e2e_dense.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/e2e_profile.py 512 5000000 8 views > gpurun_out/r03c_e2e_views.txt 2>&1 || exit $?
head -8 gpurun_out/r03c_e2e_dense.txt gpurun_out/r03c_e2e_views.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -s -k "full_size" > gpurun_out/r03c_tests.log 2>&1; rc=$?
grep -E "normwise|passed|failed" gpurun_out/r03c_tests.log | tail -30
exit $rc

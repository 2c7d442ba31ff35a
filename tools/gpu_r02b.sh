#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -s -v --timeout 120 --timeout-method thread \
  "tests/test_gpu_rbf.py::test_golden_gaussian_scipy_oracle" "tests/test_gpu_rbf.py::test_extreme_pivots_take_the_ieee_path" \
  "tests/test_gpu_rbf.py::test_c3_full_size_gaussian_sampled" tests/test_gpu_zslab.py > gpurun_out/r02b_tests.log 2>&1
rc=$?
tail -8 gpurun_out/r02b_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
for cfg in "--config c4 --no-cpu-baseline" "--config c3 --no-cpu-baseline --steps 3 --warmup 1" "--config c5 --no-cpu-baseline --steps 3 --warmup 1"; do
  timeout -k 10 400 python -u bench.py $cfg >> gpurun_out/r02b_bench.json 2>> gpurun_out/r02b_bench.err || exit $?
  tail -1 gpurun_out/r02b_bench.json | cut -c1-400
done

#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/debug_c5div.py 512 2000000 > gpurun_out/r02c_dbg.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/debug_c5div.py 2048 50000000 >> gpurun_out/r02c_dbg.log 2>&1 || exit $?
cat gpurun_out/r02c_dbg.log
timeout -k 10 600 python -u -m pytest -s -v --timeout 120 --timeout-method thread tests/test_gpu_zslab.py::test_c5_rank_share_f32_and_divergence > gpurun_out/r02c_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r02c_tests.log; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r02c_bench.json 2> gpurun_out/r02c_bench.err || exit $?
cut -c1-3000 gpurun_out/r02c_bench.json

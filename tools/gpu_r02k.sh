#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_nearest_div.py tests/test_gpu_zslab.py::test_slab_cull_matches_whole_grid > gpurun_out/r02k_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r02k_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 tools/ab_lib.sh ptv_interpolation_amd/libptv_amd.so ab/libptv_prev.so 2
tools/gpu_r02j.sh

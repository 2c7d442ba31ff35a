#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/void_split.py > gpurun_out/r02d_void.log 2>&1 || { cat gpurun_out/r02d_void.log; exit 1; }
cat gpurun_out/r02d_void.log
timeout -k 10 600 tools/ab_lib.sh ptv_interpolation_amd/libptv_amd.so ab/libptv_w5.so 2

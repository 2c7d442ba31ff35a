#!/bin/bash
mkdir -p gpurun_out
OCCS=1.2,2.2,3.5,5.5,8 timeout -k 10 500 python -u tools/void_split.py > gpurun_out/r02e_void.log 2>&1 || { cat gpurun_out/r02e_void.log; exit 1; }
cat gpurun_out/r02e_void.log

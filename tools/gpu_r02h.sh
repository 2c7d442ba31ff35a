#!/bin/bash
mkdir -p gpurun_out
OCCS=16,24,32,48 XREFS=4,6,8,12 timeout -k 10 800 python -u tools/void_split.py > gpurun_out/r02h_void.log 2>&1 || { cat gpurun_out/r02h_void.log; exit 1; }
cat gpurun_out/r02h_void.log

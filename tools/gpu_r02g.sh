#!/bin/bash
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/pmc_knn.sh gpurun_out/r02g_pmc --steps 2 --warmup 1 --no-cpu-baseline --no-e2e
ls -R gpurun_out/r02g_pmc | head -30
for db in $(find gpurun_out/r02g_pmc -name "*.db"); do python3 tools/pmc_read.py "$db" --min-grid 100000000; done > gpurun_out/r02g_pmc.txt 2>&1
cat gpurun_out/r02g_pmc.txt | cut -c1-600

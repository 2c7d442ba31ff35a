#!/bin/bash
# SQ counters of the outlier-filter search kernel (one rocprofv3 --pmc pass, kernel-trace only)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/pmc_filter; rm -rf "$OUT"; mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $OUT/p1 -- python3 bench.py --method filter --steps 2 --warmup 1 --no-cpu-baseline > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p2 -- python3 bench.py --method filter --steps 2 --warmup 1 --no-cpu-baseline > $OUT/p2.log 2>&1 || { tail -5 $OUT/p2.log; exit 1; }
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt | grep -v "^  void\|^  ptv\|^  __"

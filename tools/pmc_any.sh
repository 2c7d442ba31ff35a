#!/bin/bash
# SQ counter passes (one rocprofv3 run each) over any bench configuration, summarised per kernel:
# tools/pmc_any.sh OUTDIR KERNEL_SUBSTR [bench args...]
set -o pipefail
out=$1; kern=$2; shift 2
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
rm -rf "$out"; mkdir -p "$out"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_BRANCH" \
           "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -- python3 bench.py --no-cpu-baseline --no-e2e "$@" > "$out/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$out/p$i.log"; exit 1; }
done
python3 tools/pmc_kernel.py "$out" "$kern" | tee "$out/summary.txt"

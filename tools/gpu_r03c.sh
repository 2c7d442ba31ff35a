#!/bin/bash
# Round-3 check after the packed-key lists: the whole -m gpu suite, per-wave stamps (stamp-all
# dev build) for k = 8 / Sibson 30 / IDW 50, and SQ + traffic counter passes of the k = 50 and
# Sibson 30 main launches.  usage: gpurun -- bash tools/gpu_r03c.sh TAG
set -o pipefail
tag=${1:-r03c}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/${tag}
mkdir -p "$out"
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
rc=$?
[ -n "$SKIP_TESTS" ] || tail -3 $out/tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $out/tests.log | head -20; exit $rc; fi
export PTV_LIB=$(realpath ab/libptv_stamp.so)
for spec in "8 idw" "30 sibson" "50 idw"; do
  timeout -k 10 300 python -u tools/stamp_k.py 512 5000000 $spec >> $out/stamps.txt 2>&1 || exit $?
done
cat $out/stamps.txt
unset PTV_LIB
export TMPDIR=/tmp
B50="--method idw --k 50 --steps 2 --warmup 1 --no-e2e --no-cpu-baseline"
B30="--method sibson --k 30 --steps 2 --warmup 1 --no-e2e --no-cpu-baseline"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAVES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  for which in 50 30; do
    eval args=\$B$which
    timeout -s KILL 240 rocprofv3 --pmc $grp -d "$out/k${which}_p$i" -o run -- python3 bench.py $args > "$out/k${which}_p$i.log" 2>&1 || { echo "pass $i k$which failed"; tail -5 "$out/k${which}_p$i.log"; exit 1; }
  done
done
python3 tools/pmc_db.py "k_knn_interp<56" $out/k50_p* > $out/k50_summary.txt 2>&1
python3 tools/pmc_db.py "k_knn_interp<32" $out/k30_p* > $out/k30_summary.txt 2>&1
grep -E "grid=|per wave|share of wave cycles SQ_ACTIVE_INST_VALU|per dispatch" $out/k50_summary.txt $out/k30_summary.txt

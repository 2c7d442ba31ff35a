#!/bin/bash
# Kernel timeline of one headline step per env setting: tools/gpu_trace.sh "A=1" "A=2" ...
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1)); rm -rf gpurun_out/trace$i
  for kv in $cfg; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace$i -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/trace$i.log 2>&1 || { tail -5 gpurun_out/trace$i.log; exit 1; }
  for kv in $cfg; do unset "${kv%%=*}"; done
  echo "== $cfg"; python3 tools/trace_step.py gpurun_out/trace$i
done

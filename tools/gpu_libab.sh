#!/bin/bash
# Same bench line under several library builds (same box): tools/gpu_libab.sh "libA libB" "bench args"
set -o pipefail
libs=$1; args=$2
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in $libs; do
    PTV_LIB=$(realpath $lib) timeout -k 10 300 python -u bench.py $args --no-cpu-baseline --no-e2e > gpurun_out/libab.json 2> gpurun_out/libab.err || { tail -5 gpurun_out/libab.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/libab.json')); r=d['roofline']; print('$lib', d['value'], d['unit'], d['ms_per_step'], 'ms kernel', r.get('kernel_ms'))"
  done
done

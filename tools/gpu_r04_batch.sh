#!/bin/bash
# A/B of the batched rank-2r broadcasts (PTV_NS_BATCH) on TPS k = 20 / 32, then the RBF suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/r04_batch
mkdir -p "$out"
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in ab/libptv_nb0.so ptv_interpolation_amd/libptv_amd.so; do
    for kk in 20 32; do
      PTV_LIB=$(realpath $lib) timeout -k 10 300 python -u bench.py --method rbf --k $kk --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > "$out/ab.json" 2> "$out/ab.err" || { echo "AB FAILED $lib"; tail -5 "$out/ab.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$out/ab.json').read().strip().splitlines()[-1]); print('$lib k=$kk', d['roofline'].get('kernel_ms'), d['roofline'].get('frac'))"
    done
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_rbf.py -q --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { echo TESTS FAILED; tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"

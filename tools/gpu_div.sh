#!/bin/bash
# Divergence kernel round trip: parity tests, f64 / f32 bench lines (both tile orders), optional PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_nearest_div.py -x -q --timeout 120 --timeout-method thread -k divergence > gpurun_out/pytest_div.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_div.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/pytest_div.log | head; exit $rc; }
for x in 0 1; do for dt in f64 f32; do
  PTV_DIV_XCD=$x timeout -k 10 200 python -u bench.py --method div --div-dtype $dt --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_div_$dt.log 2>&1 || { tail -20 gpurun_out/bench_div_$dt.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_div_$dt.log').read().strip().splitlines()[-1]);r=d['roofline'];print('xcd=$x $dt', r['kernel_ms'],'ms', r['achieved'],'GB/s', r['frac'])"
done; done
if [ "$1" = "pmc" ]; then
  export TMPDIR=/tmp
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/pmc_div_$c
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_div_$c -- python3 bench.py --method div --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_div_$c.log 2>&1 || { tail -5 gpurun_out/pmc_div_$c.log; exit 1; }
  done
fi

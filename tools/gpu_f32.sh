#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_out_f32.py tests/test_gpu_parity.py tests/test_gpu_mask_filter.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_f32.log 2>&1 || { tail -30 gpurun_out/pytest_f32.log; exit 1; }
tail -1 gpurun_out/pytest_f32.log
timeout -k 10 200 python -u bench.py --out-dtype f32 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r01_f32out_bench.json 2>gpurun_out/f32.err || { tail gpurun_out/f32.err; exit 1; }
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r01_f64out_bench.json 2>gpurun_out/f64.err || { tail gpurun_out/f64.err; exit 1; }
timeout -k 10 200 python -u bench.py --method filter --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/fb.json 2>gpurun_out/fb.err || { tail gpurun_out/fb.err; exit 1; }
for f in r01_f32out_bench r01_f64out_bench fb; do python3 -c "import json,sys;d=json.loads(open('gpurun_out/$f.json').read().strip().splitlines()[-1]);print('$f', d['value'], d.get('breakdown_ms'), d['roofline']['frac'])"; done

#!/bin/bash
mkdir -p gpurun_out
for r in 0.8 1.3 1.6 2.0 2.5; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --r0-scale $r > gpurun_out/r02j.log 2>&1 || { tail -3 gpurun_out/r02j.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/r02j.log').read().strip().splitlines()[-1]);print('r0', sys.argv[1], d['breakdown_ms'], d['ms_per_step'])" $r
done

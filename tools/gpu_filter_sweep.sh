#!/bin/bash
# Dev sweep of the outlier-filter search knobs (first radius scale, cell occupancy).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 120 python -u bench.py --method filter --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/fs.log 2>&1 || { tail -5 gpurun_out/fs.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/fs.log').read().strip().splitlines()[-1]);print(sys.argv[1:], d['breakdown_ms'])" "$@"
}
run PTV_FILTER_R0=1.0
run PTV_FILTER_R0=1.3
run PTV_FILTER_R0=0.8
run PTV_FILTER_OCC=0.6
run PTV_FILTER_OCC=2.5
run PTV_FILTER_OCC=5.5

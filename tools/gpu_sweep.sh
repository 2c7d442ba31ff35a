#!/bin/bash
# Same-box sweep of dev knobs (a PTV_DEV_KNOBS build under PTV_LIB) over one bench configuration:
# tools/gpu_sweep.sh "bench args" "VAR=a VAR2=b" "VAR=c" ...  (one line of breakdown per setting)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
cfg=$1; shift
for setting in "$@"; do
  env $setting timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e $cfg > gpurun_out/sweep.log 2>&1 || { tail -5 gpurun_out/sweep.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/sweep.log').read().strip().splitlines()[-1]);print(sys.argv[1], '|', sys.argv[2], d.get('breakdown_ms'), d['ms_per_step'], d.get('cull', {}).get('particles_binned'))" "$cfg" "$setting"
done

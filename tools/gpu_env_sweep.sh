#!/bin/bash
# Dev-knob sweep of bench lines under the dev-knob build (ab/libptv_knobs.so), same box:
# tools/gpu_env_sweep.sh "bench args" "SPEC SPEC ..."   (SPEC = NAME=VALUE[,NAME=VALUE], '-' = none)
# Several bench arg sets: separate them with '|'.
set -o pipefail
argsets=$1; specs=$2
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PTV_LIB=$(realpath ab/libptv_knobs.so)
IFS='|' read -ra ARGS <<< "$argsets"
for args in "${ARGS[@]}"; do
  for spec in $specs; do
    envs=()
    [ "$spec" != "-" ] && IFS=',' read -ra envs <<< "$spec"
    env "${envs[@]}" timeout -k 10 300 python -u bench.py $args --no-cpu-baseline --no-e2e > gpurun_out/envsweep.json 2> gpurun_out/envsweep.err || { tail -5 gpurun_out/envsweep.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/envsweep.json')); r=d['roofline']; b=d.get('breakdown_ms', {}); print('$args [$spec]:', d['ms_per_step'], 'ms step, kernel', r.get('kernel_ms'), 'bin', b.get('bin'), 'lattice', b.get('lattice'))"
  done
done

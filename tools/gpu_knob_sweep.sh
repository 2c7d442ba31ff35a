#!/bin/bash
# Cell-shape sweep of one bench line under the dev-knob build (ab/libptv_knobs.so):
# tools/gpu_knob_sweep.sh "bench args" "occ:xref occ:xref ..."
set -o pipefail
args=$1; specs=$2
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PTV_LIB=$(realpath ab/libptv_knobs.so)
for spec in $specs; do
  occ=${spec%%:*}; xref=${spec##*:}
  PTV_CELL_OCC=$occ PTV_CELL_XREF=$xref PTV_FILTER_OCC=$occ timeout -k 10 300 python -u bench.py $args --no-cpu-baseline --no-e2e > gpurun_out/knob.json 2> gpurun_out/knob.err || { tail -5 gpurun_out/knob.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/knob.json')); r=d['roofline']; b=d.get('breakdown_ms', {}); print('$args occ=$occ xref=$xref:', d['ms_per_step'], 'ms step, kernel', r.get('kernel_ms'), 'bin', b.get('bin'), 'lattice', b.get('lattice'))"
done

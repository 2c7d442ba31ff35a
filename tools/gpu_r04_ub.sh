#!/bin/bash
# A/B of the radius growth toward a loose lattice bound (PTV_KNN_UB_GROW): lattice-level time in
# the headline and the worst z-slab shares, then the k-NN exactness tests on the shipped build.
set -o pipefail
tag=${1:-r04_ub}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for lib in ab/libptv_ubold.so ptv_interpolation_amd/libptv_amd.so ab/libptv_ub2.so; do
  for args in "--steps 10 --warmup 2" "--share 2/8" "--share 1/4" "--method filter" "--method sibson --k 30 --steps 5 --warmup 1"; do
    PTV_LIB=$(realpath $lib) timeout -k 10 300 python -u bench.py $args --no-cpu-baseline --no-e2e > "$out/ab.json" 2> "$out/ab.err" || { echo "AB FAILED $lib $args"; tail -5 "$out/ab.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/ab.json').read().strip().splitlines()[-1]); print('$lib', '$args', d['ms_per_step'], d.get('breakdown_ms'))"
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_keys.py tests/test_gpu_launcher.py -q --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { echo TESTS FAILED; tail -30 "$out/tests.log"; exit 1; }
tail -2 "$out/tests.log"

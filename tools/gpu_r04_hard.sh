#!/bin/bash
# A/B of the void-tile re-routing (k_kdist_hard; dev knob PTV_KNN_HARD = factor of r0, 0 = off)
# on the headline, the worst strong-split shares and C2; then the k-NN exactness tests on the
# shipped build.  usage: gpurun -- bash tools/gpu_r04_hard.sh
set -o pipefail
tag=${1:-r04_hard}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
lib=$(realpath ab/libptv_hdev.so)
for f in 0 8 4 16; do
  for args in "--steps 10 --warmup 2" "--share 2/8" "--share 1/4" "--share 0/8" "--config c2"; do
    PTV_KNN_HARD=$f PTV_LIB=$lib timeout -k 10 300 python -u bench.py $args --no-cpu-baseline --no-e2e > "$out/ab.json" 2> "$out/ab.err" || { echo "AB FAILED $f $args"; tail -5 "$out/ab.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/ab.json').read().strip().splitlines()[-1]); print('hard=$f', '$args', d['ms_per_step'], d.get('breakdown_ms'))"
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_keys.py tests/test_gpu_launcher.py tests/test_gpu_zslab.py -q --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { echo TESTS FAILED; tail -30 "$out/tests.log"; exit 1; }
tail -2 "$out/tests.log"

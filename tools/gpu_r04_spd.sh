#!/bin/bash
# RBF suite (incl. the SPD register kernel vs the LDS kernel bit-identity and C3 at full size)
# and the C3 / TPS lines without CPU baselines.  usage: gpurun -- bash tools/gpu_r04_spd.sh tag
set -o pipefail
tag=${1:-r04_spd}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_rbf.py -v -s --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { echo TESTS FAILED; tail -40 "$out/tests.log"; exit 1; }
tail -2 "$out/tests.log"
for a in "--config c3" "--method rbf --k 20 --steps 3 --warmup 1"; do
  timeout -k 10 600 python -u bench.py $a --no-cpu-baseline > "$out/l.json" 2> "$out/l.err" || { echo "BENCH FAILED $a"; tail -20 "$out/l.err"; exit 1; }
  python -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$a', l['ms_per_step'], l['roofline'].get('kernel_ms'), l['roofline'].get('frac'))" "$out/l.json"
done

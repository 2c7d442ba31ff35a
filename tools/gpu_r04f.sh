#!/bin/bash
# Round 4 GPU check of the persistent null-space kernel: RBF tests, stamps, TPS k=20/32 lines.
set -o pipefail
tag=${1:-r04f}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_rbf.py -v -s --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { echo TESTS FAILED; tail -40 "$out/tests.log"; exit 1; }
tail -2 "$out/tests.log"
PTV_LIB=ab/libptv_nsst.so timeout -k 10 300 python -u tools/ns_stamps.py 256 625000 20 32 > "$out/stamps.txt" 2>&1; cat "$out/stamps.txt"
for kk in 20 32; do
  timeout -k 10 300 python -u bench.py --method rbf --k $kk --steps 3 --warmup 1 --no-cpu-baseline > "$out/tps$kk.json" 2> "$out/tps$kk.err" || { echo "BENCH FAILED k=$kk"; tail -20 "$out/tps$kk.err"; exit 1; }
  python -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], l['ms_per_step'], l['roofline'])" "$out/tps$kk.json"
done

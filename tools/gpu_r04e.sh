#!/bin/bash
# Round 4 GPU check: tests for the changed paths, null-space stamps + TPS lines, the large-k
# epilogue A/B (base / LDS slot lists at 3 and 2 waves / rolled), the --share rehearsal.
set -o pipefail
tag=${1:-r04e}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_launcher.py tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { echo TESTS FAILED; tail -40 "$out/tests.log"; exit 1; }
tail -2 "$out/tests.log"
grep -E "binned per slab|whole-launch|null-space vs oracle" "$out/tests.log" | head -30
PTV_LIB=ab/libptv_nsst.so timeout -k 10 300 python -u tools/ns_stamps.py 256 625000 20 32 > "$out/stamps.txt" 2>&1; cat "$out/stamps.txt"
for kk in 20 32; do
  timeout -k 10 300 python -u bench.py --method rbf --k $kk --steps 3 --warmup 1 --no-cpu-baseline > "$out/tps$kk.json" 2> "$out/tps$kk.err" || { echo "BENCH FAILED k=$kk"; tail -20 "$out/tps$kk.err"; exit 1; }
  python -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], l['roofline'])" "$out/tps$kk.json"
done
for args in "--method sibson --k 30 --steps 5 --warmup 1" "--method idw --k 50 --steps 3 --warmup 1"; do
  for lib in ab/libptv_base.so ptv_interpolation_amd/libptv_amd.so ab/libptv_w2.so ab/libptv_roll.so; do
    PTV_LIB=$(realpath $lib) timeout -k 10 300 python -u bench.py $args --no-cpu-baseline --no-e2e > "$out/ab.json" 2> "$out/ab.err" || { echo "AB FAILED $lib $args"; tail -5 "$out/ab.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/ab.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$args', '$lib', d['ms_per_step'], 'ms, kernel', r.get('kernel_ms'), 'frac', r.get('frac'))"
  done
done
bash tools/gpu_r04_share.sh ${tag}_share

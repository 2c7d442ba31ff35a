#!/bin/bash
# Full refresh on one box: smoke, every gpu test, headline bench + profiles (round_evidence),
# divergence f64/f32 and nearest bench lines with CPU baselines, divergence stats profile.
set -o pipefail
R=${1:-r01}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/round_evidence.sh "$R" || exit 1
for dt in f64 f32; do
  timeout -k 10 300 python -u bench.py --method div --div-dtype $dt --steps 20 --warmup 3 > gpurun_out/${R}_div_${dt}_bench.json 2> gpurun_out/${R}_div_${dt}.err || { tail -20 gpurun_out/${R}_div_${dt}.err; exit 1; }
done
timeout -k 10 300 python -u bench.py --method nearest --steps 5 --warmup 2 > gpurun_out/${R}_nearest_bench.json 2> gpurun_out/${R}_nearest.err || { tail -20 gpurun_out/${R}_nearest.err; exit 1; }
export TMPDIR=/tmp
OUT=gpurun_out/prof_${R}_div; rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -- python3 bench.py --method div --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/stats.log" 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --method rbf --k 32 --rbf-kernel gaussian --epsilon 0.3 --degree -1 --steps 2 --warmup 1 > gpurun_out/${R}_rbf_gaussian_bench.json 2> gpurun_out/${R}_rbf.err || { tail -20 gpurun_out/${R}_rbf.err; exit 1; }
timeout -k 10 300 python -u bench.py --method filter --steps 5 --warmup 2 > gpurun_out/${R}_filter_bench.json 2> gpurun_out/${R}_filter.err || { tail -20 gpurun_out/${R}_filter.err; exit 1; }
timeout -k 10 300 python -u bench.py --method mask --steps 10 --warmup 3 > gpurun_out/${R}_mask_bench.json 2> gpurun_out/${R}_mask.err || { tail -20 gpurun_out/${R}_mask.err; exit 1; }
timeout -k 10 300 python -u bench.py --mask --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${R}_masked512_bench.json 2> gpurun_out/${R}_m512.err || { tail -20 gpurun_out/${R}_m512.err; exit 1; }
cat gpurun_out/${R}_bench.json

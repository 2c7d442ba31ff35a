#!/bin/bash
# GPU round trip for the nearest / divergence rows: parity tests, bench lines, rocprof stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nearest_div.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_new.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench.py --method div --steps 20 --warmup 3 > gpurun_out/bench_div64.log 2>&1 || { tail -20 gpurun_out/bench_div64.log; exit 1; }
tail -1 gpurun_out/bench_div64.log
timeout -k 10 200 python -u bench.py --method div --div-dtype f32 --steps 20 --warmup 3 > gpurun_out/bench_div32.log 2>&1 || { tail -20 gpurun_out/bench_div32.log; exit 1; }
tail -1 gpurun_out/bench_div32.log
timeout -k 10 200 python -u bench.py --method nearest --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_nearest.log 2>&1 || { tail -20 gpurun_out/bench_nearest.log; exit 1; }
tail -1 gpurun_out/bench_nearest.log
rm -rf gpurun_out/prof_div
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_div -- python3 bench.py --method div --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_div.log 2>&1 || { tail -20 gpurun_out/prof_div.log; exit 1; }
find gpurun_out/prof_div -name "*kernel_stats.csv" | head -1 | xargs head -5

# Round profile collection on the GPU box (run from the repo root via gpurun):
#   1. rocprofv3 --kernel-trace --stats of the default bench command
#   2. separate --pmc FETCH_SIZE and --pmc WRITE_SIZE passes (they do not fit one pass)
#   3. tools/traffic.py turns them into profiles/traffic_<round>.json + a stats summary
# Usage: bash tools/collect_profiles.sh r01
set -e
R=${1:-r01}
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$R
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -- python3 $B > "$OUT/stats.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -- python3 $B > "$OUT/fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -- python3 $B > "$OUT/write.log" 2>&1
python3 tools/traffic.py "$OUT" "$R"

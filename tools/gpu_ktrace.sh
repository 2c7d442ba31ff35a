#!/bin/bash
# rocprofv3 kernel-trace stats of one short bench run: tools/gpu_ktrace.sh <tag> "bench args" [ENV=val ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
tag=$1; cfg=$2; shift 2
out=gpurun_out/kt_$tag
rm -rf "$out"; mkdir -p "$out"
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e $cfg > "$out/bench.log" 2>&1 || { tail -5 "$out/bench.log"; exit 1; }
f=$(find "$out" -name "*kernel_stats.csv" | head -1)
python3 - "$f" "$tag" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print("==", sys.argv[2])
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms total {int(r["Calls"]):5d} calls {float(r["AverageNs"])/1e3:10.1f} us avg {float(r["MaxNs"])/1e3:10.1f} us max  {r["Name"][:90]}')
PY

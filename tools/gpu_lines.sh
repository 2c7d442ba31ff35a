#!/bin/bash
# Every bench line of the round in one GPU call (config lines + the rows next to the path), each
# under its own time limit; stops at the first failure.  Output: gpurun_out/<tag>_lines/<name>.json
# usage: gpurun -- bash tools/gpu_lines.sh r02
set -o pipefail
tag=${1:-r02}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/${tag}_lines
mkdir -p "$out"
run() {  # name, time limit, bench args...  (LINES="a b c" runs only those)
  local name=$1 lim=$2; shift 2
  if [ -n "$LINES" ] && [[ " $LINES " != *" $name "* ]]; then return 0; fi
  echo "== $name: bench.py $*"
  timeout -k 10 "$lim" python -u bench.py "$@" > "$out/$name.json" 2> "$out/$name.err" || { echo "FAILED $name"; tail -5 "$out/$name.err"; exit 1; }
  tail -c 400 "$out/$name.json"; echo
  if [ -n "$KT" ]; then  # the same line again under rocprofv3 kernel-trace: its kernels' durations
    export TMPDIR=/tmp
    rm -rf "$out/kt_$name"
    timeout -k 10 "$lim" rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt_$name" -- python3 bench.py "$@" \
      --no-cpu-baseline --no-e2e > "$out/kt_$name.log" 2>&1 || { echo "FAILED kt $name"; tail -5 "$out/kt_$name.log"; exit 1; }
    python3 tools/kt_summary.py "$out/kt_$name" 12 > "$out/$name.kt.txt" && head -4 "$out/$name.kt.txt"
    find "$out/kt_$name" -name "*kernel_trace.csv" -delete
  fi
}
run headline 300
run nearest 300 --method nearest --no-e2e
run sibson 300 --method sibson --k 30 --no-e2e
run idw_k50 400 --method idw --k 50 --steps 5 --warmup 1 --no-e2e
run sibson_k50 400 --method sibson --k 50 --steps 5 --warmup 1 --no-e2e
run rbf_tps20 600 --method rbf --k 20 --steps 3 --warmup 1
run rbf_tps32 600 --method rbf --k 32 --steps 3 --warmup 1
run c2 300 --config c2
run c2r 300 --config c2r
run c3 600 --config c3
run c4 600 --config c4 --steps 5 --warmup 1
run c5 900 --config c5 --steps 3 --warmup 1
run linear 600 --method linear --steps 10 --warmup 2
run filter 300 --method filter
run mask 300 --method mask
run div_f64 300 --method div
run div_f32 300 --method div --div-dtype f32
# one-GPU rehearsal of every rank share of the strong split (only when LINES names them)
for s in 0/8 1/8 2/8 3/8 4/8 5/8 6/8 7/8 0/4 1/4 2/4 3/4 0/2 1/2; do
  n=share_${s/\//of}
  if [ -n "$LINES" ] && [[ " $LINES " == *" $n "* || " $LINES " == *" shares "* ]]; then
    LINES="$n" run $n 300 --share $s --no-cpu-baseline
  fi
done

#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter per run) for the filter, mask and divergence benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/pmc_rows; rm -rf "$OUT"; mkdir -p "$OUT"
for row in filter mask div; do
  steps=3; [ $row = filter ] && steps=2
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$OUT/${row}_$([ $c = FETCH_SIZE ] && echo fetch || echo write)
    timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $d -- python3 bench.py --method $row --steps $steps --warmup 1 --no-cpu-baseline > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  done
done
ls $OUT

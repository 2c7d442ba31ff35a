#!/bin/bash
# One development iteration on the GPU box: the named test files, then optional bench lines.
# usage: gpurun -- bash tools/gpu_iter.sh TAG "tests/test_a.py tests/test_b.py" [bench args; bench args; ...]
set -o pipefail
tag=${1:-iter}; tests=$2; shift 2
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
if [ -n "$tests" ]; then
  timeout -k 10 900 python -u -m pytest $tests -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed|repaired|normwise|Error" gpurun_out/${tag}_tests.log | tail -60
  if [ $rc -ne 0 ]; then echo "pytest exit $rc"; exit $rc; fi
fi
i=0
for extra in "$@"; do
  i=$((i+1))
  timeout -k 10 600 python -u bench.py $extra > gpurun_out/${tag}_bench$i.json 2> gpurun_out/${tag}_bench$i.err || { echo "bench $i failed"; tail -5 gpurun_out/${tag}_bench$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${tag}_bench$i.json')); print('$extra', '->', d['value'], d['unit'], d['ms_per_step'], 'ms', d['roofline'].get('kernel'), d['roofline'].get('kernel_ms'), 'ms frac', d['roofline'].get('frac'))"
done

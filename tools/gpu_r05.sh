#!/bin/bash
# Round-5 iteration call: selected -m gpu tests (TESTS, pytest node ids / files) then selected bench
# lines (LINES, names from tools/gpu_lines.sh), each step under its own time limit, stopping at the
# first failure.  usage: gpurun -- 'TESTS="tests/test_gpu_rbf.py" LINES="headline" bash tools/gpu_r05.sh r05a'
set -o pipefail
tag=${1:-r05}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $TESTS -m gpu -v -s --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_tests.log 2>&1
  rc=$?
  grep -E "passed|failed" gpurun_out/${tag}_tests.log | tail -2
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/${tag}_tests.log | head -30; exit $rc; fi
fi
if [ -n "$LINES" ]; then
  LINES="$LINES" bash tools/gpu_lines.sh ${tag}
fi

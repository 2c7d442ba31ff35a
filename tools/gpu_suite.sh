#!/bin/bash
# One GPU call: the -m gpu suite, then the default bench line (+ optional extra bench args as
# further lines).  Usage: tools/gpu_suite.sh TAG [extra bench.py argument strings ...]
# Stops at the first GPU fault / abort / timeout (exit status > 1 from pytest).
tag=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
    > gpurun_out/${tag}_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${tag}_tests.log
if [ $rc -gt 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit $?
cat gpurun_out/${tag}_bench.json
for extra in "$@"; do
    timeout -k 10 600 python -u bench.py $extra >> gpurun_out/${tag}_bench_extra.json 2>> gpurun_out/${tag}_bench.err || exit $?
done
exit $rc

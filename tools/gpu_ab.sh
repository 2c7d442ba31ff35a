#!/bin/bash
# One GPU call: the k-NN parity tests, then a same-box A/B of a dev knob on the headline bench.
# usage: tools/gpu_ab.sh VAR v1 v2 ...   (tests: PTV_AB_TESTS, default the parity + zslab files)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
T=${PTV_AB_TESTS:-"tests/test_gpu_parity.py tests/test_gpu_nearest_div.py tests/test_gpu_zslab.py"}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $T > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/ab_env.sh "$@"

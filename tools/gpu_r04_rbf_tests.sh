set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/tiny
timeout -k 10 600 python -u -m pytest tests/test_gpu_rbf.py -q --timeout 300 --timeout-method thread > gpurun_out/tiny/tests.log 2>&1; rc=$?; tail -15 gpurun_out/tiny/tests.log; exit $rc

# speculative cull-map reuse: the cull tests, the share-2 line and its step trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_launcher.py tests/test_gpu_zslab.py tests/test_gpu_shares.py > gpurun_out/r06p_tests.log 2>&1 || { tail -30 gpurun_out/r06p_tests.log; exit 2; }
grep -E "passed|failed" gpurun_out/r06p_tests.log | tail -1
timeout -k 10 300 python -u bench.py --share 2/8 --slabs 0,77,138,186,257,327,372,434,512 --no-cpu-baseline > gpurun_out/r06p_share2.json 2> gpurun_out/r06p_share2.err || exit 3
python3 -c "
import json; d=json.loads(open('gpurun_out/r06p_share2.json').read().strip().splitlines()[-1]); print('share2', d['ms_per_step'], d['breakdown_ms'], d['cold_call'])"
bash tools/gpu_step_trace.sh share2p "--share 2/8 --slabs 0,77,138,186,257,327,372,434,512" > gpurun_out/r06p_trace.log 2>&1 || exit 4

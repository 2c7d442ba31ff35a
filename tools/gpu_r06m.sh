# tests touching the k-NN kernel, the headline line, and the 8-way share rehearsal with re-cuts
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_keys.py tests/test_gpu_mask_filter.py tests/test_gpu_nearest_div.py tests/test_gpu_shares.py > gpurun_out/r06m_tests.log 2>&1 || { tail -30 gpurun_out/r06m_tests.log; exit 2; }
tail -1 gpurun_out/r06m_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/r06m_headline.json 2> gpurun_out/r06m_headline.err || exit 3
python3 -c "
import json; d=json.loads(open('gpurun_out/r06m_headline.json').read().strip().splitlines()[-1]); print('headline', d['ms_per_step'], d['breakdown_ms'])"
timeout -k 10 900 python -u tools/share_balance.py 8 gpurun_out/r06m_balance > gpurun_out/r06m_balance.log 2>&1 || { tail -5 gpurun_out/r06m_balance.log; exit 4; }
cat gpurun_out/r06m_balance.log

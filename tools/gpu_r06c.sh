# round-6 check: the full GPU suite (-rA -s), then the share-2 step trace, the headline and share-2 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
tag=${1:-r06c}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -rA -s --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/${tag}_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/${tag}_tests.log
[ $rc -eq 0 -o $rc -eq 1 ] || exit $rc
bash tools/gpu_step_trace.sh share2 "--share 2/8 --slabs 0,79,139,186,257,327,372,432,512" > gpurun_out/${tag}_trace.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${tag}_headline.json 2> gpurun_out/${tag}_headline.err || exit 4
tail -c 600 gpurun_out/${tag}_headline.json
timeout -k 10 300 python -u bench.py --share 2/8 --slabs 0,79,139,186,257,327,372,432,512 --no-cpu-baseline > gpurun_out/${tag}_share2.json 2> gpurun_out/${tag}_share2.err || exit 5
tail -c 600 gpurun_out/${tag}_share2.json
exit $rc

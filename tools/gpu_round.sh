# Full round check on the GPU box: GPU tests, smoke, profiles, headline bench line.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu_all.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_all.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_all.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
bash tools/collect_profiles.sh ${1:-r01} > gpurun_out/collect.log 2>&1 || { tail -30 gpurun_out/collect.log; exit 1; }
cp profiles/* gpurun_out/ 2>/dev/null
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log

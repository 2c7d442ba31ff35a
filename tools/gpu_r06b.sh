set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -rA -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bigk.py tests/test_gpu_keys.py::test_k_above_n_raises tests/test_gpu_rbf.py::test_huge_systems_vs_oracle tests/test_gpu_rbf.py::test_large_systems_vs_oracle > gpurun_out/r06b_bigk.log 2>&1
rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 -o $rc -eq 1 ] || exit $rc
bash tools/gpu_step_trace.sh share2 "--share 2/8 --slabs 0,79,139,186,257,327,372,432,512" > gpurun_out/r06b_trace.log 2>&1 || exit 3
bash tools/gpu_ab.sh r06b "- abr6/libptv_k1w4.so" "--method nearest --steps 10 --warmup 3" > gpurun_out/r06b_ab1.log 2>&1 || exit 4
bash tools/gpu_ab.sh r06c "- abr6/libptv_keep24.so" "--method sibson --k 30 --steps 6 --warmup 2" > gpurun_out/r06b_ab2.log 2>&1 || exit 5
exit $rc

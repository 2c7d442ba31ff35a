# adaptive lattice split: A/B of the split rule on shares 2 and 0 and the headline (dev knob library),
# then the shipped library's lattice-sensitive tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
L=abr6/libptv_knobs.so
S="--slabs 0,79,139,186,257,327,372,432,512 --steps 20 --warmup 5"
bash tools/gpu_envab.sh r06h2 $L "--share 2/8 $S" "-; PTV_LAT_SPLIT_POW=1; PTV_LAT_SPLIT_POW=3; PTV_LAT_SPLIT=8; PTV_LAT_SPLIT_BLOCKS=192" > gpurun_out/r06h2.log 2>&1 || exit 2
bash tools/gpu_envab.sh r06h0 $L "--share 0/8 $S" "-; PTV_LAT_SPLIT_POW=1; PTV_LAT_SPLIT_POW=3; PTV_LAT_SPLIT=8" > gpurun_out/r06h0.log 2>&1 || exit 3
bash tools/gpu_envab.sh r06hh $L "--steps 10 --warmup 3" "-; PTV_LAT_SPLIT_POW=1; PTV_LAT_SPLIT_POW=3; PTV_LAT_SPLIT=8; PTV_LAT_SPLIT_ADAPT=0 PTV_LAT_SPLIT_BLOCKS=64" > gpurun_out/r06hh.log 2>&1 || exit 4
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_shares.py tests/test_gpu_parity.py tests/test_gpu_keys.py tests/test_gpu_launcher.py tests/test_gpu_zslab.py > gpurun_out/r06h_tests.log 2>&1

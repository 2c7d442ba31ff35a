set -o pipefail
mkdir -p gpurun_out/r04d
timeout -k 10 600 python -u -m pytest tests/test_gpu_launcher.py tests/test_gpu_parity.py "tests/test_gpu_keys.py::test_lattice_ties_whole_launch_rerun" -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04d/tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r04d/tests.log; exit 1; }
tail -3 gpurun_out/r04d/tests.log
grep -E "binned per slab|excluded voxels|whole-launch" gpurun_out/r04d/tests.log | head -20
PTV_LIB=ab/libptv_nsst.so timeout -k 10 300 python -u tools/ns_stamps.py 256 625000 20 32 > gpurun_out/r04d/stamps.txt 2>&1; cat gpurun_out/r04d/stamps.txt
bash tools/gpu_r04_share.sh r04d_share

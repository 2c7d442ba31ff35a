cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof1 gpurun_out/prof2 gpurun_out/prof3
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -- python tools/quick_time.py 512 5000000 8 > gpurun_out/prof1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM --output-format csv -d gpurun_out/prof2 -- python tools/quick_time.py 512 5000000 8 > gpurun_out/prof2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INST_LEVEL_SMEM SQ_INST_CYCLES_SMEM SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof3 -- python tools/quick_time.py 512 5000000 8 > gpurun_out/prof3.log 2>&1

cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof1 gpurun_out/prof2 gpurun_out/prof3; mkdir -p gpurun_out/prof1 gpurun_out/prof2 gpurun_out/prof3
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof1 -- python tools/quick_time.py 512 5000000 8 > gpurun_out/prof1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/prof2 -- python tools/quick_time.py 512 5000000 8 > gpurun_out/prof2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof3 -- python tools/quick_time.py 512 5000000 8 > gpurun_out/prof3.log 2>&1

# PMC passes on the main k-NN kernel (each pass alone, kernel-trace only)
cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmc1 -- python3 tools/quick_time.py 512 5000000 8 > gpurun_out/pmc1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmc2 -- python3 tools/quick_time.py 512 5000000 8 > gpurun_out/pmc2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_VALU_FP64 SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc3 -- python3 tools/quick_time.py 512 5000000 8 > gpurun_out/pmc3.log 2>&1
python3 tools/pmc_summary.py gpurun_out > gpurun_out/pmc_summary.txt 2>&1
cat gpurun_out/pmc_summary.txt

cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_FLAT -d gpurun_out/pmc1 -o p -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INSTS_SALU -d gpurun_out/pmc2 -o p -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc2.log 2>&1
echo EXIT $?

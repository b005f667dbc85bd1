set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --msm 20 --no-prover --inflight 1"
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_conc -o run -- python bench.py --steps 8 --warmup 1 --no-cpu-baseline --msm 16,20,24 > gpurun_out/prof_conc.log 2>&1 && \
export FTZ_SERIAL=1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_serial -o run -- $B > gpurun_out/prof_serial.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o p -- $B > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o p -- $B > gpurun_out/pmc_write.log 2>&1
echo EXIT $?

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
FTZ_SERIAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline --msm= --no-prover --inflight 1 > gpurun_out/prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
tail -1 gpurun_out/prof.log
echo EXIT 0

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo TESTS_FAIL; tail -20 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
timeout -k 10 200 python bench.py --no-cpu-baseline --msm= > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; exit 1; }
tail -1 gpurun_out/bench.log
FTZ_SERIAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline --msm= --no-prover --inflight 1 > gpurun_out/prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo EXIT 0

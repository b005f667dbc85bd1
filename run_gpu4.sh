set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_msm.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/msm_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1
echo EXIT $?

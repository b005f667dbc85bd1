set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 240 python fabric-token-sdk_amd/tools/fpvariants.py libfpm_A.so libfpm_E.so libfpm_F.so > gpurun_out/fpv.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --msm 20 > gpurun_out/bench.log 2>&1
echo EXIT $?

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
echo EXIT $?

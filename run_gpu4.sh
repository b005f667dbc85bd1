set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=fabric-token-sdk_amd/tools/msmtune.py
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof -o run -- python $T 20 "0,0,0" > gpurun_out/prof.log 2>&1
echo EXIT $?

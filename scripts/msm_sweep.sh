#!/bin/bash
# MSM plan sweep (window bits C, slot cap T, slots per segment S) at 2^20 and 2^24
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u fabric-token-sdk_amd/tools/msmtune.py 20 "0,0,0 0,0,4 0,0,16 0,0,32 0,48,0 0,96,0 16,0,0 18,0,0" > gpurun_out/msm20.txt 2>&1 || { tail -5 gpurun_out/msm20.txt; exit 4; }
cat gpurun_out/msm20.txt
timeout -k 10 400 python -u fabric-token-sdk_amd/tools/msmtune.py 24 "0,0,0 0,0,8 0,0,32 0,0,64 20,0,0" > gpurun_out/msm24.txt 2>&1 || { tail -5 gpurun_out/msm24.txt; exit 5; }
cat gpurun_out/msm24.txt

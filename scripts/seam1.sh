cd $GRAFT_REPO_ROOT; export GPU_MAX_HW_QUEUES=16; mkdir -p gpurun_out
FTZ_CALLERS_DEBUG=1 SEAM_SECONDS=1 timeout -k 10 200 python -u fabric-token-sdk_amd/tools/seamsweep.py "" > gpurun_out/seam1.log 2>&1; echo rc=$?; tail -5 gpurun_out/seam1.log

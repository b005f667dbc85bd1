#!/bin/bash
# Prover probe: planning threads sweep (host-bound pass period?).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
mkdir -p gpurun_out
cat /sys/fs/cgroup/cpu.max 2>/dev/null; nproc
for t in 4 8 12 16 24; do
  timeout -k 10 120 python -u fabric-token-sdk_amd/tools/provebench.py --steps 16 --threads $t --no-split >> gpurun_out/prover_threads.log 2>&1 || { echo "provebench $t failed"; tail -20 gpurun_out/prover_threads.log; exit 8; }
done
cat gpurun_out/prover_threads.log

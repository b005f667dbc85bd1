#!/bin/bash
# round 6: request path, request decode threads 16 / 8 / 4 / 12 alternating on one box (tools/reqcpu.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for t in 16 8 4 12; do
    timeout -k 10 300 python3 -u fabric-token-sdk_amd/tools/reqcpu.py --n 100000 --rthreads $t > gpurun_out/rq3_${t}_$r.log 2>&1 || { echo "$t failed"; tail gpurun_out/rq3_${t}_$r.log; exit 3; }
    echo "[rthreads $t round $r]"; tail -4 gpurun_out/rq3_${t}_$r.log
  done
done

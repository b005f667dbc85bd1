#!/bin/bash
# round 6: request path, chunk ramp (first chunks CH/8, CH/4, CH/2) vs variant noramp, alternating on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  timeout -k 10 300 python3 -u fabric-token-sdk_amd/tools/reqcpu.py --n 100000 > gpurun_out/rq4_ramp_$r.log 2>&1 || { echo "ramp failed"; tail gpurun_out/rq4_ramp_$r.log; exit 3; }
  echo "[ramp $r]"; tail -4 gpurun_out/rq4_ramp_$r.log
  timeout -k 10 300 python3 -u fabric-token-sdk_amd/tools/reqcpu.py --n 100000 --lib $PWD/fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_noramp.so > gpurun_out/rq4_noramp_$r.log 2>&1 || { echo "noramp failed"; tail gpurun_out/rq4_noramp_$r.log; exit 4; }
  echo "[noramp $r]"; tail -4 gpurun_out/rq4_noramp_$r.log
done

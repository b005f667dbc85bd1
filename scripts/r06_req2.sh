#!/bin/bash
# round 6: request path A/B on one box: hd = HEAD before the decode changes (host checks),
# new0 = decode changes + host checks, new1 = decode changes + device checks (request_checks=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python3 -u fabric-token-sdk_amd/tools/reqcpu.py --n 100000 --lib $PWD/fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_hd.so > gpurun_out/rq_hd_$r.log 2>&1 || { echo "hd failed"; tail gpurun_out/rq_hd_$r.log; exit 3; }
  echo "[hd $r]"; cat gpurun_out/rq_hd_$r.log
  timeout -k 10 300 python3 -u fabric-token-sdk_amd/tools/reqcpu.py --n 100000 --checks 0 > gpurun_out/rq_n0_$r.log 2>&1 || { echo "n0 failed"; tail gpurun_out/rq_n0_$r.log; exit 4; }
  echo "[new0 $r]"; cat gpurun_out/rq_n0_$r.log
  timeout -k 10 300 python3 -u fabric-token-sdk_amd/tools/reqcpu.py --n 100000 --checks 1 > gpurun_out/rq_n1_$r.log 2>&1 || { echo "n1 failed"; tail gpurun_out/rq_n1_$r.log; exit 5; }
  echo "[new1 $r]"; cat gpurun_out/rq_n1_$r.log
done

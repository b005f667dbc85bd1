#!/bin/bash
# round 6: request path, decode-ahead thread (phase A of chunk k+1 beside phase B of chunk k) vs variant seq (FTS_REQ_AHEAD=0), alternating on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  timeout -k 10 300 python3 -u fabric-token-sdk_amd/tools/reqcpu.py --n 100000 > gpurun_out/rq5_ramp_$r.log 2>&1 || { echo "ahead failed"; tail gpurun_out/rq5_ramp_$r.log; exit 3; }
  echo "[ahead $r]"; tail -4 gpurun_out/rq5_ramp_$r.log
  timeout -k 10 300 python3 -u fabric-token-sdk_amd/tools/reqcpu.py --n 100000 --lib $PWD/fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_seq.so > gpurun_out/rq5_seq_$r.log 2>&1 || { echo "seq failed"; tail gpurun_out/rq5_seq_$r.log; exit 4; }
  echo "[seq $r]"; tail -4 gpurun_out/rq5_seq_$r.log
done

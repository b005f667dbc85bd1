#!/bin/bash
# round 6: host Montgomery products in 4 x 64-bit limbs (FTS_HOST64) -- GPU tests
# of every path with host field work, then the request path A/B against the
# 8 x 32-bit host build (variant h32)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_requests.py tests/test_idemix_bn254.py tests/test_idemix.py tests/test_msm.py tests/test_gpu.py tests/test_abi.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06e_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06e_tests.log; exit 3; }
echo tests ok
for r in 1 2; do
  for v in new h32; do
    if [ $v = new ]; then lib=""; else lib="--lib fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_h32.so"; fi
    timeout -k 10 240 python -u fabric-token-sdk_amd/tools/reqbench.py --n 100000 $lib > gpurun_out/r06e_req_${v}_$r.log 2>&1 || { echo "reqbench $v failed"; tail -20 gpurun_out/r06e_req_${v}_$r.log; exit 4; }
    echo "[$v $r]"; tail -1 gpurun_out/r06e_req_${v}_$r.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); b=d['batched_get_states']
print(' batched', b['transfers_per_s'], b['verdicts_bit_exact'], b['calling_thread_ms'], 'per_key', d['per_key_get_state']['transfers_per_s'])"
  done
done
echo all ok

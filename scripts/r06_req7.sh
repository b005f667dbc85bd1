#!/bin/bash
# round 6: request pipeline shape in bench.requests_leg: default (4096-request chunks, 8 in flight, ramp /8)
# vs 2048 / 8192 chunks, ramp /16, 4 in flight; alternating, 2 rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in default c2k c8k r16 if4; do
    lib=""; [ $v != default ] && lib="--lib $PWD/fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_$v.so"
    timeout -k 10 300 python3 -u fabric-token-sdk_amd/tools/reqbench.py --n 100000 $lib > gpurun_out/rq7_${v}_$r.log 2>&1 || { echo "$v failed"; tail gpurun_out/rq7_${v}_$r.log; exit 3; }
    echo "[$v $r] $(python3 -c "import json; d=json.loads(open('gpurun_out/rq7_${v}_$r.log').read().strip().splitlines()[-1]); print(d['batched_get_states']['transfers_per_s'], d['per_key_get_state']['transfers_per_s'])")"
  done
done

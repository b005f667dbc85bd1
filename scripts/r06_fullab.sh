#!/bin/bash
# round 6: the full default bench (every leg) alternating between the final tree and the same tree with the
# round-6 request-path host changes reverted (variant oldreq): the token_requests leg across boxes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in new oldreq; do
    lib=""; [ $v = oldreq ] && lib="--lib $PWD/fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_oldreq.so"
    timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 $lib --detail-out gpurun_out/fab_${v}_$r.json > gpurun_out/fab_${v}_$r.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/fab_${v}_$r.log; exit 5; }
    python3 -c "
import json
d=json.load(open('gpurun_out/fab_${v}_$r.json')); t=d['token_requests']
print('[$v $r] value', d['value'], 'req batched', t['batched_get_states']['transfers_per_s'], 'per_key', t['per_key_get_state']['transfers_per_s'], 'ratio', t['vs_verify_transfers'], t['batched_get_states']['calling_thread_ms'])
"
  done
done

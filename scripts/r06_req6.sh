#!/bin/bash
# round 6: the bench's own request leg (tools/reqbench.py = bench.requests_leg), ramp vs noramp, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3 4; do
  timeout -k 10 300 python3 -u fabric-token-sdk_amd/tools/reqbench.py --n 100000 > gpurun_out/rq6_ramp_$r.log 2>&1 || { echo "ramp failed"; tail gpurun_out/rq6_ramp_$r.log; exit 3; }
  echo "[ramp $r] $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/rq6_ramp_$r.log').read().strip().splitlines()[-1]); print(d['batched_get_states']['transfers_per_s'], d['per_key_get_state']['transfers_per_s'])")"
  timeout -k 10 300 python3 -u fabric-token-sdk_amd/tools/reqbench.py --n 100000 --lib $PWD/fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_noramp.so > gpurun_out/rq6_noramp_$r.log 2>&1 || { echo "noramp failed"; tail gpurun_out/rq6_noramp_$r.log; exit 4; }
  echo "[noramp $r] $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/rq6_noramp_$r.log').read().strip().splitlines()[-1]); print(d['batched_get_states']['transfers_per_s'], d['per_key_get_state']['transfers_per_s'])")"
done

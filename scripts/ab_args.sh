#!/bin/bash
# A/B runs of the headline bench over argument sets, one bench per set, each
# with its own time limit; stops at the first failure.
#   AB="--batch 4096|--batch 8192 --slots 3" bash scripts/ab_args.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
BASE=${BASE_ARGS:---steps 20 --warmup 2 --no-cpu-baseline --no-prover --msm 20}
IFS='|' read -ra SETS <<< "${AB:-}"
i=0
for s in "${SETS[@]}"; do
  i=$((i + 1))
  timeout -k 10 300 python -u bench.py $BASE $s > gpurun_out/aa$i.log 2>&1 || { echo "[$s] bench failed"; tail -30 gpurun_out/aa$i.log; exit 4; }
  echo "[$s]"
  tail -1 gpurun_out/aa$i.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
r=d.get('roofline') or {}
e=d.get('engine') or {}
print(' value', d['value'], 'ms/step', d['ms_per_step'], 'exact', d.get('verdicts_bit_exact'), 'plan ms', e.get('host_plan_ms_per_batch'))
print(' serial', r.get('serial_ms'))
print(' frac', r.get('per_kernel_frac'))
print(' device_only', (d.get('device_only') or {}).get('transfers_per_s'))
"
done

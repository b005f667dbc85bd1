#!/bin/bash
# Sweep of (environment, bench arguments) pairs, one bench per pair and round,
# each under its own time limit; prints value / device-only / engine stats.
#   SETS="GPU_MAX_HW_QUEUES=4;--threads 8|GPU_MAX_HW_QUEUES=12;--slots 6" ROUNDS=2 bash scripts/sweep_env_args.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
BASE=${BASE_ARGS:---steps 256 --warmup 3 --no-cpu-baseline --no-prover --msm= --no-seam --no-ppb}
IFS='|' read -ra SETS <<< "${SETS:-}"
for r in $(seq 1 "${ROUNDS:-1}"); do
  i=0
  for s in "${SETS[@]}"; do
    i=$((i + 1))
    envs=${s%%;*}
    args=${s#*;}
    log=gpurun_out/sweep_${i}_$r.log
    env $envs timeout -k 10 300 python -u bench.py $BASE $args > $log 2>&1 || { echo "[$s] bench failed"; tail -30 $log; exit 4; }
    tail -1 $log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
e=d['engine']
print('[%s] r%s value %.0f dev_only %.0f plan %.2f submit %.2f dev %.1f q %s' % ('$s', '$r', d['value'],
      (d.get('device_only') or {}).get('transfers_per_s', 0), e['host_plan_ms_per_batch'], e['enqueue_ms_per_batch'],
      e['device_ms_per_batch'], e['hw_queues']))
"
  done
done

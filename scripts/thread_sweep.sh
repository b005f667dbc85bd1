#!/bin/bash
# e2e headline vs host planning threads and slots (one box, one session)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/sweep.txt
for cfg in "16 4" "8 4" "12 4" "6 4" "12 6" "8 6"; do
  set -- $cfg
  timeout -k 10 240 python -u bench.py --steps 40 --no-extras --no-prover --msm "" --no-cpu-baseline --threads $1 --slots $2 > gpurun_out/sw.log 2>&1 || { echo "run $cfg failed"; tail -5 gpurun_out/sw.log; exit 4; }
  grep '^{' gpurun_out/sw.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['engine']; print('threads $1 slots $2', d['value'], 'plan', e['host_plan_ms_per_batch'], 'dev', e['device_ms_per_batch'], 'inflight', e['max_in_flight'])" | tee -a gpurun_out/sweep.txt
done

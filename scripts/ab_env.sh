#!/bin/bash
# A/B runs of the headline bench under environment settings, one bench per
# setting, each with its own time limit; stops at the first failure.
#   AB="FTZ_X=0|FTZ_X=1" BENCH_ARGS="..." TESTS="tests/test_gpu.py" bash scripts/ab_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:---steps 20 --warmup 2 --no-cpu-baseline --no-prover --msm 20}
IFS='|' read -ra SETS <<< "${AB:-}"
i=0
for s in "${SETS[@]}"; do
  i=$((i + 1))
  if [ -n "${TESTS:-}" ]; then
    env $s timeout -k 10 300 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/ab$i.test.log 2>&1 || { echo "[$s] tests failed"; tail -30 gpurun_out/ab$i.test.log; exit 3; }
    echo "[$s] $(tail -1 gpurun_out/ab$i.test.log)"
  fi
  env $s timeout -k 10 300 python -u bench.py $ARGS > gpurun_out/ab$i.log 2>&1 || { echo "[$s] bench failed"; tail -30 gpurun_out/ab$i.log; exit 4; }
  echo "[$s]"
  tail -1 gpurun_out/ab$i.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
r=d.get('roofline') or {}
print(' value', d['value'], 'ms/step', d['ms_per_step'], 'exact', d.get('verdicts_bit_exact'))
print(' serial', r.get('serial_ms'))
print(' frac', r.get('per_kernel_frac'))
print(' device_only', (d.get('device_only') or {}).get('transfers_per_s'), 'msm20', d.get('msm_2^20_latency_ms'))
"
done

#!/bin/bash
# Same-box A/B of library builds (fabric-token-sdk_amd/build.py --variant):
# ROUNDS alternating passes over LIBS ("name=path|name=path", path relative to
# the repo; "default" = the in-tree library), one bench per (round, library),
# each under its own time limit; stops at the first failure.
#   LIBS="kara=default|sb=fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_sb.so" ROUNDS=3 bash scripts/ab_lib.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:---steps 64 --warmup 2 --no-cpu-baseline --no-prover --msm= --no-seam --no-ppb}
IFS='|' read -ra SETS <<< "${LIBS:-}"
for r in $(seq 1 "${ROUNDS:-2}"); do
  for s in "${SETS[@]}"; do
    name=${s%%=*}
    path=${s#*=}
    if [ "$path" = "default" ]; then lib=""; else lib="--lib $PWD/$path"; fi
    log=gpurun_out/ablib_${name}_$r.log
    timeout -k 10 300 python -u bench.py $ARGS $lib > $log 2>&1 || { echo "[$name] bench failed"; tail -30 $log; exit 4; }
    echo "[$name round $r]"
    tail -1 $log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
r=d.get('roofline') or {}
print(' value', d['value'], 'ms/step', d['ms_per_step'], 'exact', d.get('verdicts_bit_exact'))
print(' serial', r.get('serial_ms'))
print(' frac', r.get('per_kernel_frac'))
print(' device_only', (d.get('device_only') or {}).get('transfers_per_s'))
"
  done
done

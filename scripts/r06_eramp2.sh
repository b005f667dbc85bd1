#!/bin/bash
# round 6: engine ramp after an idle engine only (variant ramp2: first_pass 1024 / 2048, doubling to the batch)
# vs the default (first pass 4096); bench.py --steps 20 --warmup 5, legs off, 3 alternating rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-prover --msm= --no-seam --no-ppb"
L="--lib $PWD/fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_ramp2.so"
for r in 1 2 3 4; do
  for v in default r2_1024; do
    case $v in
      default) x="";;
      r2_1024) x="$L --opt first_pass=1024";;
      r2_2048) x="$L --opt first_pass=2048";;
    esac
    timeout -k 10 300 python -u bench.py $ARGS $x > gpurun_out/er2_${v}_$r.log 2>&1 || { echo "$v failed"; tail -20 gpurun_out/er2_${v}_$r.log; exit 4; }
    echo "[$v $r] $(tail -1 gpurun_out/er2_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], (d.get('device_only') or {}).get('transfers_per_s'))")"
  done
done

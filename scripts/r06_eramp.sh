#!/bin/bash
# round 6: engine pass ramp (first passes fp1, 2 fp1, 4 fp1 ... while few are in flight) vs the round-5 first pass
# (variant noramp: only the first pass is 4096); bench.py --steps 20 --warmup 5, legs off, 3 alternating rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-prover --msm= --no-seam --no-ppb"
for r in 1 2 3; do
  for v in r1024 r2048 noramp; do
    case $v in
      r1024) x="--opt first_pass=1024";;
      r2048) x="--opt first_pass=2048";;
      noramp) x="--lib $PWD/fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_noramp.so";;
    esac
    timeout -k 10 300 python -u bench.py $ARGS $x > gpurun_out/er_${v}_$r.log 2>&1 || { echo "$v failed"; tail -20 gpurun_out/er_${v}_$r.log; exit 4; }
    echo "[$v $r] $(tail -1 gpurun_out/er_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], (d.get('device_only') or {}).get('transfers_per_s'))")"
  done
done

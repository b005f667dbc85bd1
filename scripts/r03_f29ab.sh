#!/bin/bash
# A/B of the f29 product form: operand scanning (in-tree build) vs product
# scanning (_lib/ab/libftsamd_ps.so): MSM 2^20 / 2^24 + bench headline, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=fabric-token-sdk_amd/zkatdlog/_lib
cp $L/libftsamd.so $L/ab/libftsamd_os.so
Q="--steps 64 --warmup 3 --no-extras --no-cpu-baseline --msm=20,24 --no-prover"
for v in os ps os ps; do
  cp $L/ab/libftsamd_$v.so $L/libftsamd.so
  timeout -k 10 240 python -u bench.py $Q > gpurun_out/f29ab_$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/f29ab_$v.log; cp $L/ab/libftsamd_os.so $L/libftsamd.so; exit 5; }
  python3 - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = [json.loads(l) for l in open("gpurun_out/f29ab_%s.log" % v) if l.startswith("{")][-1]
print(v, "value", d["value"], "msm", [(m["n"], m["device_ms"]) for m in d["msm"]], flush=True)
PY
done
cp $L/ab/libftsamd_os.so $L/libftsamd.so
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f29 -o k -- python3 fabric-token-sdk_amd/tools/msmtune.py 20 "0,0,0" > gpurun_out/prof_f29.log 2>&1 || { echo "trace failed"; exit 6; }
echo "trace ok"

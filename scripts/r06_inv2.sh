#!/bin/bash
# round 6: divsteps inversion on 30-bit limbs (default) vs 62-bit limbs (variant sg62): device check,
# one lane's latency, GPU tests, bench A/B with the seam leg
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 -u fabric-token-sdk_amd/tools/invbench.py > gpurun_out/r06i2_bench.log 2>&1 || { echo "invbench failed"; cat gpurun_out/r06i2_bench.log; exit 3; }
cat gpurun_out/r06i2_bench.log
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_engine.py tests/test_msm.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06i2_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06i2_tests.log; exit 4; }
tail -1 gpurun_out/r06i2_tests.log
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-prover --msm=20 --no-ppb"
for r in 1 2; do
  for v in sg30 sg62; do
    lib=""; [ $v = sg62 ] && lib="--lib $PWD/fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_sg62.so"
    timeout -k 10 400 python -u bench.py $ARGS $lib --detail-out gpurun_out/r06i2_${v}_$r.json > gpurun_out/r06i2_${v}_$r.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/r06i2_${v}_$r.log; exit 5; }
    python3 -c "
import json
d=json.load(open('gpurun_out/r06i2_${v}_$r.json'))
s=d.get('seam') or {}
print('[$v $r] value', d['value'], 'device_only', (d.get('device_only') or {}).get('transfers_per_s'), 'n1_ms', (s.get('call_latency_ms_by_size') or {}).get('1'), 'serial', (d.get('roofline') or {}).get('serial_ms'))
"
  done
done

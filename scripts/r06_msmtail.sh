#!/bin/bash
# round 6: MSM tail A/B: new (host Horner, quad tree, quad segments) vs qt (one-lane
# segments) and old (device Horner, one-lane tree and segments); kernel timeline of new
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_msm.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06t_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06t_tests.log; exit 4; }
echo tests ok
for r in 1 2; do
  for lg in 16 20 24; do
    for v in new qt old; do
      lib=""; [ $v != new ] && lib=fabric-token-sdk_amd/zkatdlog/_lib/ab/libftsamd_$v.so
      timeout -k 10 200 python -u fabric-token-sdk_amd/tools/msmtune.py $lg "0,0,0,0,0,0" $lib > gpurun_out/r06t_one.log 2>&1 || { echo "msmtune $v $lg failed"; cat gpurun_out/r06t_one.log; exit 5; }
      echo "$v $(grep n=2 gpurun_out/r06t_one.log)" | tee -a gpurun_out/r06t_msm.log
    done
  done
done
for lg in 16 20; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mts$lg -o k -- python3 fabric-token-sdk_amd/tools/msmtune.py $lg "0,0,0,0,0,0" > gpurun_out/mts$lg.log 2>&1 || { echo "trace $lg failed"; tail gpurun_out/mts$lg.log; exit 3; }
  f=$(find gpurun_out/mts$lg -name '*kernel_trace.csv' | head -1)
  python3 fabric-token-sdk_amd/tools/ktrace.py $f 16 > gpurun_out/mts${lg}_timeline.txt
  cat gpurun_out/mts${lg}_timeline.txt
done

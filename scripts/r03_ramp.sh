#!/bin/bash
# Pass-ramp A/B at the driver's bench shape (--steps 20 --warmup 5), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
Q="--steps 20 --warmup 5 --no-extras --no-cpu-baseline --msm= --no-prover"
for r in 0 1 0 1; do
  timeout -k 10 200 python -u bench.py $Q --ramp $r > gpurun_out/ramp_$r.log 2>&1 || { echo "bench ramp $r failed"; tail -20 gpurun_out/ramp_$r.log; exit 5; }
  echo "ramp $r: $(grep -o '"value": [0-9.]*' gpurun_out/ramp_$r.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ramp_$r.log) $(grep -o '"batches": [0-9]*' gpurun_out/ramp_$r.log)"
done
for r in 0 1; do
  timeout -k 10 300 python -u bench.py --steps 256 --warmup 3 --no-extras --no-cpu-baseline --msm= --no-prover --ramp $r > gpurun_out/ramp256_$r.log 2>&1 || { echo "bench256 ramp $r failed"; exit 5; }
  echo "256 steps ramp $r: $(grep -o '"value": [0-9.]*' gpurun_out/ramp256_$r.log)"
done

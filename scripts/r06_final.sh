#!/bin/bash
# round 6 final tree: GPU suite, smoke, driver-like bench (one box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06m_gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r06m_gputest.log; exit 3; }
tail -3 gpurun_out/r06m_gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06m_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r06m_smoke.log; exit 4; }
tail -2 gpurun_out/r06m_smoke.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 --detail-out gpurun_out/r06m_bench_detail.json > gpurun_out/r06m_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r06m_bench.log; exit 5; }
tail -1 gpurun_out/r06m_bench.log | cut -c1-400

#!/bin/bash
# round 6, last tree: GPU suite and smoke (one box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06l_gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r06l_gputest.log; exit 3; }
tail -1 gpurun_out/r06l_gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06l_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r06l_smoke.log; exit 4; }
tail -1 gpurun_out/r06l_smoke.log

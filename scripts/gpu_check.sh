#!/bin/bash
# One GPU-box session: GPU tests, smoke, a short bench.  Each GPU step has its
# own time limit; a crash / abort / timeout (exit >= 2 from pytest, or any
# non-zero from the others) ends the session there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
rc=0
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -v --timeout 300 --timeout-method thread -rP \
    > gpurun_out/gputest.log 2>&1
  rc=$?
  tail -5 gpurun_out/gputest.log
  if [ $rc -ge 2 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
fi
if [ "${SMOKE:-1}" = 1 ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 4; }
  tail -2 gpurun_out/smoke.log
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 5; }
  tail -c 3000 gpurun_out/bench.log
fi
exit $rc

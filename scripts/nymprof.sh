#!/bin/bash
# idemix owner-signature leg: GPU tests, the bench leg alone, and its rocprofv3 kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/nymprof
timeout -k 10 300 python -u -m pytest tests/test_idemix.py -m gpu -q -s --timeout 120 --timeout-method thread > gpurun_out/nymprof/test.log 2>&1 || { tail -30 gpurun_out/nymprof/test.log; exit 4; }
tail -3 gpurun_out/nymprof/test.log
cat > /tmp/nymleg.py <<'PY'
import json, os, sys
sys.path.insert(0, os.path.join(os.getcwd(), "fabric-token-sdk_amd")); sys.path.insert(0, os.getcwd())
import bench, zkatdlog
g = json.load(open("tests/golden/zkatdlog_golden.json"))["pp_a"]
ctx = zkatdlog.Context(g["pp"].encode(), device=0)
print(json.dumps(bench.owner_signatures(ctx)), flush=True)
ctx.close()
PY
timeout -k 10 300 python -u /tmp/nymleg.py > gpurun_out/nymprof/leg.log 2>&1 || { tail -30 gpurun_out/nymprof/leg.log; exit 5; }
cat gpurun_out/nymprof/leg.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/nymprof/trace -o k -- python3 /tmp/nymleg.py > gpurun_out/nymprof/trace.log 2>&1 || { tail -20 gpurun_out/nymprof/trace.log; exit 6; }
f=$(find gpurun_out/nymprof/trace -name "*kernel_stats.csv" | head -1)
head -8 "$f"

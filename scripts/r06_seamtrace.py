#!/usr/bin/env python3
"""One n = 1 ftz_verify_transfers call, repeated (the drop-in seam): run under
rocprofv3 --kernel-trace to see the call's kernel chain (tools/ktrace.py)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))
import zkatdlog  # noqa: E402
from zkatdlog import workload as W  # noqa: E402

g = json.load(open(os.path.join(ROOT, "tests", "golden", "zkatdlog_golden.json")))["pp_a"]
ctx = zkatdlog.Context(g["pp"].encode(), device=0)
valid = W.prove_distinct(ctx, 64, tag=b"seam-trace")
job = W.mixed_job(valid, None, 1)
calls = []
for _ in range(30):
    t0 = time.perf_counter()
    ctx.verify_transfers_packed(job.ptr(), job.n)
    calls.append((time.perf_counter() - t0) * 1e3)
time.sleep(0.05)
t0 = time.perf_counter()
ctx.verify_transfers_packed(job.ptr(), job.n)
print("last call ms %.3f (median of 30: %.3f)" % ((time.perf_counter() - t0) * 1e3, sorted(calls)[15]), flush=True)
ctx.close()

#!/usr/bin/env python3
"""Where the time of a small device pass goes (the drop-in seam, one transfer
per call): per-stage device time (HIP events, ftz_batch_stats) of a staged
pass of n transfers, serial (every kernel on one stream) and as scheduled,
plus the wall time of one ftz_batch_run and of one ftz_verify_transfers call.
    python scripts/seam_probe.py [n ...]
SEAM_LAYOUT=one_lane|sextet forces the t' + lines stage's layout (default: the
engine's choice, sextet for small passes)."""
import json
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "12")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))
import zkatdlog  # noqa: E402
from zkatdlog import workload as W  # noqa: E402

g = json.load(open(os.path.join(ROOT, "tests", "golden", "zkatdlog_golden.json")))["pp_a"]
ctx = zkatdlog.Context(g["pp"].encode(), device=0)
if os.environ.get("SEAM_LAYOUT"):
    ctx.set_layout("g2lines", os.environ["SEAM_LAYOUT"])
valid = W.prove_distinct(ctx, 256, tag=b"seam-probe")
for n in [int(a) for a in sys.argv[1:]] or [1, 16, 64]:
    job = W.mixed_job(valid, None, n)
    for serial in (True, False):
        b = ctx.load_packed(job.ptr(), job.n)
        ctx.set_serial(serial)
        b.run()
        walls = []
        for _ in range(20):
            t0 = time.perf_counter()
            b.run()
            walls.append((time.perf_counter() - t0) * 1e3)
        st = b.stats()
        b.close()
        walls.sort()
        print(json.dumps({"n": n, "serial": serial, "batch_run_ms": round(walls[10], 3),
                          "stage_ms": {k: round(v[0], 3) for k, v in st.items() if v[0] > 0.001}}), flush=True)
    ctx.set_serial(False)
    calls = []
    for _ in range(20):
        t0 = time.perf_counter()
        ctx.verify_transfers_packed(job.ptr(), job.n)
        calls.append((time.perf_counter() - t0) * 1e3)
    calls.sort()
    print(json.dumps({"n": n, "verify_call_ms": round(calls[10], 3)}), flush=True)
ctx.close()

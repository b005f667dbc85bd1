#!/usr/bin/env python3
"""Probe: serial per-kernel times of one staged 4096-transfer batch, repeated
across fresh loads (allocation placement) -- diagnostic for kernel-time
variance between runs.  Prints one line per probe."""
import os
import sys
import time

if True:  # as bench.py: 12 (16 oversubscribes the hardware scheduler with two contexts)
    os.environ["GPU_MAX_HW_QUEUES"] = "12"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))
import json  # noqa: E402

import zkatdlog  # noqa: E402
from zkatdlog import workload as W  # noqa: E402

g = json.load(open(os.path.join(ROOT, "tests", "golden", "zkatdlog_golden.json")))["pp_a"]
ctx = zkatdlog.Context(g["pp"].encode(), device=0)
valid = W.prove_distinct(ctx, 4096, tag=b"probe")
job = W.mixed_job(valid, None, 4096)
keep = []
big = W.mixed_job(valid, None, 40 * 4096)


def run_engine():
    t0 = time.time()
    ctx.verify_transfers_packed(big.ptr(), big.n)
    print("engine run %.3f s" % (time.time() - t0), flush=True)


for probe in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    if probe == 2:
        run_engine()
    if probe == 4:
        for _ in range(4):
            ctx.load_packed(job.ptr(), job.n).close()
    b = ctx.load_packed(job.ptr(), job.n)
    ctx.set_serial(True)
    b.run()
    acc = {}
    for _ in range(3):
        b.run()
        for k, v in b.stats().items():
            acc[k] = acc.get(k, 0) + v[0] / 3
    ctx.set_serial(False)
    print("probe %d: " % probe + " ".join("%s=%.3f" % (k, v) for k, v in acc.items()), flush=True)
    if probe % 2:
        b.close()
    else:
        keep.append(b)

#!/usr/bin/env python3
"""Drop-in seam sweep: bench.seam_leg (one-call latency by size, closed-loop
n=1 callers) under several job-engine option sets (ftz_options hold_inflight /
small_pass / window_us / slots), one JSON line per set.

    python fabric-token-sdk_amd/tools/seamsweep.py "hold_inflight=2" "small_pass=4096" ...
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))
import bench  # noqa: E402
import zkatdlog  # noqa: E402
from zkatdlog import workload as W  # noqa: E402

g = json.load(open(os.path.join(ROOT, "tests", "golden", "zkatdlog_golden.json")))["pp_a"]
pp = g["pp"].encode()
ctx = zkatdlog.Context(pp, device=0)
valid = W.prove_distinct(ctx, 16384, tag=b"seam")
bad = W.golden_tampered()
ctx.close()
for spec in sys.argv[1:]:
    opts = {k: int(v) for k, v in (kv.split("=") for kv in spec.split(",") if kv)}
    r = bench.seam_leg(pp, 0, valid, bad, seconds=float(os.environ.get("SEAM_SECONDS", "2")), **opts)
    print(json.dumps({"spec": spec, **r}), flush=True)

#!/usr/bin/env python3
"""Batch prover alone (bench.py's prover leg in a fresh process, nothing else
on the device): steps x 4096 2-in/2-out PP-A transfer proofs, one
ftz_prove_transfers call, every proof re-verified.  With --serial every kernel
of a prover pass runs on one stream (per-kernel durations under rocprofv3).
    python fabric-token-sdk_amd/tools/provebench.py --steps 16
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))

import bench  # noqa: E402  (sets GPU_MAX_HW_QUEUES before HIP starts)

import zkatdlog  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--serial", action="store_true")
    a = ap.parse_args()
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "zkatdlog_golden.json")))["pp_a"]
    with zkatdlog.Context(g["pp"].encode(), device=0) as ctx:
        if a.serial:
            ctx.set_serial(True)
        bench.prover_bench(ctx, 4096, 1)  # warm-up: slots and tables
        print(json.dumps(bench.prover_bench(ctx, 4096, a.steps)), flush=True)


if __name__ == "__main__":
    main()

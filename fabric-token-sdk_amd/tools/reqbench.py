#!/usr/bin/env python3
"""Block-level request path on one GPU (bench.py requests_leg alone), with the
pipeline's per-stage calling-thread times and the engine's pass counters, for
several context settings.
    python fabric-token-sdk_amd/tools/reqbench.py --n 100000 --threads 16,32
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100000)
    ap.add_argument("--threads", default="16")
    ap.add_argument("--slots", default="4")
    ap.add_argument("--lib", default=None, help="A/B: a variant build (build.py --variant)")
    a = ap.parse_args()
    import bench
    import zkatdlog
    if a.lib:
        zkatdlog._abi.use_library(a.lib)
    from zkatdlog import workload as W
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "zkatdlog_golden.json")))["pp_a"]
    for th in [int(x) for x in a.threads.split(",")]:
        for sl in [int(x) for x in a.slots.split(",")]:
            with zkatdlog.Context(g["pp"].encode(), device=0, threads=th, slots=sl) as ctx:
                valid = W.prove_distinct(ctx, 16384, tag=b"reqbench")
                out = bench.requests_leg(ctx, valid, n_req=a.n)
                out["threads"], out["slots"] = th, sl
                print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""The PP-B (configs[0]: b = 16, e = 16, 64-bit values) verify / prove leg of
bench.py alone, for profiling (rocprofv3 --kernel-trace --stats -- python3
fabric-token-sdk_amd/tools/ppbleg.py).  Prints the leg's JSON."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--device-batch", type=int, default=None)
    a = ap.parse_args()
    import bench
    from zkatdlog import workload as W

    class Args:
        pass
    args = Args()
    args.device_batch = a.device_batch
    out, _ = bench.ppb_leg(0, args, W.golden_tampered("pp_b"))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

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
    ap.add_argument("--threads", type=int, default=None, help="host planning threads (ftz_options.threads)")
    ap.add_argument("--slots", type=int, default=None, help="passes in flight (ftz_options.slots)")
    ap.add_argument("--layout", default=None, help="prover t' / line stage layout: one_lane | sextet")
    ap.add_argument("--batch", type=int, default=None, help="proofs per device pass (ftz_options.batch)")
    ap.add_argument("--no-split", action="store_true")
    a = ap.parse_args()
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "zkatdlog_golden.json")))["pp_a"]
    import time

    from zkatdlog import workload as W
    with zkatdlog.Context(g["pp"].encode(), device=0, threads=a.threads, slots=a.slots, batch=a.batch) as ctx:
        if a.serial:
            ctx.set_serial(True)
        if a.layout:
            ctx.set_layout("prover_g2lines", a.layout)
        bench.prover_bench(ctx, 4096, 2)  # warm-up: slots and tables
        ctx.prover_stats(reset=True)
        r = bench.prover_bench(ctx, 4096, a.steps)
        r["pass_proofs"] = min(ctx.options["batch"], 4096)
        r["threads"] = ctx.options["threads"]
        r["slots"] = ctx.options["slots"]
        r["layout"] = a.layout or "default"
        print(json.dumps(r), flush=True)
        if a.no_split:
            return
        # one staged pass: host planning + upload (ftz_prover_load) apart from the
        # device run (ftz_prover_run)
        bases, sd = W.witness_bases(), W.seeds(4096, b"split")
        ws = [dict(bases[i % len(bases)], seed=sd[32 * i:32 * i + 32]) for i in range(4096)]
        import ctypes

        from zkatdlog import _abi as A
        arr, keep = A.pack_transfer_witnesses(ws)
        lib = ctx._lib
        for rep in range(3):
            h = ctypes.c_void_p()
            t0 = time.perf_counter()
            assert lib.ftz_prover_load_transfers(ctx._h, len(ws), arr, ctypes.byref(h)) == 0
            t1 = time.perf_counter()
            assert lib.ftz_prover_run(h) == 0
            t2 = time.perf_counter()
            assert lib.ftz_prover_run(h) == 0
            t3 = time.perf_counter()
            st = A.Stats()
            assert lib.ftz_prover_stats(h, ctypes.byref(st)) == 0
            lib.ftz_prover_destroy(h)
            stage_ms = {name: round(st.ms[k], 3) for k, name in enumerate(A.PROVER_STAGE_NAMES)}
            print(json.dumps({"plan_upload_ms": round((t1 - t0) * 1e3, 3), "run_ms": round((t2 - t1) * 1e3, 3),
                              "rerun_ms": round((t3 - t2) * 1e3, 3), "stage_ms": stage_ms}), flush=True)


if __name__ == "__main__":
    main()

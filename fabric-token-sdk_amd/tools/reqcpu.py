#!/usr/bin/env python3
"""Host CPU seconds (getrusage, all threads) of the block-level request path
against plain ftz_verify_transfers over the same proofs: is the request path
bound by the host's cores?
    python fabric-token-sdk_amd/tools/reqcpu.py --n 100000 [--lib variant.so]"""
import argparse
import ctypes
import json
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))


def cpu():
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime + r.ru_stime


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--rthreads", type=int, default=None, help="ftz_options.request_threads")
    a = ap.parse_args()
    import numpy as np
    import zkatdlog
    if a.lib:
        zkatdlog._abi.use_library(a.lib)
    from zkatdlog import workload as W
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "zkatdlog_golden.json")))["pp_a"]
    i32 = ctypes.POINTER(ctypes.c_int32)
    opts = {} if a.rthreads is None else {"request_threads": a.rthreads}
    with zkatdlog.Context(g["pp"].encode(), device=0, threads=a.threads, **opts) as ctx:
        valid = W.prove_distinct(ctx, 16384, tag=b"reqcpu")
        rs = W.RequestSet(valid, a.n, per=2)
        led = zkatdlog.NativeLedger(rs.ledger)
        codes = np.zeros(a.n, dtype=np.int32)
        failed = np.zeros(a.n, dtype=np.int32)
        job = W.mixed_job(valid, None, 2 * a.n, rate=0)
        for rep in range(3):
            c0, t0 = cpu(), time.perf_counter()
            ctx.verify_token_requests_packed(rs.ptr(), a.n, led, codes.ctypes.data_as(i32),
                                             failed.ctypes.data_as(i32), batched=True)
            dt, dc = time.perf_counter() - t0, cpu() - c0
            st = ctx.request_stats(reset=True)
            print("requests  %7.1f k transfers/s  wall %.3f s  cpu %.2f s  cores %.1f  %s" % (
                2 * a.n / dt / 1e3, dt, dc, dc / dt, json.dumps(st)), flush=True)
            c0, t0 = cpu(), time.perf_counter()
            tc = ctx.verify_transfers_packed(job.ptr(), job.n)
            dt, dc = time.perf_counter() - t0, cpu() - c0
            assert (tc == 0).all()
            if True:
                print("transfers %7.1f k transfers/s  wall %.3f s  cpu %.2f s  cores %.1f" % (
                    2 * a.n / dt / 1e3, dt, dc, dc / dt), flush=True)
        led.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""MSM plan sweep: device latency of ftz_msm_run for window bits C, slot cap T,
slots per segment S, resident-point mode P and sort digit bits R (ftz_options
msm_window_bits / msm_slot_cap / msm_seg_slots / msm_precompute /
msm_radix_bits; 0 = the planner's choice / off) and graph replay G
(ftz_options.msm_graph, default 1).
    python msmtune.py 20 "0,0,0 16,16,0 16,32,0 15,0,0 17,0,0,1 0,0,0,0,8" [variant.so]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))
import numpy as np  # noqa: E402

import zkatdlog  # noqa: E402

if len(sys.argv) > 3:  # A/B: a variant build (build.py --variant)
    zkatdlog._abi.use_library(sys.argv[3])

lg = int(sys.argv[1])
combos = [tuple(int(v) for v in (c + ",0,0,0,0,1"[len(c.split(",")) * 2 - 2:]).split(",")[:6])
          for c in sys.argv[2].split()]
pp = json.load(open(os.path.join(ROOT, "tests", "golden", "zkatdlog_golden.json")))["pp_a"]["pp"].encode()
scal = np.random.default_rng(lg).bytes(32 << lg)
ref = None
import time  # noqa: E402
for c, t, s, pre, rb, gr in combos:
    ctx = zkatdlog.Context(pp, device=0, msm_window_bits=c, msm_slot_cap=t, msm_seg_slots=s, msm_precompute=pre,
                           msm_radix_bits=rb, msm_graph=gr)
    t0 = time.perf_counter()
    m = zkatdlog.Msm(ctx, scalars=scal, gen_offset=1)
    load_s = time.perf_counter() - t0
    out = m.run()
    ms = []
    for _ in range(4):
        assert m.run() == out
        ms.append(m.info()["last_ms"])
    ref = ref or out
    print("n=2^%d C=%2d T=%3d S=%3d P=%d R=%d G=%d  %8.3f ms  load %.2f s  %s" % (
        lg, m.info()["window_bits"], t, s, pre, rb, gr, min(ms), load_s, "ok" if out == ref else "MISMATCH"),
        flush=True)
    m.close()
    ctx.close()

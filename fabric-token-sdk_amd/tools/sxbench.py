#!/usr/bin/env python3
"""Sextet primitive throughput: ops/s and the implied MAD rate."""
import ctypes
import os
lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "..", "zkatdlog", "_lib", "libftssxbench.so"))
lib.ftz_sxbench.restype = ctypes.c_double
lib.ftz_sxbench.argtypes = [ctypes.c_int] * 4
# MADs per lane per op (w2_mac 192, redc 72, reduced Fp2 product 3 x 136)
MADS = {0: 6 * 192 + 144, 1: 4 * 192 + 144, 2: 3 * 192 + 144, 3: 2 * 192 + 144, 4: 408}
NAMES = {0: "sx_mul", 1: "sx_sqr", 2: "sx_mul_line", 3: "sx_cyc_sqr", 4: "fp2_mul/lane"}
for op in range(5):
    for blocks in (1024, 2048, 4096):
        r = lib.ftz_sxbench(0, op, blocks, 200)
        lanes_mad = r * 6 * MADS[op]
        print("%-14s blocks=%5d  %8.2f M ops/s  %6.2f T MAD/s (lane MADs)" % (NAMES[op], blocks, r / 1e6, lanes_mad / 1e12),
              flush=True)

#!/usr/bin/env python3
"""Microbenchmark: C CIOS vs inline-asm FIPS Montgomery products on the GPU."""
import ctypes
lib = ctypes.CDLL('fabric-token-sdk_amd/zkatdlog/_lib/libftsfpcheck.so')
lib.ftz_fpbench.restype = ctypes.c_double
lib.ftz_fpbench.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
for impl in (0, 1):
    for w in (1, 2, 4, 8):
        r = lib.ftz_fpbench(0, impl, 2000, w)
        print("impl=%d waves/simd=%d  %.2f G mont-mul/s  (%.2f TMAD/s eq)" % (impl, w, r / 1e9, r * 136 / 1e12))

#!/usr/bin/env python3
"""dev/row29.h on one MI355X: the device check against dev/fp29.h
(ftz_rowcheck) and the cycles per dependent Montgomery product of one wave,
one-lane f29_mul_c (impl 0) against the row-wide row_mul (impl 1).
    python fabric-token-sdk_amd/tools/rowbench.py
"""
import ctypes, os
lib = ctypes.CDLL(os.path.join("fabric-token-sdk_amd", "zkatdlog", "_lib", "libftsfpcheck.so"))
lib.ftz_rowbench.restype = ctypes.c_long
out = (ctypes.c_uint32 * 3)()
lib.ftz_rowcheck.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
print("rowcheck", lib.ftz_rowcheck(0, 777, out), list(out))
for impl in (0, 1, 0, 1):
    print("impl", impl, "cycles/product", lib.ftz_rowbench(0, impl, 2000))

#!/usr/bin/env python3
"""Montgomery-product throughput vs chains/lane and waves (design data)."""
import ctypes
import os
lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "..", "zkatdlog", "_lib", "libftsfpmicro.so"))
lib.ftz_fpmicro.restype = ctypes.c_double
lib.ftz_fpmicro.argtypes = [ctypes.c_int] * 5
for impl in (0, 1):
    for ch in (1, 2, 4):
        row = []
        for waves in (256, 512, 1024, 2048, 4096, 8192):
            r = lib.ftz_fpmicro(0, impl, ch, waves, 2000)
            row.append("%6.1f" % (r / 1e9))
        print("impl=%s chains=%d  G mont/s @waves 256..8192: %s" % ("cios" if impl == 0 else "fips", ch, " ".join(row)),
              flush=True)

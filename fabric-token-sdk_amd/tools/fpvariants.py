#!/usr/bin/env python3
"""A/B of Montgomery-product builds: python fpvariants.py libfpm_A.so libfpm_B.so ...
(each built from csrc/tools/fpmicro.hip with different -D options)."""
import ctypes
import os
import sys

D = os.path.join(os.path.dirname(__file__), "..", "zkatdlog", "_lib")
for name in sys.argv[1:]:
    lib = ctypes.CDLL(os.path.join(D, name))
    lib.ftz_fpmicro.restype = ctypes.c_double
    lib.ftz_fpmicro.argtypes = [ctypes.c_int] * 5
    for impl in (1, 2):
        for ch in (1, 2, 4):
            row = []
            for waves in (1024, 2048, 4096, 8192):
                row.append("%6.1f" % (lib.ftz_fpmicro(0, impl, ch, waves, 1000) / 1e9))
            print("%s impl=%s chains=%d G/s @waves 1024..8192: %s" % (name, ("fips", "wide")[impl - 1], ch,
                                                                     " ".join(row)), flush=True)

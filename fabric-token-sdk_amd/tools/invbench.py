#!/usr/bin/env python3
"""dev/safegcd.h on one MI355X: the device check against the binary Euclid
(ftz_invcheck) and one lane's cycles per dependent inversion, Euclid (impl 0)
against Bernstein-Yang divsteps on 62-bit (impl 1) and 30-bit limbs (impl 2).
    python fabric-token-sdk_amd/tools/invbench.py
"""
import ctypes, os
lib = ctypes.CDLL(os.path.join("fabric-token-sdk_amd", "zkatdlog", "_lib", "libftsfpcheck.so"))
lib.ftz_invbench.restype = ctypes.c_long
lib.ftz_invcheck.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32]
print("invcheck mismatches", lib.ftz_invcheck(0, 1024, 4242))
for impl in (0, 1, 2, 0, 1, 2):
    print("impl", impl, "cycles/inversion", lib.ftz_invbench(0, impl, 200))

"""dev/fp29.h -- the carry-free 9 x 29-bit BN254 field form the G1 loops run in
(variable-base GLV, fixed-base windows) -- against the fp.h arithmetic they
replace: products and sums at the bounds the formulas use, conversions both
ways, and long j29_dbl / j29_madd chains against jac_dbl / jac_add_aff with the
exceptional additions (from infinity, P + P, P + (-P)).  The G1 results of the
verifier pipeline itself are checked end to end by the golden verdict tests,
which run the same loops (tests/native/emu_exec.cpp)."""
import ctypes

import pytest


@pytest.mark.parametrize("seed", [1, 7, 0xfeedface])
def test_fp29_matches_fp(emu, seed):
    emu.emu_f29_check.restype = ctypes.c_int
    emu.emu_f29_check.argtypes = [ctypes.c_uint64, ctypes.c_int]
    assert emu.emu_f29_check(seed, 3000) == 0

"""Sextet (6 lanes per pairing job) arithmetic, host-emulated with six threads
and a barrier: every operation must equal the one-lane tower / pairing code
bit for bit (which test_emu.py pins to the Python oracle)."""
import ctypes
import random

import pytest
from conftest import build_emu

from ftsoracle import bn254 as C


@pytest.fixture(scope="module")
def sx():
    return ctypes.CDLL(build_emu())


def test_sextet_field_ops(sx):
    # mul, sqr, sparse line mul, cyclotomic sqr, frobenius 1/2/3, inverse, conj, expt
    assert sx.sxe_ops(20241016, 4) == 0


@pytest.mark.parametrize("variant", [0, 1], ids=["exact", "fuentes"])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_sextet_final_exp(sx, seed, variant):
    a, b = (ctypes.c_uint8 * 384)(), (ctypes.c_uint8 * 384)()
    assert sx.sxe_fexp(seed, variant, a, b) == 0
    assert bytes(a) == bytes(b)


@pytest.mark.parametrize("variant", [0, 1], ids=["exact", "fuentes"])
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_sextet_final_exp_carry_free(sx, seed, variant):
    # dev/sx29.h: the 29-bit balanced-limb accumulation the device kernels run
    a, b = (ctypes.c_uint8 * 384)(), (ctypes.c_uint8 * 384)()
    assert sx.sxe_fexp29(seed, variant, a, b) == 0
    assert bytes(a) == bytes(b)


@pytest.mark.parametrize("case", ["both", "p2_inf", "p1_inf", "q2_inf"])
def test_sextet_miller(sx, case):
    rng = random.Random(case)
    p1 = C.g1_bytes(C.g1_mul(C.G1_GEN, rng.randrange(1, C.R)))
    p2 = C.g1_bytes(C.g1_mul(C.G1_GEN, rng.randrange(1, C.R)))
    q2 = C.g2_bytes(C.g2_mul(C.G2_GEN, rng.randrange(1, C.R)))
    qf = C.g2_bytes(C.g2_mul(C.G2_GEN, rng.randrange(1, C.R)))
    if case == "p2_inf":
        p2 = bytes(64)
    if case == "p1_inf":
        p1 = bytes(64)
    if case == "q2_inf":
        q2 = bytes(128)
    a, b = (ctypes.c_uint8 * 384)(), (ctypes.c_uint8 * 384)()
    assert sx.sxe_miller(p1, p2, q2, qf, a, b) == 0
    assert sx.sxe_miller29(p1, p2, q2, qf) == 0  # the carry-free f-chain of the device kernel


@pytest.mark.parametrize("case", ["random", "r_infinity", "zero_scalar", "all_zero", "madd_doubling", "madd_cancel"])
def test_sextet_g2_lines(sx, case):
    """G2 fixed-base combination + the 88 evaluated pair-2 lines, six lanes vs one, and
    the split one-lane path with both part kernels (32-bit Jacobian and the carry-free
    XYZZ form of dev/g2x29.h).  madd_doubling / madd_cancel make one part lane add a
    table point equal to (minus) its running sum: with the emulation's 8-bit windows
    (32 per base) part lane 0 takes window 4 of base 0 and then window 0 of base 1, and
    B1 = +-2^32 B0 with k0 = d 2^32, k1 = d makes those two table points equal (opposite)."""
    rng = random.Random("g2" + case)
    B = [C.g2_mul(C.G2_GEN, rng.randrange(1, C.R)) for _ in range(3)]
    ks = [rng.randrange(C.R) for _ in range(3)]
    if case == "zero_scalar":
        ks[1] = 0
    if case == "all_zero":
        ks = [0, 0, 0]
    if case in ("madd_doubling", "madd_cancel"):
        d = 77
        B[1] = C.g2_mul(B[0], (1 << 32) if case == "madd_doubling" else C.R - (1 << 32))
        ks[0] = d << 32
        ks[1] = d
    bases = b"".join(C.g2_bytes(b) for b in B)
    p2 = C.g1_bytes(C.g1_mul(C.G1_GEN, rng.randrange(1, C.R))) if case != "r_infinity" else bytes(64)
    scal = b"".join(k.to_bytes(32, "big") for k in ks)
    assert sx.sxe_g2lines(bases, p2, scal) == 0


@pytest.mark.parametrize("case", ["random", "r_infinity", "zero_scalar", "all_zero", "p1_infinity"])
def test_g2_lines_carry_free(sx, case):
    """One-lane t' + pair-2 lines on the carry-free form -- tests/native/g2l29.h, and the
    device's k_g2_part + k_g2lines1 (dev/g2x29.h, dev/g2lines29.h): same t', and the same
    GT after the Miller f-chain and the final exponentiation as the 32-bit one-lane lines
    (which test_sextet_g2_lines pins to the sextet ones)."""
    rng = random.Random("g29" + case)
    bases = b"".join(C.g2_bytes(C.g2_mul(C.G2_GEN, rng.randrange(1, C.R))) for _ in range(3))
    p2 = C.g1_bytes(C.g1_mul(C.G1_GEN, rng.randrange(1, C.R))) if case != "r_infinity" else bytes(64)
    p1 = C.g1_bytes(C.g1_mul(C.G1_GEN, rng.randrange(1, C.R))) if case != "p1_infinity" else bytes(64)
    qf = C.g2_bytes(C.g2_mul(C.G2_GEN, rng.randrange(1, C.R)))
    ks = [rng.randrange(C.R) for _ in range(3)]
    if case == "zero_scalar":
        ks[1] = 0
    if case == "all_zero":
        ks = [0, 0, 0]
    scal = b"".join(k.to_bytes(32, "big") for k in ks)
    gt = (ctypes.c_uint8 * 384)()
    assert sx.sxe_g2lines29(bases, p2, scal, p1, qf, gt) == 0
    assert sx.sxe_g2l29_consts() == 0


def test_g2x29_scanned_products(sx):
    """dev/g2x29.h q2_mulb / q2_sqrb (product scanning) return the words of sx29.h's
    column product w29_prod1 for balanced operands, differences of two, and limbs at
    the bounds (2^29 operand limbs against balanced 2^28 ones)."""
    assert sx.sxe_q2_scan(12345, 400) == 0


def test_fexp_easy_split(sx):
    """The device's easy part in three launches (dev/sx29.h sq_fexp_easy_a, the batched
    inversion of k_fexp_binv, sq_fexp_easy_b) gives sq_fexp_easy's m word for word."""
    assert sx.sxe_fexp_easy_split(777) == 0

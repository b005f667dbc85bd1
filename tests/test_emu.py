"""CPU: the product's device code (dev/*.h job functions) and host planner,
compiled for the host by the TEST-ONLY emulation library, against the oracle.
This is how the CPU tier checks the GPU formulas; the product library itself
has no CPU path."""
import ctypes
import hashlib
import random

import pytest

from conftest import case_tuple
from ftsoracle import bn254 as C
from zkatdlog import _abi as A


def buf(n):
    return ctypes.create_string_buffer(n)


def test_field_ops(emu):
    rng = random.Random(7)
    for _ in range(100):
        x, y = rng.randrange(C.P), rng.randrange(C.P)
        o = buf(32)
        emu.emu_fp_mul(x.to_bytes(32, "big"), y.to_bytes(32, "big"), o)
        assert int.from_bytes(o.raw, "big") == x * y % C.P
        emu.emu_fp_inv(x.to_bytes(32, "big"), o)
        assert int.from_bytes(o.raw, "big") == pow(x, C.P - 2, C.P)
        a, b = rng.randrange(1 << 256), rng.randrange(C.R)
        emu.emu_fr_mul(a.to_bytes(32, "big"), b.to_bytes(32, "big"), o)
        assert int.from_bytes(o.raw, "big") == a * b % C.R


def test_fp_inv_var(emu):
    """binary-EEA inverse (dev/fp.h fp_inv_var) against Fermat, incl. edge values"""
    rng = random.Random(17)
    vals = [1, 2, C.P - 1, C.P - 2, (C.P + 1) // 2, 1 << 200] + [rng.randrange(1, C.P) for _ in range(300)]
    o = buf(32)
    for x in vals:
        emu.emu_fp_inv_var(x.to_bytes(32, "big"), o)
        assert int.from_bytes(o.raw, "big") == pow(x, C.P - 2, C.P)
    emu.emu_fp_inv_var(bytes(32), o)
    assert o.raw == bytes(32)


def test_group_ops(emu):
    rng = random.Random(8)
    for _ in range(8):
        k = rng.randrange(1 << 256)
        P = C.g1_mul(C.G1_GEN, rng.randrange(C.R))
        o = buf(64)
        assert emu.emu_g1_mul(C.g1_bytes(P), k.to_bytes(32, "big"), o) == 0
        assert o.raw == C.g1_bytes(C.g1_mul(P, k))
    for _ in range(3):
        k = rng.randrange(1 << 256)
        Q = C.g2_mul(C.G2_GEN, rng.randrange(C.R))
        o = buf(128)
        assert emu.emu_g2_mul(C.g2_bytes(Q), k.to_bytes(32, "big"), o) == 0
        assert o.raw == C.g2_bytes(C.g2_mul(Q, k))


def test_sha256_and_hash_to_zr(emu):
    for data in [b"", b"abc", bytes(range(256)) * 3, b"a" * 55, b"a" * 56, b"a" * 64, b"x" * 1451]:
        o, m = buf(32), buf(32)
        emu.emu_sha256(data, len(data), o, m)
        assert o.raw == hashlib.sha256(data).digest()
        assert int.from_bytes(m.raw, "big") == C.hash_to_zr(data)


def test_pairing_gt_bytes(emu):
    P, Q = C.g1_mul(C.G1_GEN, 12345), C.g2_mul(C.G2_GEN, 6789)
    o = buf(384)
    emu.emu_pairing(C.g1_bytes(P), C.g2_bytes(Q), o)
    assert o.raw == C.gt_bytes(C.pairing(P, Q))
    P2, Q2, Qf = C.g1_mul(C.G1_GEN, 7), C.g2_mul(C.G2_GEN, 9), C.g2_mul(C.G2_GEN, 31337)
    emu.emu_pairing2_fixed(C.g2_bytes(Qf), C.g1_bytes(P), C.g1_bytes(P2), C.g2_bytes(Q2), o)
    assert o.raw == C.gt_bytes(C.final_exp(C.miller_loop([(P, Qf), (P2, Q2)])))
    # infinity on the fixed pair contributes 1
    emu.emu_pairing2_fixed(C.g2_bytes(Qf), bytes(64), C.g1_bytes(P2), C.g2_bytes(Q2), o)
    assert o.raw == C.gt_bytes(C.pairing(P2, Q2))


def _run(emu, pp_json, cases):
    err = ctypes.create_string_buffer(256)
    ctx = emu.emu_ctx_create(pp_json, len(pp_json), err, 256)
    assert ctx, err.value
    try:
        got = {}
        tr = [c for c in cases if c["kind"] == "transfer"]
        iss = [c for c in cases if c["kind"] == "issue"]
        if tr:
            arr, keep = A.pack_transfers([case_tuple(c) for c in tr])
            codes = (ctypes.c_int32 * len(tr))()
            emu.emu_verify_transfers(ctx, len(tr), arr, codes)
            got.update({c["name"]: v for c, v in zip(tr, codes)})
        if iss:
            arr, keep = A.pack_issues([case_tuple(c) for c in iss])
            codes = (ctypes.c_int32 * len(iss))()
            emu.emu_verify_issues(ctx, len(iss), arr, codes)
            got.update({c["name"]: v for c, v in zip(iss, codes)})
        return got
    finally:
        emu.emu_ctx_destroy(ctx)


def test_pipeline_golden_pp_a(emu, golden):
    cases = golden["pp_a"]["cases"]
    got = _run(emu, golden["pp_a"]["pp"].encode(), cases)
    bad = {c["name"]: (got[c["name"]], c["expect"]) for c in cases if got[c["name"]] != c["expect"]}
    assert not bad, bad


def test_pipeline_golden_pp_b(emu, golden):
    if "pp_b" not in golden:
        pytest.skip("no PP-B fixtures")
    cases = golden["pp_b"]["cases"]
    got = _run(emu, golden["pp_b"]["pp"].encode(), cases)
    assert got == {c["name"]: c["expect"] for c in cases}


def test_g1_mul_glv_variants(emu):
    """Both GLV variable-base multiplications of the G1 jobs (dev/jobs.h:
    g1_mul_glv, g1_mul_glv16) against the oracle, edge scalars included."""
    rng = random.Random(11)
    lam = next(w for w in (pow(g, (C.R - 1) // 3, C.R) for g in range(2, 50)) if w != 1)  # a cube root of unity
    ks = [0, 1, 2, 3, 15, 16, 17, C.R - 1, C.R - 2, lam, C.R - lam, (1 << 127) - 1, 1 << 127, (1 << 128) + 5,
          8 * sum(16 ** i for i in range(32))]
    ks += [rng.randrange(C.R) for _ in range(24)]
    for n, k in enumerate(ks):
        P = C.g1_mul(C.G1_GEN, rng.randrange(1, C.R)) if n % 3 else C.G1_GEN
        want = C.g1_bytes(C.g1_mul(P, k % C.R))
        for which in (0, 1):
            o = buf(64)
            assert emu.emu_g1_mul_glv(C.g1_bytes(P), (k % C.R).to_bytes(32, "big"), which, o) == 0
            assert o.raw == want, (k, which)


def test_g1_variable_point_forms(emu):
    """The variable part of a G1 job (dev/jobs.h g1_var_point + the GLV
    multiplication on the isomorphic curve, g1_mul_glv16_iso) for every form the
    planner emits (planner.cpp:777-787): a unit point, Horner sums with a
    power-of-two base (PP-B, b = 16, e = 16) and a general base (PP-A, b = 100,
    e = 2; b = 10, e = 19), explicit 64-bit weights (powers the planner could
    not mark exact), zero weights, sums that cancel to the point at infinity,
    and negation -- against the oracle."""
    import ctypes
    rng = random.Random(23)
    emu.emu_g1_var_part.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p]
    M64 = (1 << 64) - 1

    def pts(n):
        return [C.g1_mul(C.G1_GEN, rng.randrange(1, C.R)) for _ in range(n)]

    G = C.G1_GEN
    cases = [
        (pts(1), [1], False),
        (pts(1), [16], True),
        (pts(16), [16] * 16, True),
        (pts(2), [100, 100], True),
        (pts(19), [10] * 19, True),
        (pts(3), [1, 2, 3], True),
        (pts(4), [1, 0, M64, 1 << 63], False),
        (pts(3), [rng.randrange(1 << 64) for _ in range(3)], False),
        (pts(2), [0, 0], False),
        ([G, C.g1_neg(C.g1_mul(G, 100))], [1, 100], False),
        ([C.g1_neg(C.g1_mul(G, 100)), G], [100, 100], True),
        ([G, C.g1_neg(C.g1_mul(G, 100))], [100, 100], True),  # 100 G - 100 G = O
        ([G, G], [1, 1], False),  # doubling inside the sum
        # signed int64 weights (horner = 2): int64(math.Pow) = -2^63 subtracts 2^63 P (range/proof.go:428)
        (pts(3), [1, 1000, -(1 << 63)], 2),
        (pts(2), [-(1 << 63), -(1 << 63)], 2),
        ([G, G], [1 << 62, -(1 << 63)], 2),  # 2^62 G - 2^63 G
        (pts(1), [-(1 << 63)], 2),
    ]
    for n, (P, w, horner) in enumerate(cases):
        cnt = len(P)
        c = [w[0] ** (cnt - 1 - t) for t in range(cnt)] if horner is True else w
        V = None
        for Pt, ct in zip(P, c):
            V = C.g1_add(V, C.g1_mul(Pt, ct % C.R))
        for vneg in (0, 1):
            k = rng.randrange(C.R) if n % 2 else C.R - 1
            want = C.g1_mul(C.g1_neg(V) if vneg else V, k)
            o = buf(64)
            warr = (ctypes.c_uint64 * cnt)(*[x % (1 << 64) for x in w])
            assert emu.emu_g1_var_part(b"".join(C.g1_bytes(p) for p in P), warr, cnt, int(horner), vneg,
                                       k.to_bytes(32, "big"), o) == 0
            assert o.raw == C.g1_bytes(want), (n, vneg)

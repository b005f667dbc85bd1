"""Token commitments (ftz_commit_tokens; token/token.go:64-76 computeTokens)
and auditor opening checks (ftz_audit_openings; audit/auditor.go:208-234
InspectOutput) against the oracle.  CPU tier: the host build of the same
planner + job code (TEST-ONLY tests/native); GPU tier: the C ABI."""
import ctypes
import random

import pytest

from ftsoracle import bn254 as C
from ftsoracle import zkat as Z
from zkatdlog import _abi as A


@pytest.fixture(scope="module")
def pp_a(golden):
    js = golden["pp_a"]["pp"].encode()
    return js, Z.PublicParams.from_json(js)


def openings(seed, n):
    rng = random.Random(seed)
    types = ["ABC", "", "tok<&>\"x\"", "USDé", "x" * 200]
    out = []
    for i in range(n):
        v = rng.choice([0, 1, rng.randrange(1 << 64), C.R - 1, C.R + 5, (1 << 256) - 1])
        out.append((types[i % len(types)], v, rng.randrange(1 << 256)))
    return out


def oracle_commit(pp, o):
    t, v, b = o
    return C.g1_bytes(Z.token_commitment(pp, t, v % C.R, b % C.R))


def audit_cases(pp, n=24):
    ops = openings(7, n)
    coms = [oracle_commit(pp, o) for o in ops]
    want = [0] * n
    # mismatches: value+1, other type, other bf
    ops[1] = (ops[1][0], ops[1][1] + 1, ops[1][2]); want[1] = A.FTZ_ERR_OPENING
    ops[2] = ("ABD", ops[2][1], ops[2][2]); want[2] = A.FTZ_ERR_OPENING
    ops[3] = (ops[3][0], ops[3][1], ops[3][2] + 1); want[3] = A.FTZ_ERR_OPENING
    bad = bytearray(coms[4]); bad[63] ^= 1; coms[4] = bytes(bad); want[4] = A.FTZ_ERR_PARSE
    coms[5] = bytes(64); want[5] = A.FTZ_ERR_OPENING  # infinity vs a real opening
    # compressed encoding of the right point is the same point (gnark SetBytes)
    P = Z.token_commitment(pp, ops[6][0], ops[6][1] % C.R, ops[6][2] % C.R)
    x, y = P[0], P[1]
    flag = 0xC0 if y > (-y) % C.P else 0x80
    coms[6] = bytes([flag | (x >> 248)]) + (x % (1 << 248)).to_bytes(31, "big") + bytes(32)
    # 64 bytes whose flag says compressed: gnark SetBytes decodes the first 32
    # (the oracle's g1_from_bytes restates it); want what the oracle decides
    try:
        Q = C.g1_from_bytes(coms[6])
        want[6] = 0 if Q == P else A.FTZ_ERR_OPENING
    except C.DecodeError:
        want[6] = A.FTZ_ERR_PARSE
    return coms, ops, want


def emu_openings(emu, js, ops, coms=None):
    emu.emu_openings.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(A.TokenOpening), ctypes.c_char_p,
                                 ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_int32)]
    ctx = emu.emu_ctx_create(js, len(js), ctypes.create_string_buffer(256), 256)
    try:
        arr, keep = A.pack_openings(ops)
        n = len(ops)
        out = (ctypes.c_uint8 * (64 * n))()
        codes = (ctypes.c_int32 * n)()
        emu.emu_openings(ctx, n, arr, b"".join(coms) if coms else None, out, codes)
        raw = bytes(out)
        return [raw[64 * i:64 * i + 64] for i in range(n)], list(codes)
    finally:
        emu.emu_ctx_destroy(ctx)


def test_emu_commit_tokens_match_oracle(emu, pp_a):
    js, pp = pp_a
    ops = openings(3, 20)
    got, codes = emu_openings(emu, js, ops)
    assert codes == [0] * len(ops)
    assert got == [oracle_commit(pp, o) for o in ops]


def test_emu_audit_openings(emu, pp_a):
    js, pp = pp_a
    coms, ops, want = audit_cases(pp)
    _, codes = emu_openings(emu, js, ops, coms)
    assert codes == want


@pytest.fixture(scope="module")
def gctx(golden):
    import zkatdlog
    c = zkatdlog.Context(golden["pp_a"]["pp"].encode(), device=0)
    yield c
    c.close()


@pytest.mark.gpu
def test_gpu_commit_tokens_match_oracle(gctx, pp_a):
    _, pp = pp_a
    ops = openings(5, 40)
    assert gctx.commit_tokens(ops) == [oracle_commit(pp, o) for o in ops]


@pytest.mark.gpu
def test_gpu_audit_openings(gctx, pp_a, emu):
    js, pp = pp_a
    coms, ops, want = audit_cases(pp)
    got = gctx.audit_openings(coms, ops)
    _, emu_codes = emu_openings(emu, js, ops, coms)
    assert got == emu_codes == want


@pytest.mark.gpu
def test_gpu_commit_tokens_large(gctx, pp_a):
    """2^17 + 3 openings (two device batches + a tail), spot-checked."""
    _, pp = pp_a
    n = (1 << 17) + 3
    base = openings(9, 64)
    ops = [base[i % 64][:2] + ((base[i % 64][2] + i) % C.R,) for i in range(n)]
    got = gctx.commit_tokens(ops)
    for i in (0, 1, 63, 65536, 65537, n - 1):
        assert got[i] == oracle_commit(pp, ops[i]), i
    assert gctx.audit_openings(got[:4096], ops[:4096]) == [0] * 4096

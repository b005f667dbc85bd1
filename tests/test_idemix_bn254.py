"""Idemix owner signatures and the auditor's owner match on BN254, the idemix
curve the reference deploys (cmd/pp/dlog/gen.go:117,
integration/nwo/token/platform.go:56, identity/msp/idemix/lm.go:153, dispatched
by identity/msp/idemix/deserializer.go:40-51 to the gurvy translator).

The issuer is the reference's own tokengen issuer
(cmd/tokengen/testdata/idemix/ca, recorded in tests/golden/idemix_bn254_golden.json
by make_idemix_bn254.py): HSk, HRand, HAttrs, W and the IPK Hash are reference
bytes.  The key's own Check proof pins the BN254 G1/G2 encodings and HashToZr
(test_idemix.py::test_bn254_issuer_key_pins_zkatdlog_encodings); here a
credential issued under the reference's IssuerSecretKey is checked with the
oracle's pairing against the reference's W, and the oracle, the host emulation
(product decoder + device job code on the CPU) and, on the GPU, the C ABI must
reproduce every golden verdict.  The NymSignature transcript layout and the
gurvy translator's decoding rules stay [EXT] (IBM/idemix is not vendored; no
reference file holds a BN254 NymSignature): parity unpinned below the pinned
encodings.
"""
import ctypes
import json
import os
import random
import time

import pytest

from ftsoracle import bn254 as C
from ftsoracle import idemix as I

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "idemix_bn254_golden.json")
BN = 1


@pytest.fixture(scope="module")
def gold():
    return json.load(open(GOLD))


@pytest.fixture(scope="module")
def ipk(gold):
    return I.IssuerPKBn254(bytes.fromhex(gold["ipk"]))


def items(cases):
    return [(bytes.fromhex(c["owner"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["sig"])) for c in cases]


def audit_items(cases):
    return [(bytes.fromhex(c["owner"]), bytes.fromhex(c["audit_info"])) for c in cases]


def test_issuer_is_the_reference_tokengen_issuer(gold, ipk):
    """the fixture's IPK/ISK are the reference's cmd/tokengen ca files (as recorded
    in idemix_golden.json's ipk_fixtures), the key's proof verifies on BN254,
    W = g2^isk, and every H is a finite BN254 point"""
    fx = json.load(open(os.path.join(HERE, "golden", "idemix_golden.json")))["ipk_fixtures"]
    ca = [f for f in fx if f["path"] == "cmd/tokengen/testdata/idemix/ca/IssuerPublicKey"][0]
    assert ca["raw"] == gold["ipk"] and ca["isk"] == gold["isk"]
    raw = bytes.fromhex(gold["ipk"])
    assert I.issuer_key_check_bn254(raw) == (True, "")
    m = I.pb_decode(raw, I.IPK_S)
    w = C.g2_from_bytes(b"".join(m[5][k] for k in (1, 2, 3, 4)))
    assert C.g2_mul(C.G2_GEN, int(gold["isk"], 16)) == w
    assert ipk.hsk_s == ipk.hrand_s == "ok" and len(ipk.hattrs) == 4
    assert all(s == "ok" and p is not None for s, p in ipk.hattrs_s)


def test_credential_under_reference_issuer_key(gold, ipk):
    """idemix Credential.Ver on the fixture credential: e(A, W g2^e) == e(B, g2)
    with the reference's W, and B = g1 HSk^sk HRand^s prod HAttrs_i^a_i over the
    reference's H bases -- the nym key sk signs every golden signature"""
    cr = gold["credential"]
    raw = bytes.fromhex(gold["ipk"])
    m = I.pb_decode(raw, I.IPK_S)
    w = C.g2_from_bytes(b"".join(m[5][k] for k in (1, 2, 3, 4)))
    A = C.g1_from_bytes(bytes.fromhex(cr["A"]))
    B = C.g1_from_bytes(bytes.fromhex(cr["B"]))
    sk, s, e = (int(cr[k], 16) for k in ("sk", "s", "e"))
    attrs = [int(a, 16) for a in cr["attrs"]]
    assert attrs[0] == C.hash_to_zr(cr["attr_strings"]["ou"].encode())
    assert attrs[2] == C.hash_to_zr(cr["attr_strings"]["enrollment_id"].encode())
    b = C.g1_add(C.g1_add(C.G1_GEN, C.g1_mul(ipk.hsk, sk)), C.g1_mul(ipk.hrand, s))
    for h, a in zip(ipk.hattrs, attrs):
        b = C.g1_add(b, C.g1_mul(h, a))
    assert b == B
    lhs = C.pairing(A, C.g2_add(w, C.g2_mul(C.G2_GEN, e)))
    rhs = C.pairing(B, C.G2_GEN)
    assert C.f12_eq(lhs, rhs)
    assert not C.f12_eq(C.pairing(A, C.g2_add(w, C.g2_mul(C.G2_GEN, e + 1))), rhs)


def test_oracle_reproduces_golden(gold, ipk):
    for c, (o, m, s) in zip(gold["cases"], items(gold["cases"])):
        assert I.bn_owner_verify(ipk, o, m, s) == (c["expect"], c["text"]), c["name"]
    assert {c["expect"] for c in gold["cases"]} == {0, I.ERR_OWNER, I.ERR_SIGNATURE, I.ERR_UNSUPPORTED}
    for c, (o, a) in zip(gold["audit_cases"], audit_items(gold["audit_cases"])):
        assert I.bn_audit_owner_match(ipk, o, a) == (c["expect"], c["text"]), c["name"]
    assert {c["expect"] for c in gold["audit_cases"]} == {0, I.ERR_OWNER, I.ERR_AUDIT, I.ERR_PANIC,
                                                          I.ERR_UNSUPPORTED}


def test_bn254_transcript_differs_from_fp256bn(gold, ipk):
    """negative controls: the FP256BN transcript conventions (65-byte G1, first-32-
    byte Zr) reject every valid BN254 signature, and dropping the 2 tail bytes does too"""
    valid = [t for c, t in zip(gold["cases"], items(gold["cases"])) if c["name"].startswith("valid_len_")]
    saved = I.bn_proof_data
    try:
        I.bn_proof_data = lambda t, nym, h, msg: saved(t, nym, h, msg)[:-2]
        assert all(I.bn_owner_verify(ipk, *t)[0] == I.ERR_SIGNATURE for t in valid)
        I.bn_proof_data = lambda t, nym, h, msg: (b"sign" + b"\x04" + C.g1_bytes(t) + b"\x04" + C.g1_bytes(nym)
                                                  + h[:32] + msg)
        assert all(I.bn_owner_verify(ipk, *t)[0] == I.ERR_SIGNATURE for t in valid)
    finally:
        I.bn_proof_data = saved
    assert all(I.bn_owner_verify(ipk, *t)[0] == 0 for t in valid)


@pytest.fixture(scope="module")
def emu_bn(gold):
    from conftest import build_emu
    lib = ctypes.CDLL(build_emu())
    lib.emu_idemix_create_curve.restype = ctypes.c_void_p
    lib.emu_idemix_create_curve.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_char_p,
                                            ctypes.c_size_t]
    lib.emu_idemix_destroy.argtypes = [ctypes.c_void_p]
    raw = bytes.fromhex(gold["ipk"])
    err = ctypes.create_string_buffer(256)
    h = lib.emu_idemix_create_curve(raw, len(raw), BN, err, 256)
    assert h, err.value
    yield lib, h
    lib.emu_idemix_destroy(h)


def emu_verify(emu_bn, its):
    from zkatdlog import _abi as A
    lib, h = emu_bn
    lib.emu_verify_owner_signatures.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(A.OwnerSig),
                                                ctypes.POINTER(ctypes.c_int32)]
    arr, keep = A.pack_owner_sigs(its)
    codes = (ctypes.c_int32 * len(its))()
    assert lib.emu_verify_owner_signatures(h, len(its), arr, codes) == 0
    return list(codes)


def emu_audit(emu_bn, its):
    from zkatdlog import _abi as A
    lib, h = emu_bn
    lib.emu_audit_owners.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(A.OwnerAudit),
                                     ctypes.POINTER(ctypes.c_int32)]
    arr, keep = A.pack_owner_audits(its)
    codes = (ctypes.c_int32 * max(len(its), 1))()
    assert lib.emu_audit_owners(h, len(its), arr, codes) == 0
    return list(codes[:len(its)])


def test_emu_reproduces_golden(gold, emu_bn):
    """product host decoder (BN254 branch) + device job code (NymCurve<fp>) on the CPU"""
    assert emu_verify(emu_bn, items(gold["cases"])) == [c["expect"] for c in gold["cases"]]
    lib, _ = emu_bn
    lib.emu_decode_owner_signature_curve.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                                     ctypes.c_size_t, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
    why = ctypes.create_string_buffer(256)
    for c, (o, m, s) in zip(gold["cases"], items(gold["cases"])):
        code = lib.emu_decode_owner_signature_curve(o, len(o), s, len(s), BN, why, 256)
        if code:
            assert (code, why.value.decode()) == (c["expect"], c["text"]), c["name"]


def test_emu_audit_reproduces_golden(gold, emu_bn):
    cs = gold["audit_cases"]
    assert emu_audit(emu_bn, audit_items(cs)) == [c["expect"] for c in cs]
    lib, _ = emu_bn
    lib.emu_decode_owner_audit_curve.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                                 ctypes.c_size_t, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
    why = ctypes.create_string_buffer(256)
    for c, (o, a) in zip(cs, audit_items(cs)):
        code = lib.emu_decode_owner_audit_curve(o, len(o), a, len(a), 4, BN, why, 256)
        if code:
            assert (code, why.value.decode()) == (c["expect"], c["text"]), c["name"]


def test_emu_random_tamper_matches_oracle(gold, ipk, emu_bn):
    """single-bit corruptions of owners and signatures (and of audit pairs):
    host emulation == oracle on BN254"""
    base = [t for c, t in zip(gold["cases"], items(gold["cases"])) if c["expect"] == 0][:8]
    rng = random.Random(254)
    its = []
    for k in range(80):
        o, m, s = base[k % len(base)]
        o, s = bytearray(o), bytearray(s)
        tgt = o if k % 2 else s
        tgt[rng.randrange(len(tgt))] ^= 1 << rng.randrange(8)
        its.append((bytes(o), m, bytes(s)))
    want = [I.bn_owner_verify(ipk, o, m, s)[0] for o, m, s in its]
    assert emu_verify(emu_bn, its) == want
    assert len(set(want)) >= 3
    cs = gold["audit_cases"]
    abase = [t for c, t in zip(cs, audit_items(cs)) if c["expect"] == 0]
    its = []
    for k in range(120):
        o, a = abase[k % len(abase)]
        o, a = bytearray(o), bytearray(a)
        tgt = o if k % 2 else a
        tgt[rng.randrange(len(tgt))] ^= 1 << rng.randrange(8)
        its.append((bytes(o), bytes(a)))
    want = [I.bn_audit_owner_match(ipk, o, a)[0] for o, a in its]
    assert emu_audit(emu_bn, its) == want


def test_emu_bn_glv_split_and_mod_r(emu_bn):
    """host/idemix.cpp nym_glv_split_bn (k = k1 + k2 lambda mod r, |k_i| < 2^128,
    lambda the eigenvalue of dev/constants.h GLV_BETA) and be_mod_r"""
    lib, _ = emu_bn
    lib.emu_nym_glv_split_bn.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32)]
    lib.emu_be_mod_r.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    rng = random.Random(5)
    lam = [L for L in (pow(5, (C.R - 1) // 3, C.R), pow(5, 2 * (C.R - 1) // 3, C.R))]
    out = (ctypes.c_uint32 * 12)()
    found = set(lam)
    for k in [0, 1, C.R - 1, C.R // 2] + [rng.randrange(C.R) for _ in range(1500)]:
        lib.emu_nym_glv_split_bn(k.to_bytes(32, "big"), out)
        k1 = sum(out[i] << (32 * i) for i in range(5)) * (-1 if out[10] & 1 else 1)
        k2 = sum(out[5 + i] << (32 * i) for i in range(5)) * (-1 if out[10] & 2 else 1)
        assert abs(k1) < 1 << 128 and abs(k2) < 1 << 128
        found &= {L for L in lam if (k1 + k2 * L - k) % C.R == 0}
        assert found, k
    assert len(found) == 1
    buf = ctypes.create_string_buffer(32)
    for n in (0, 1, 5, 31, 32, 33, 40, 64, 100):
        for _ in range(20):
            b = bytes(rng.randrange(256) for _ in range(n))
            lib.emu_be_mod_r(b, len(b), buf)
            assert int.from_bytes(buf.raw, "big") == int.from_bytes(b, "big") % C.R


def test_abi_accepts_bn254_curve_id_argument_checks():
    """no GPU in the CPU tier: the curve id is validated before any device call"""
    from zkatdlog import _abi as A
    lib = A.load()
    out = ctypes.c_void_p()
    assert lib.ftz_idemix_create(None, b"x", 1, BN, ctypes.byref(out)) == -1


# ---------------------------------------------------------------- GPU tier
@pytest.fixture(scope="module")
def gpu_bn(gold):
    import zkatdlog
    from zkatdlog import _abi
    g = json.load(open(os.path.join(HERE, "golden", "zkatdlog_golden.json")))["pp_a"]
    ctx = zkatdlog.Context(g["pp"].encode(), device=0)
    ix = zkatdlog.Idemix(ctx, bytes.fromhex(gold["ipk"]), curve_id=_abi.FTZ_CURVE_BN254)
    yield ix
    ix.close()
    ctx.close()


@pytest.mark.gpu
def test_gpu_bn254_golden(gold, gpu_bn):
    assert gpu_bn.verify_owner_signatures(items(gold["cases"])) == [c["expect"] for c in gold["cases"]]


@pytest.mark.gpu
def test_gpu_bn254_batch_and_tamper(gold, ipk, gpu_bn):
    """8192 signatures (golden cases tiled) plus 400 oracle-labelled single-bit
    corruptions, bit-exact"""
    cs = gold["cases"]
    its = items(cs)
    n = 8192
    sel = [k % len(cs) for k in range(n)]
    t0 = time.perf_counter()
    got = gpu_bn.verify_owner_signatures([its[k] for k in sel])
    dt = time.perf_counter() - t0
    assert got == [cs[k]["expect"] for k in sel]
    print("%d BN254 owner signatures: %.1f ms (%.0f/s)" % (n, dt * 1e3, n / dt))
    base = [t for c, t in zip(cs, its) if c["expect"] == 0]
    rng = random.Random(99)
    tam = []
    for k in range(400):
        o, m, s = base[k % len(base)]
        o, s = bytearray(o), bytearray(s)
        tgt = o if k % 2 else s
        tgt[rng.randrange(len(tgt))] ^= 1 << rng.randrange(8)
        tam.append((bytes(o), m, bytes(s)))
    assert gpu_bn.verify_owner_signatures(tam) == [I.bn_owner_verify(ipk, *t)[0] for t in tam]


@pytest.mark.gpu
def test_gpu_bn254_audit_owners(gold, gpu_bn):
    cs = gold["audit_cases"]
    its = audit_items(cs)
    assert gpu_bn.audit_owners(its) == [c["expect"] for c in cs]
    sel = [k % len(cs) for k in range(4096)]
    assert gpu_bn.audit_owners([its[k] for k in sel]) == [cs[k]["expect"] for k in sel]


@pytest.mark.gpu
def test_gpu_bn254_owner_verifier_api(gold, gpu_bn):
    import zkatdlog
    ok = [t for c, t in zip(gold["cases"], items(gold["cases"])) if c["name"] == "valid_len_100"][0]
    gpu_bn.owner_verifier(ok[0]).verify(ok[1], ok[2])
    with pytest.raises(zkatdlog.ZKError, match="pseudonym signature invalid"):
        gpu_bn.owner_verifier(ok[0]).verify(ok[1] + b"!", ok[2])

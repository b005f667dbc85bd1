"""CPU: pin the oracle before trusting it -- known-answer facts of BN254 and
SHA-256, pairing properties, the final-exponent identity, and the reference's
own test classes as round trips."""
import hashlib

import pytest

from ftsoracle import bn254 as C
from ftsoracle import gojson as J
from ftsoracle import zkat as Z


def test_sha256_fips180_vectors():
    # FIPS 180-4 / NIST CSRC examples
    assert hashlib.sha256(b"abc").hexdigest() == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"
    assert hashlib.sha256(b"").hexdigest() == "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"
    m = b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq"
    assert hashlib.sha256(m).hexdigest() == "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"


def test_bn254_constants():
    assert C.P == 21888242871839275222246405745257275088696311157297823662689037894645226208583
    assert C.R == 21888242871839275222246405745257275088548364400416034343698204186575808495617
    x = C.X
    assert C.P == 36 * x ** 4 + 36 * x ** 3 + 24 * x ** 2 + 6 * x + 1
    assert C.R == 36 * x ** 4 + 36 * x ** 3 + 18 * x ** 2 + 6 * x + 1
    assert C.g1_on_curve(C.G1_GEN) and C.g2_on_curve(C.G2_GEN)
    assert C.g1_mul(C.G1_GEN, C.R) is None and C.g2_mul(C.G2_GEN, C.R) is None


def test_final_exponent_variants():
    x, p = C.X, C.P
    l0, l1 = 1 + 6 * x + 12 * x ** 2 + 12 * x ** 3, 4 * x + 6 * x ** 2 + 12 * x ** 3
    l2, l3 = 6 * x + 6 * x ** 2 + 12 * x ** 3, -1 + 4 * x + 6 * x ** 2 + 12 * x ** 3
    assert l0 + l1 * p + l2 * p ** 2 + l3 * p ** 3 == C.HARD_FUENTES
    assert C.HARD_FUENTES == 2 * x * (6 * x * x + 3 * x + 1) * C.HARD_EXACT
    assert (p ** 4 - p ** 2 + 1) == C.HARD_EXACT * C.R


def test_pairing_bilinear_nondegenerate():
    e = C.pairing(C.G1_GEN, C.G2_GEN)
    assert e != C.F12_ONE
    assert C.f12_pow(e, C.R) == C.F12_ONE
    a, b = 0x1234567, 0xABCDEF
    assert C.pairing(C.g1_mul(C.G1_GEN, a), C.g2_mul(C.G2_GEN, b)) == C.f12_pow(e, a * b)
    # both variants are pairings; they differ by the exponent s = 2x(6x^2+3x+1)
    ef = C.pairing(C.G1_GEN, C.G2_GEN, C.FE_FUENTES)
    assert C.f12_pow(e, 2 * C.X * (6 * C.X ** 2 + 3 * C.X + 1)) == ef  # default is FE_EXACT


def test_g1_codec_rules():
    P = C.g1_mul(C.G1_GEN, 5)
    raw = C.g1_bytes(P)
    assert C.g1_from_bytes(raw) == P
    assert C.g1_from_bytes(b"\x40" + bytes(63)) is None
    assert C.g1_from_bytes(bytes(64)) is None
    y = int.from_bytes(raw[32:], "big")
    assert C.g1_from_bytes(raw[:32] + (y + C.P).to_bytes(32, "big")) == P   # reduced, not rejected
    with pytest.raises(C.DecodeError):
        C.g1_from_bytes(raw[:63] + bytes([raw[63] ^ 1]))
    with pytest.raises(C.DecodeError):
        C.g1_from_bytes(raw[:40])


def test_gojson_semantics():
    v = J.parse(b'{"a":1,"A":2,"b":null}')
    assert J.dec_int(J.field(v, "a")) == 2          # case-insensitive, last wins
    assert J.field(v, "B") == ("null", None)
    assert J.b64_std_decode("QUJD\nRA==") == b"ABCD"
    with pytest.raises(J.GoJSONError):
        J.b64_std_decode("QUJDRA")
    with pytest.raises(J.GoJSONError):
        J.dec_int(("num", "1.0"))


@pytest.fixture(scope="module")
def pp():
    return Z.setup(10, 2, Z.Rand(b"oracle-test"))


def test_ps_signature_quirk(pp):
    # pssign/sign.go:97-98: R stays the generator
    assert all(R_ == C.G1_GEN for R_, _ in pp.signed_values)


def test_pp_json_round_trip(pp):
    pp2 = Z.PublicParams.from_json(pp.to_json())
    assert pp2.ped == pp.ped and pp2.sign_pk == pp.sign_pk and pp2.q == pp.q
    assert pp2.signed_values == pp.signed_values and pp2.exponent == 2


def test_reference_transfer_classes(pp):
    """transfer/transfer_test.go:53-84 with base 10 (range 0..99)."""
    rnd = Z.Rand(b"t")
    inw = [(9, 11), (6, 22)]
    ins = [Z.token_commitment(pp, "ABC", v, b) for v, b in inw]
    outw = [(5, 33), (10, 44)]
    outs = [Z.token_commitment(pp, "ABC", v, b) for v, b in outw]
    proof = Z.transfer_prove(pp, rnd, ins, outs, inw, outw, "ABC")
    assert Z.transfer_verify(pp, ins, outs, proof) == (True, Z.OK, "")
    badw = [(11, 33), (4, 44)]
    bad = [Z.token_commitment(pp, "ABC", v, b) for v, b in badw]
    p2 = Z.transfer_prove(pp, rnd, ins, bad, inw, [(12, 33), (4, 44)], "ABC")
    ok, code, msg = Z.transfer_verify(pp, ins, bad, p2)
    assert not ok and "invalid zero-knowledge transfer" in msg
    with pytest.raises(ValueError, match="outside authorized range"):
        Z.transfer_prove(pp, rnd, ins, outs, inw, [(100, 1), (5, 2)], "ABC")


def test_reference_membership_bogus_value(pp):
    """sigproof/membership_test.go:34-47: a commitment to a value the signature
    does not sign is rejected with "invalid membership proof"."""
    rnd = Z.Rand(b"m")
    com = C.g1_add(C.g1_mul(pp.ped[0], 7), C.g1_mul(pp.ped[1], 99))
    wire = lambda mp: Z.dec_membership(J.parse(Z.enc_membership(mp)))
    mp = Z.membership_prove(pp, rnd, "x", pp.signed_values[3], 7, 99, com)
    with pytest.raises(Z.VerifyError, match="invalid membership proof"):
        Z.membership_verify(pp, ("pt", com), wire(mp))
    good = Z.membership_prove(pp, rnd, "y", pp.signed_values[7], 7, 99, com)
    Z.membership_verify(pp, ("pt", com), wire(good))


def test_golden_sample_reverifies(golden):
    """The committed fixtures still match the oracle (a sample; all of them run
    through the emulated device pipeline in test_emu.py)."""
    import base64
    pp = Z.PublicParams.from_json(golden["pp_a"]["pp"].encode())
    pick = {"valid_2in_2out", "wf_challenge_plus_r", "range_exponent_mismatch", "g1_compressed_accepts"}
    for c in golden["pp_a"]["cases"]:
        if c["name"] not in pick:
            continue
        ins = [C.g1_from_bytes(bytes.fromhex(c["inputs"])[64 * i:64 * i + 64]) for i in range(len(c["inputs"]) // 128)]
        outs = [C.g1_from_bytes(bytes.fromhex(c["outputs"])[64 * i:64 * i + 64]) for i in range(len(c["outputs"]) // 128)]
        ok, code, _ = Z.transfer_verify(pp, ins, outs, base64.b64decode(c["proof"]))
        assert code == c["expect"], c["name"]

#!/usr/bin/env python3
"""Fixture maker for idemix owner signatures on BN254 (tests/golden/idemix_bn254_golden.json).

BN254 is the idemix curve the reference DEPLOYS: cmd/pp/dlog/gen.go:117 writes
IdemixCurveID = BN254 into every public-parameter file, and so do the NWO
platforms (integration/nwo/token/platform.go:56, fabric/fabric.go:81,
orion/orion.go:72) and the wallet's local membership
(identity/msp/idemix/lm.go:153).  The issuer is the reference's own tokengen
issuer: cmd/tokengen/testdata/idemix/ca/{IssuerPublicKey, IssuerSecretKey}
(read here only, recorded as hex data).  HSk, HRand, HAttrs, W and Hash are
therefore the reference's bytes; the user secret, nym randomness and signature
randomness are drawn from a seeded RNG, and a full idemix credential for the
user is issued under the reference's IssuerSecretKey (A = B^(1/(e + isk)),
B = g1 HSk^sk HRand^s prod HAttrs_i^a_i) so the test can check it with the
oracle's pairing against the key's W.

Every case records the oracle's verdict (ftsoracle.idemix.bn_owner_verify /
bn_audit_owner_match); the [EXT] assumptions are listed in the fixture.

    python tests/golden/make_idemix_bn254.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle", "py"))
from ftsoracle import bn254 as C  # noqa: E402
from ftsoracle import idemix as I  # noqa: E402

sys.path.insert(0, HERE)
from make_idemix import expand  # noqa: E402

CA = "/root/reference/cmd/tokengen/testdata/idemix/ca"


def main():
    ipk_raw = open(os.path.join(CA, "IssuerPublicKey"), "rb").read()
    isk_raw = open(os.path.join(CA, "IssuerSecretKey"), "rb").read()
    ipk = I.IssuerPKBn254(ipk_raw)
    assert I.issuer_key_check_bn254(ipk_raw) == (True, "")
    rng = random.Random(0xB254)

    def rz():
        return rng.randrange(1, C.R)

    sk = rz()
    ou_s, eid_s = b"org1.department1", b"alice"
    role = I.pb_field(1, 2, b"idemix") + I.pb_field(2, 0, 2)
    ou = I.pb_field(1, 2, b"idemix") + I.pb_field(2, 2, ou_s) + I.pb_field(3, 2, b"")

    # ---- a credential under the reference's issuer secret key
    isk = int.from_bytes(isk_raw, "big")
    attrs = [C.hash_to_zr(ou_s), 2, C.hash_to_zr(eid_s), 1234]
    s_cred, e_cred = rz(), rz()
    B = C.g1_add(C.g1_add(C.G1_GEN, C.g1_mul(ipk.hsk, sk)), C.g1_mul(ipk.hrand, s_cred))
    for h, a in zip(ipk.hattrs, attrs):
        B = C.g1_add(B, C.g1_mul(h, a))
    A = C.g1_mul(B, pow(e_cred + isk, -1, C.R))

    def identity(nym, **kw):
        kw.setdefault("ou", ou)
        kw.setdefault("role", role)
        return I.bn_serialize_idemix_identity(nym, **kw)

    def owner(ident, typ=b"si", tag=0x13):
        return I.raw_owner_encode(typ, ident, tag)

    def sigf(vals, extra=b""):
        return b"".join(I.pb_field(k + 1, 2, v) for k, v in enumerate(vals)) + extra

    cases = []

    def add(name, own, msg, sig):
        code, text = I.bn_owner_verify(ipk, own, msg, sig)
        cases.append({"name": name, "owner": own.hex(), "msg": msg.hex(), "sig": sig.hex(), "expect": code,
                      "text": text})

    users = []
    for k in range(4):
        rn = rz()
        users.append((rn, I.bn_make_nym(ipk, sk, rn)))
    # valid signatures over messages of every SHA-256 block position (prefix 164 bytes + 2 tail bytes)
    for L in (0, 1, 2, 27, 28, 29, 53, 54, 55, 56, 63, 64, 65, 100, 1000, 5000, 20000):
        rn, nym = users[L % 4]
        msg = bytes(rng.randrange(256) for _ in range(L))
        add("valid_len_%d" % L, owner(identity(nym)), msg, I.bn_nym_sign(ipk, sk, rn, nym, msg, rz(), rz(), rz()))

    rn, nym = users[0]
    msg = bytes(rng.randrange(256) for _ in range(300))
    sig_ok = I.bn_nym_sign(ipk, sk, rn, nym, msg, rz(), rz(), rz())
    f = I.pb_decode(sig_ok, I.NYMSIG_S)
    vals = [f[1], f[2], f[3], f[4]]
    own = owner(identity(nym))
    # ---- signature tampering
    for idx, nm in enumerate(("proof_c", "s_sk", "s_rnym", "nonce")):
        v = list(vals)
        b = bytearray(v[idx])
        b[31] ^= 1
        v[idx] = bytes(b)
        add("flip_%s" % nm, own, msg, sigf(v))
    add("wrong_message", own, msg + b"x", sig_ok)
    add("other_users_nym", owner(identity(users[1][1])), msg, sig_ok)
    # big.Int SetBytes over whole fields: leading zeros change nothing, a longer
    # field is another integer
    add("leading_zero_padded_fields_accept", own, msg, sigf([b"\x00\x00" + v for v in vals]))
    add("long_fields_are_other_integers", own, msg, sigf([v + b"\xff\x00" for v in vals[:3]] + vals[3:]))
    add("short_proof_c_is_other_integer", own, msg, sigf([vals[0][:31]] + vals[1:]))
    s_sk = int.from_bytes(vals[1], "big")
    add("s_sk_plus_r_accepts", own, msg, sigf([vals[0], (s_sk + C.R).to_bytes(32, "big"), vals[2], vals[3]]))
    add("s_sk_plus_7r_40_bytes_accepts", own, msg, sigf([vals[0], (s_sk + 7 * C.R).to_bytes(40, "big"), vals[2], vals[3]]))
    pc = int.from_bytes(vals[0], "big")
    add("proof_c_plus_r_rejects", own, msg, sigf([(pc + C.R).to_bytes(32, "big")] + vals[1:]))
    add("proof_c_33_bytes_rejects", own, msg, sigf([b"\x01" + vals[0]] + vals[1:]))
    add("nonce_33_bytes_panics", own, msg, sigf(vals[:3] + [b"\x01" + vals[3]]))
    add("nonce_40_zero_padded_accepts", own, msg, sigf(vals[:3] + [bytes(8) + vals[3]]))
    nonce_big = (1 << 256) - 1 - rng.randrange(1 << 200)  # >= r, < 2^256: hashed as its 32 bytes
    add("nonce_unreduced_accepts", own, msg, I.bn_nym_sign(ipk, sk, rn, nym, msg, rz(), rz(), nonce_big))
    z = I.pb_decode(I.bn_nym_sign(ipk, sk, rn, nym, msg, rz(), rz(), 0), I.NYMSIG_S)
    add("absent_nonce_is_zero_accepts", own, msg, sigf([z[1], z[2], z[3]]))
    add("empty_nonce_is_zero_accepts", own, msg, sigf([z[1], z[2], z[3], b""]))
    add("missing_nonce_rejects", own, msg, sigf(vals[:3]))
    add("empty_signature", own, msg, b"")
    add("unknown_field_skipped", own, msg, sig_ok + I.pb_field(9, 2, b"junk") + I.pb_field(12, 0, 7))
    add("duplicate_field_last_wins", own, msg, I.pb_field(1, 2, bytes(32)) + sig_ok)
    add("wrong_wiretype_is_unknown", own, msg, I.pb_field(1, 0, 5) + sig_ok)
    add("group_skipped", own, msg, bytes([(7 << 3) | 3, (1 << 3) | 0, 1, (7 << 3) | 4]) + sig_ok)
    add("stray_end_group", own, msg, sig_ok + bytes([(7 << 3) | 4]))
    add("reserved_wiretype", own, msg, sig_ok + bytes([(7 << 3) | 7]))
    add("truncated_signature", own, msg, sig_ok[:-5])
    add("varint_overflow", own, msg, sig_ok + bytes([(9 << 3)] + [0xff] * 9 + [0x02]))
    # ---- owner identity
    add("htlc_owner_unsupported", owner(b"{}", typ=b"htlc"), msg, sig_ok)
    add("unknown_owner_type", owner(identity(nym), typ=b"xx"), msg, sig_ok)
    add("raw_owner_utf8string", owner(identity(nym), tag=0x0C), msg, sig_ok)
    add("raw_owner_truncated", own[:-3], msg, sig_ok)
    add("identity_not_proto", owner(b"\x0a\xff"), msg, sig_ok)
    raw = C.g1_bytes(nym)
    x, y = raw[:32], raw[32:]
    add("nym_x_empty_is_nil", owner(identity(nym, nymx=b"", nymy=x + y)), msg, sig_ok)
    add("nym_split_31_33_accepts", owner(identity(nym, nymx=x[:31], nymy=x[31:] + y)), msg, sig_ok)
    add("nym_short_halves", owner(identity(nym, nymx=x[:31], nymy=y[:31])), msg, sig_ok)
    add("nym_33_byte_halves", owner(identity(nym, nymx=b"\x00" + x, nymy=b"\x00" + y)), msg, sig_ok)
    add("nym_65_bytes", owner(identity(nym, nymx=x, nymy=y + b"\x00")), msg, sig_ok)
    add("nym_off_curve_rejected", owner(identity(nym, nymy=(nym[1] ^ 1).to_bytes(32, "big"))), msg, sig_ok)
    add("nym_y_plus_p_reduced_accepts", owner(identity(nym, nymy=(nym[1] + C.P).to_bytes(32, "big"))),
        msg, sig_ok)
    # x + p keeps the 00 flags when it stays below 2^254: the coordinate is reduced
    xs = [u for u in users if u[1][0] + C.P < 1 << 254]
    if xs:
        rn2, nym2 = xs[0]
        sig2 = I.bn_nym_sign(ipk, sk, rn2, nym2, msg, rz(), rz(), rz())
        add("nym_x_plus_p_reduced_accepts", owner(identity(nym2, nymx=(nym2[0] + C.P).to_bytes(32, "big"))), msg, sig2)
    # compressed forms of X (gnark SetBytes flags 10 / 11; Y bytes are ignored)
    lexi_largest = nym[1] > C.P - nym[1]
    comp = bytearray(x)
    comp[0] |= 0xC0 if lexi_largest else 0x80
    add("nym_compressed_x_accepts", owner(identity(nym, nymx=bytes(comp), nymy=bytes(32))), msg, sig_ok)
    comp2 = bytearray(x)
    comp2[0] |= 0x80 if lexi_largest else 0xC0
    add("nym_compressed_other_root_rejects", owner(identity(nym, nymx=bytes(comp2), nymy=y)), msg, sig_ok)
    bad = bytearray(C.P.to_bytes(32, "big"))
    bad[0] |= 0x80
    add("nym_compressed_x_ge_p", owner(identity(nym, nymx=bytes(bad), nymy=y)), msg, sig_ok)
    # [EXT] the point at infinity decodes (all-zero RawBytes, or the compressed-infinity
    # flag): a signature made against it without any secret verifies
    ssk, sr, nonce = rz(), rz(), rz()
    t = C.g1_add(C.g1_mul(ipk.hsk, ssk), C.g1_mul(ipk.hrand, sr))
    c = C.hash_to_zr(I.bn_proof_data(t, None, ipk.hash, msg))
    fc = C.hash_to_zr(c.to_bytes(32, "big") + nonce.to_bytes(32, "big"))
    forged = sigf([v.to_bytes(32, "big") for v in (fc, ssk, sr, nonce)])
    add("infinity_nym_forgery_accepts", owner(identity(None, nymx=bytes(32), nymy=bytes(32))), msg, forged)
    add("compressed_infinity_nym_forgery_accepts", owner(identity(None, nymx=b"\x40" + bytes(31), nymy=bytes(32))),
        msg, forged)
    add("ou_not_proto", owner(identity(nym, ou=b"\x0a\x05ab")), msg, sig_ok)
    add("role_not_proto", owner(identity(nym, role=b"\x10")), msg, sig_ok)

    # bench workload (bench.py owner_signatures leg, BN254): as the FP256BN one
    bench = []
    for r in range(32):
        seed = bytes([r]) * 8
        m = expand(seed, 9500)
        for u in range(2):
            rn_u, nym_u = users[(r + u) % 4]
            bench.append({"owner": owner(identity(nym_u)).hex(), "msg_seed": seed.hex(), "msg_len": len(m),
                          "sig": I.bn_nym_sign(ipk, sk, rn_u, nym_u, m, rz(), rz(), rz()).hex()})

    # ---- auditor owner match on BN254
    audits = []

    def aadd(name, o, ai):
        code, text = I.bn_audit_owner_match(ipk, o, ai)
        audits.append({"name": name, "owner": o.hex(), "audit_info": ai.hex(), "expect": code, "text": text})

    def enc(rnym, eid_zr, at, curve=I.BN254_CURVE_ID, nbytes=32):
        from ftsoracle import gojson as J
        z = (lambda v: "null" if v is None else J.enc_elem(v.to_bytes(nbytes, "big") if nbytes else b"", curve))
        return J.enc_struct([("RNymEid", z(rnym)), ("EID", z(eid_zr)),
                             ("Attributes", J.enc_list(at, J.enc_bytes))]).encode()

    at = [ou_s, b"2", eid_s, b"rh"]
    heid = lambda r_: C.g1_add(C.g1_mul(ipk.hattrs[2], C.hash_to_zr(eid_s)), C.g1_mul(ipk.hrand, r_))  # noqa: E731
    for u in range(3):
        r_eid = rz()
        aadd("eid_match_%d" % u, owner(identity(users[u][1], proof=I.bn_signature_with_eid_nym(heid(r_eid)))),
             enc(r_eid, C.hash_to_zr(eid_s), at))
    r_eid = rz()
    good = I.bn_signature_with_eid_nym(heid(r_eid))
    own_a = owner(identity(nym, proof=good))
    ai = enc(r_eid, C.hash_to_zr(eid_s), at)
    aadd("eid_match_rnym_plus_r_40_bytes", own_a, enc(r_eid + 3 * C.R, 0, at, nbytes=40))
    aadd("eid_rnym_empty_element_is_zero",
         owner(identity(nym, proof=I.bn_signature_with_eid_nym(C.g1_mul(ipk.hattrs[2], C.hash_to_zr(eid_s))))),
         enc(0, 0, at, nbytes=0))
    aadd("eid_other_enrollment_id", own_a, enc(r_eid, 0, [at[0], at[1], b"mallory", at[3]]))
    aadd("eid_wrong_rnym", own_a, enc(r_eid + 1, 0, at))
    aadd("eid_nym_of_other_identity", owner(identity(nym, proof=I.bn_signature_with_eid_nym(C.g1_mul(ipk.hrand, 5)))),
         ai)
    ne = heid(r_eid)
    nb = C.g1_bytes(ne)
    off = I.pb_field(18, 2, I.pb_field(1, 2, I.pb_field(1, 2, nb[:32]) + I.pb_field(2, 2, ((ne[1] + 1) % C.P).to_bytes(32, "big"))))
    aadd("eid_nym_off_curve_is_error", owner(identity(nym, proof=off)), ai)
    short = I.pb_field(18, 2, I.pb_field(1, 2, I.pb_field(1, 2, nb[:31]) + I.pb_field(2, 2, nb[32:])))
    aadd("eid_short_nym_coordinate_is_error", owner(identity(nym, proof=short)), ai)
    aadd("eid_short_coordinate_before_nil_rnym", owner(identity(nym, proof=short)), enc(None, 0, at))
    inf = I.pb_field(18, 2, I.pb_field(1, 2, I.pb_field(1, 2, bytes(32)) + I.pb_field(2, 2, bytes(32))))
    aadd("eid_nym_infinity_mismatch", owner(identity(nym, proof=inf)), ai)
    comp = bytearray(nb[:32])
    comp[0] |= 0xC0 if ne[1] > C.P - ne[1] else 0x80
    cpt = I.pb_field(18, 2, I.pb_field(1, 2, I.pb_field(1, 2, bytes(comp)) + I.pb_field(2, 2, bytes(32))))
    aadd("eid_nym_compressed_matches", owner(identity(nym, proof=cpt)), ai)
    aadd("eid_no_eid_nym", owner(identity(nym, proof=I.pb_field(4, 2, bytes(32)))), ai)
    aadd("eid_bad_signature_proto", owner(identity(nym, proof=b"\x0a\x05ab")), ai)
    aadd("eid_attributes_too_short_panics", own_a, enc(r_eid, 0, at[:2]))
    aadd("eid_null_audit_info_panics", own_a, b"null")
    aadd("eid_nil_rnym_panics", own_a, enc(None, 0, at))
    aadd("eid_fp256bn_curve_zr_panics", own_a, enc(r_eid, 0, at, curve=0))
    aadd("eid_foreign_curve_eid_panics", own_a, enc(r_eid, 7, at, curve=1).replace(b'"EID":{"curve":1', b'"EID":{"curve":2'))
    aadd("audit_info_not_json", own_a, b"{oops")
    aadd("audit_info_empty", own_a, b"")
    aadd("redeem_token", b"", ai)
    aadd("htlc_owner_script", owner(b"script", typ=b"htlc"), ai)
    aadd("identity_not_proto", owner(b"\x0a\xff"), ai)

    out = {
        "comment": "idemix owner signatures on BN254, the deployed idemix curve (SURVEY 8(f) row 3); "
                   "issuer = cmd/tokengen/testdata/idemix/ca; made by make_idemix_bn254.py",
        "parity": "UNPINNED for the signature transcript: no file under the reference holds a BN254 "
                  "NymSignature, so the expected verdicts are the oracle's restatement of IBM/idemix + mathlib "
                  "[EXT]; pinned by the reference's tokengen issuer key: HSk, HRand, HAttrs, W, ipk.Hash, the "
                  "G1/G2 RawBytes encodings and HashToZr (tests/test_idemix.py issuer-key proof). The [EXT] "
                  "choices a real Go-made NymSignature would confirm or refute: the 2-byte transcript tail "
                  "(proofData sized for 65-byte points, dev/idemix.h NymCurve<fp>::TAIL), ProofC >= r never "
                  "matching (host/idemix.cpp), and Nonce >= 2^256 mapped to a recovered panic "
                  "(FTZ_ERR_SIGNATURE).",
        "ext_assumptions": {
            "nym_signature": "IBM/idemix NymSignature.Ver over mathlib BN254: t = HSk^SSk HRand^SRNym Nym^-C, "
                             "c = HashToZr('sign'||t||Nym||ipk.Hash@132||msg@164||00 00) "
                             "(proofData sized for 65-byte G1s), C == HashToZr(c||Nonce)",
            "g1_bytes": "gnark RawBytes X||Y (64 bytes); infinity 64 zero bytes",
            "g1_from_proto": "Gurvy translator: exactly 32-byte X and Y, gnark SetBytes(X||Y) behind recover",
            "nym_import": "NymX||NymY split at len/2 into G1FromProto (64-byte total only)",
            "zr_from_bytes": "big.Int SetBytes over the whole field, unreduced; Mul uses k mod r; "
                             "Bytes() of a value >= 2^256 panics (recovered)",
            "audit": "AuditNymEid: EidNym via G1FromProto (error, not panic) before the RNymEid use",
        },
        "ipk": ipk_raw.hex(),
        "isk": isk_raw.hex(),
        "credential": {"sk": "%064x" % sk, "attrs": ["%064x" % a for a in attrs], "s": "%064x" % s_cred,
                       "e": "%064x" % e_cred, "A": C.g1_bytes(A).hex(), "B": C.g1_bytes(B).hex(),
                       "attr_strings": {"ou": ou_s.decode(), "enrollment_id": eid_s.decode()}},
        "cases": cases,
        "audit_cases": audits,
        "bench": bench,
    }
    path = os.path.join(HERE, "idemix_bn254_golden.json")
    json.dump(out, open(path, "w"), indent=1)
    print("wrote", path, len(cases), "cases;", sum(c["expect"] == 0 for c in cases), "accept;",
          len(audits), "audit cases;", sum(c["expect"] == 0 for c in audits), "match")


if __name__ == "__main__":
    main()

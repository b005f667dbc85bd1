#!/usr/bin/env python3
"""Fixture maker for idemix owner-signature verification (tests/golden/idemix_golden.json).

Reference data (copied as data, read here only): the idemix IssuerPublicKey and
the user SignerConfig of the reference's validator tests
(token/core/zkatdlog/crypto/validator/testdata/idemix/{msp/IssuerPublicKey,
user/SignerConfig}).  The fixture records the pins the oracle must reproduce
(every IPK point on FP256BN, IPK Hash = HashToZr(proto without Hash), the
credential's B = G + sk HSk + S HRand + sum attr_i HAttrs_i) and a corpus of
owner identities / messages / NymSignatures made with the oracle's restated
NewNymSignature from the SignerConfig's secret key, with the oracle's verdicts.

    python tests/golden/make_idemix.py
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle", "py"))
from ftsoracle import idemix as I  # noqa: E402

REF = "/root/reference/token/core/zkatdlog/crypto/validator/testdata/idemix"


def expand(seed, n):
    """message bytes of a bench entry: SHA-256(seed || counter) blocks (bench.py repeats this)"""
    out = bytearray()
    k = 0
    while len(out) < n:
        out += hashlib.sha256(seed + k.to_bytes(4, "big")).digest()
        k += 1
    return bytes(out[:n])


IPK_FILES = ["token/core/zkatdlog/crypto/validator/testdata/idemix/msp/IssuerPublicKey",
             "token/core/zkatdlog/crypto/testdata/idemix/msp/IssuerPublicKey",
             "token/core/zkatdlog/crypto/audit/testdata/idemix/msp/IssuerPublicKey",
             "cmd/tokengen/testdata/idemix/msp/IssuerPublicKey",
             "cmd/tokengen/testdata/idemix/ca/IssuerPublicKey"]


def ipk_fixtures():
    out = []
    for rel in IPK_FILES:
        raw = open(os.path.join("/root/reference", rel), "rb").read()
        ok, why = I.issuer_key_check(raw)
        ok2, why2 = I.issuer_key_check_bn254(raw)
        f = {"path": rel, "raw": raw.hex(), "check_ok": ok, "why": why, "check_bn254_ok": ok2, "why_bn254": why2}
        isk = os.path.join("/root/reference", os.path.dirname(rel), "IssuerSecretKey")
        if os.path.exists(isk):  # cmd/tokengen/testdata/idemix/ca holds the issuer's secret key too
            f["isk"] = open(isk, "rb").read().hex()
        out.append(f)
    return out


def main():
    ipk_raw = open(os.path.join(REF, "msp", "IssuerPublicKey"), "rb").read()
    sc = I.pb_decode(open(os.path.join(REF, "user", "SignerConfig"), "rb").read(),
                     {1: "bytes", 2: "bytes", 3: "string", 4: "enum", 5: "string"})
    cred = I.pb_decode(sc[1], {1: ("msg", I.ECP_S), 2: ("msg", I.ECP_S), 3: "bytes", 4: "bytes", 5: "*bytes"})
    sk = int.from_bytes(sc[2], "big")
    ipk = I.IssuerPK(ipk_raw)
    rng = random.Random(0x1DE)

    def rz():
        return rng.randrange(1, I.N)

    ou = I.pb_field(1, 2, b"idemix") + I.pb_field(2, 2, sc[3]) + I.pb_field(3, 2, b"")
    role = I.pb_field(1, 2, b"idemix") + I.pb_field(2, 0, 2)

    def identity(nym, **kw):
        kw.setdefault("ou", ou)
        kw.setdefault("role", role)
        return I.serialize_idemix_identity(nym, **kw)

    def owner(ident, typ=b"si", tag=0x13):
        return I.raw_owner_encode(typ, ident, tag)

    cases = []

    def add(name, own, msg, sig):
        code, text = I.owner_verify(ipk, own, msg, sig)
        cases.append({"name": name, "owner": own.hex(), "msg": msg.hex(), "sig": sig.hex(), "expect": code,
                      "text": text})

    # valid signatures over messages of every SHA-256 block position
    users = []
    for k in range(4):
        rn = rz()
        nym = I.make_nym(ipk, sk, rn)
        users.append((rn, nym))
    for L in (0, 1, 25, 26, 27, 55, 56, 63, 64, 65, 100, 1000, 5000, 20000):
        rn, nym = users[L % 4]
        msg = bytes(rng.randrange(256) for _ in range(L))
        sig = I.nym_sign(ipk, sk, rn, nym, msg, rz(), rz(), rz())
        add("valid_len_%d" % L, owner(identity(nym)), msg, sig)

    rn, nym = users[0]
    msg = bytes(rng.randrange(256) for _ in range(300))
    sig_ok = I.nym_sign(ipk, sk, rn, nym, msg, rz(), rz(), rz())
    f = I.pb_decode(sig_ok, I.NYMSIG_S)
    own = owner(identity(nym))

    def sigf(vals, extra=b""):
        return b"".join(I.pb_field(k + 1, 2, v) for k, v in enumerate(vals)) + extra

    vals = [f[1], f[2], f[3], f[4]]
    # ---- signature tampering
    for idx, nm in enumerate(("proof_c", "s_sk", "s_rnym", "nonce")):
        v = list(vals)
        b = bytearray(v[idx])
        b[31] ^= 1
        v[idx] = bytes(b)
        add("flip_%s" % nm, own, msg, sigf(v))
    add("wrong_message", own, msg + b"x", sig_ok)
    add("other_users_nym", owner(identity(users[1][1])), msg, sig_ok)
    add("long_fields_tail_ignored", own, msg, sigf([v + b"\xff\x00" for v in vals]))
    add("short_proof_c", own, msg, sigf([vals[0][:31]] + vals[1:]))
    add("short_nonce", own, msg, sigf(vals[:3] + [vals[3][:16]]))
    add("missing_nonce", own, msg, sigf(vals[:3]))
    add("empty_signature", own, msg, b"")
    add("unknown_field_skipped", own, msg, sig_ok + I.pb_field(9, 2, b"junk") + I.pb_field(12, 0, 7))
    add("duplicate_field_last_wins", own, msg, I.pb_field(1, 2, bytes(32)) + sig_ok)
    add("wrong_wiretype_is_unknown", own, msg, I.pb_field(1, 0, 5) + sig_ok)
    add("only_varint_proof_c", own, msg, I.pb_field(1, 0, 5) + sigf([b"", vals[1], vals[2], vals[3]])[2:])
    add("group_skipped", own, msg, bytes([(7 << 3) | 3, (1 << 3) | 0, 1, (7 << 3) | 4]) + sig_ok)
    add("stray_end_group", own, msg, sig_ok + bytes([(7 << 3) | 4]))
    add("reserved_wiretype", own, msg, sig_ok + bytes([(7 << 3) | 7]))
    add("field_number_zero", own, msg, bytes([0x02, 0x00]) + sig_ok)
    add("truncated_signature", own, msg, sig_ok[:-5])
    add("varint_overflow", own, msg, sig_ok + bytes([(9 << 3)] + [0xff] * 9 + [0x02]))
    nonce_big = (1 << 256) - 1 - rng.randrange(1 << 200)  # raw nonce >= n is hashed as-is
    add("nonce_unreduced_accepts", own, msg, I.nym_sign(ipk, sk, rn, nym, msg, rz(), rz(), nonce_big))
    # ---- owner identity
    add("htlc_owner_unsupported", owner(b"{}", typ=b"htlc"), msg, sig_ok)
    add("unknown_owner_type", owner(identity(nym), typ=b"xx"), msg, sig_ok)
    add("raw_owner_utf8string", owner(identity(nym), tag=0x0C), msg, sig_ok)
    add("raw_owner_ia5string", owner(identity(nym), tag=0x16), msg, sig_ok)
    add("raw_owner_bmpstring", I._der(0x30, I._der(0x1E, "si".encode("utf-16-be")) + I._der(0x04, identity(nym))),
        msg, sig_ok)
    add("raw_owner_trailing_bytes", own + b"\x00\x01", msg, sig_ok)
    add("raw_owner_extra_element", I._der(0x30, I._der(0x13, b"si") + I._der(0x04, identity(nym)) + I._der(0x02, b"\x01")),
        msg, sig_ok)
    add("raw_owner_truncated", own[:-3], msg, sig_ok)
    add("raw_owner_octet_type", I._der(0x30, I._der(0x04, b"si") + I._der(0x04, identity(nym))), msg, sig_ok)
    add("raw_owner_bad_printable", owner(identity(nym), typ=b"s!"), msg, sig_ok)
    add("identity_not_proto", owner(b"\x0a\xff"), msg, sig_ok)
    add("mspid_invalid_utf8", owner(I.pb_field(1, 2, b"\xff\xfe") + I.pb_field(2, 2, b"")), msg, sig_ok)
    x, y = nym[0].to_bytes(32, "big"), nym[1].to_bytes(32, "big")
    inner_nox = I.pb_field(2, 2, y)
    add("nym_x_missing", owner(I.pb_field(1, 2, b"idemix") + I.pb_field(2, 2, inner_nox)), msg, sig_ok)
    add("nym_x_empty_is_nil", owner(identity(nym, nymx=b"", nymy=x + y)), msg, sig_ok)
    inner_twice = I.pb_field(1, 2, x) + I.pb_field(2, 2, y) + I.pb_field(1, 2, b"")
    add("nym_x_last_value_empty_is_nil", owner(I.pb_field(1, 2, b"idemix") + I.pb_field(2, 2, inner_twice)),
        msg, sig_ok)
    add("nym_short_halves", owner(identity(nym, nymx=x[:31], nymy=y[:31])), msg, sig_ok)
    add("nym_33_byte_halves", owner(identity(nym, nymx=b"\x00" + x, nymy=b"\x00" + y)), msg, sig_ok)
    add("nym_off_curve", owner(identity(nym, nymy=(nym[1] ^ 1).to_bytes(32, "big"))), msg, sig_ok)
    add("ou_not_proto", owner(identity(nym, ou=b"\x0a\x05ab")), msg, sig_ok)
    add("ou_invalid_utf8", owner(identity(nym, ou=I.pb_field(2, 2, b"\xc0\xaf"))), msg, sig_ok)
    add("role_not_proto", owner(identity(nym, role=b"\x10")), msg, sig_ok)
    add("role_unknown_enum_value", owner(identity(nym, role=I.pb_field(2, 0, 77))), msg, sig_ok)
    # [EXT] an off-curve nym is the point at infinity (amcl NewECPbigs): a
    # signature made against it without any secret verifies
    off = identity(nym, nymy=(nym[1] ^ 1).to_bytes(32, "big"))
    ssk, sr, nonce = rz(), rz(), rz()
    t = I.add(I.mul(ipk.hsk, ssk), I.mul(ipk.hrand, sr))
    c = I.hash_to_zr(I._proof_data(t, None, ipk.hash, msg))
    pc = I.hash_to_zr(c.to_bytes(32, "big") + nonce.to_bytes(32, "big"))
    add("off_curve_nym_forgery_accepts", owner(off), msg, sigf([v.to_bytes(32, "big") for v in (pc, ssk, sr, nonce)]))

    # bench workload (bench.py owner_signatures leg): 32 requests of ~9.5 KB (the
    # size of asn1(TokenRequest) for one 2-in/2-out transfer action), each signed by
    # two input owners; messages are expanded from a seed so the fixture stays small
    bench = []
    for r in range(32):
        seed = bytes([r]) * 8
        msg = expand(seed, 9500)
        for u in range(2):
            rn, nym = users[(r + u) % 4]
            sig = I.nym_sign(ipk, sk, rn, nym, msg, rz(), rz(), rz())
            bench.append({"owner": owner(identity(nym)).hex(), "msg_seed": seed.hex(), "msg_len": len(msg),
                          "sig": sig.hex()})

    # auditor owner match (ftz_audit_owners): AuditInfo JSON + owner identities whose
    # proof carries an EidNym, with the oracle's verdicts (idemix.audit_owner_match)
    arng = random.Random(0xA0D1)
    eid = pins_eid = sc[5]
    audits = []

    def aadd(name, own, ai):
        code, text = I.audit_owner_match(ipk, own, ai)
        audits.append({"name": name, "owner": own.hex(), "audit_info": ai.hex(), "expect": code, "text": text})
    attrs = [sc[3], b"role", eid, b"rh"]
    for u in range(3):
        r_eid = arng.randrange(1, I.N)
        ne = I.add(I.mul(ipk.hattrs[2], I.hash_to_zr(eid)), I.mul(ipk.hrand, r_eid))
        own = owner(identity(users[u][1], proof=I.signature_with_eid_nym(ne)))
        aadd("eid_match_%d" % u, own, I.audit_info_encode(r_eid, I.hash_to_zr(eid), attrs))
    r_eid = arng.randrange(1, I.N)
    ne = I.add(I.mul(ipk.hattrs[2], I.hash_to_zr(eid)), I.mul(ipk.hrand, r_eid))
    good_proof = I.signature_with_eid_nym(ne)
    own = owner(identity(nym, proof=good_proof))
    ai = I.audit_info_encode(r_eid, I.hash_to_zr(eid), attrs)
    r_u = arng.randrange(1, (1 << 256) - I.N)
    ne_u = I.add(I.mul(ipk.hattrs[2], I.hash_to_zr(eid)), I.mul(ipk.hrand, r_u))
    aadd("eid_match_unreduced_rnym", owner(identity(nym, proof=I.signature_with_eid_nym(ne_u))),
         I.audit_info_encode(r_u + I.N, 0, attrs))
    aadd("eid_other_enrollment_id", own, I.audit_info_encode(r_eid, 0, [attrs[0], attrs[1], b"mallory", attrs[3]]))
    aadd("eid_wrong_rnym", own, I.audit_info_encode(r_eid + 1, 0, attrs))
    aadd("eid_nym_of_other_identity", owner(identity(nym, proof=I.signature_with_eid_nym(I.mul(ipk.hrand, 5)))), ai)
    off = (ne[0], (ne[1] + 1) % I.Q)
    aadd("eid_nym_off_curve", owner(identity(nym, proof=I.signature_with_eid_nym(off))), ai)
    full = (I.pb_field(1, 2, I.pb_field(1, 2, bytes(32)) + I.pb_field(2, 2, bytes(32))) + I.pb_field(4, 2, bytes(32))
            + I.pb_field(10, 2, b"a") + I.pb_field(10, 2, b"b") + I.pb_field(16, 0, 7)
            + I.pb_field(17, 2, I.pb_field(1, 0, 1) + I.pb_field(2, 2, b"x")))
    aadd("eid_full_signature_proto", owner(identity(nym, proof=I.signature_with_eid_nym(ne, extra=full))), ai)
    aadd("eid_no_eid_nym", owner(identity(nym, proof=full)), ai)
    aadd("eid_bad_signature_proto", owner(identity(nym, proof=b"\x0a\x05ab")), ai)
    aadd("eid_bad_ecp_inside_signature", owner(identity(nym, proof=I.pb_field(1, 2, b"\x0a\x09") + good_proof)), ai)
    aadd("eid_short_nym_coordinate", owner(identity(nym, proof=I.pb_field(18, 2, I.pb_field(1, 2, I.pb_field(1, 2, b"\x01" * 31) + I.pb_field(2, 2, bytes(32)))))), ai)
    aadd("eid_attributes_too_short_panics", own, I.audit_info_encode(r_eid, 0, attrs[:2]))
    aadd("eid_null_audit_info_panics", own, b"null")
    aadd("eid_nil_rnym_panics", own, I.audit_info_encode(None, 0, attrs))
    aadd("eid_foreign_curve_panics", own, I.audit_info_encode(r_eid, 0, attrs, curve=1))
    aadd("audit_info_not_json", own, b"{oops")
    aadd("audit_info_array", own, b"[]")
    aadd("audit_info_bad_attribute", own, ai.replace(b'"Attributes":[', b'"Attributes":[1,'))
    aadd("audit_info_empty", own, b"")
    aadd("redeem_token", b"", ai)
    aadd("owner_not_asn1", b"\x30\x05", ai)
    aadd("htlc_owner_script", owner(b"script", typ=b"htlc"), ai)
    aadd("identity_not_proto", owner(b"\x0a\xff"), ai)
    aadd("idemix_identity_not_proto", owner(I.pb_field(1, 2, b"idemix") + I.pb_field(2, 2, b"\x0a\xff")), ai)
    aadd("audit_info_lowercase_keys", own, ai.replace(b'"RNymEid"', b'"rnymeid"').replace(b'"Attributes"', b'"attributes"'))

    out = {
        "comment": "idemix owner signatures on FP256BN (SURVEY 8(f) row 3); made by make_idemix.py",
        "ext_assumptions": {
            "nym_signature": "IBM/idemix NymSignature.Ver: t = HSk^SSk HRand^SRNym Nym^-C, "
                             "c = HashToZr('sign'||t||Nym||ipk.Hash[32 slot]||msg), C == HashToZr(c||Nonce)",
            "g1_bytes": "amcl ECP.ToBytes(false): 0x04||X||Y (65 bytes); infinity 0x04||0^32||1",
            "zr_from_bytes": "amcl FromBytes: first 32 bytes big-endian, unreduced; shorter panics (recovered)",
            "nym_import": "NymX||NymY split at len/2; NewECPbigs: coords mod q, off-curve -> infinity",
            "protobuf": "google.golang.org/protobuf v1.27.1 proto3 decoding (unknown skipped, last wins, "
                        "wrong wire type = unknown, UTF-8 strings)",
        },
        "ipk": ipk_raw.hex(),
        # every IssuerPublicKey file the reference holds, with IssuerPublicKey.Check's
        # verdict (ftsoracle.idemix.issuer_key_check): the proof pins the G2
        # generator, G1/G2 byte layouts and HashModOrder against reference bytes
        "ipk_fixtures": ipk_fixtures(),
        "pins": {
            "sk": sc[2].hex(),
            "cred_b": [cred[2][1].hex(), cred[2][2].hex()],
            "cred_s": cred[4].hex(),
            "cred_attrs": [a.hex() for a in cred[5]],
            "attr_strings": {"ou": sc[3].decode(), "enrollment_id": sc[5].decode()},
        },
        "cases": cases,
        "audit_cases": audits,
        "bench": bench,
    }
    path = os.path.join(HERE, "idemix_golden.json")
    json.dump(out, open(path, "w"), indent=1)
    print("wrote", path, len(cases), "cases;", sum(c["expect"] == 0 for c in cases), "accept")


if __name__ == "__main__":
    main()

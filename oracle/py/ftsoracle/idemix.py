"""TEST INFRASTRUCTURE ONLY -- oracle restatement of idemix owner-signature
verification; nothing in the product imports it.

The reference path (paths relative to /root/reference/token/core/):
* zkatdlog/crypto/validator/validator_transfer.go:42-82 TransferSignatureValidate:
  for every input token, ctx.Deserializer.GetOwnerVerifier(tok.Owner) and
  ctx.SignatureProvider.HasBeenSignedBy(tok.Owner, verifier), i.e.
  verifier.Verify(message, sigma) (common/backend.go:32-41);
* zkatdlog/nogh/deserializer.go:45-66: the owner deserializer is
  htlc.NewDeserializer(identity.NewRawOwnerIdentityDeserializer(idemixDes));
  interop/htlc/deserializer.go:31-43 dispatches on RawOwner.Type ("si" ->
  identity/owner.go:62-68 -> idemix, "htlc" -> an HTLC script, anything else an
  error); RawOwner is Go encoding/asn1 of struct{Type string; Identity []byte}
  (identity/owner.go:23-37);
* identity/msp/idemix/deserializer.go:83-95 DeserializeVerifier ->
  common.go:36-117 Deserialize(raw, checkValidity=false): proto
  msp.SerializedIdentity, then msp.SerializedIdemixIdentity (NymX, NymY must be
  non-nil), the nym public key imported from NymX||NymY, OU and Role protos;
* deserializer.go:153-163 Verifier.Verify -> CSP.Verify(NymPK, sigma, msg,
  IdemixNymSignerOpts{IssuerPK}) -> IBM/idemix NymSignature.Ver.

[EXT] IBM/idemix v0.0.0-20220113150823-80dd4cb2d74e, IBM/mathlib
v0.0.0-20220112091634-0a7378db6912 (go.mod:6-7) and hyperledger/fabric-amcl
(go.mod:101) are not vendored; what follows restates their published
algorithms:
* NymSignature.Ver: t = HSk^ProofSSk * HRand^ProofSRNym * Nym^-ProofC;
  c = HashToZr("sign" || t || Nym || ipk.Hash || msg) (G1 as 65 bytes
  0x04||X||Y, ipk.Hash in a 32-byte slot, proofData of length
  4 + 2*65 + 32 + len(msg)); accept iff ProofC == HashToZr(c || Nonce)
  (32-byte big-endian each); error text "pseudonym signature invalid:
  zero-knowledge proof is invalid".
* Zr from bytes is amcl FromBytes: the first 32 bytes, big-endian, NOT reduced
  (a shorter slice panics; the bridge recovers and returns an error);
  Equals compares the raw integers; G1 Mul by an unreduced scalar = (k mod n) P.
* The nym public key: raw = NymX || NymY, halves at len(raw)/2, each read by
  FromBytes; amcl NewECPbigs reduces the coordinates mod q and yields the point
  at infinity when (x, y) is not on the curve; infinity serialises as
  0x04 || 0^32 || 1 (amcl's (0, 1, 0) representative) [EXT, unpinned].
* HashToZr = SHA-256 read big-endian, mod n (pinned: the reference's
  IssuerPublicKey fixture carries Hash = HashToZr(proto without Hash)).
* Protobuf (golang/protobuf v1.5.2 over google.golang.org/protobuf v1.27.1,
  go.mod:10,226): proto3 decoding with unknown fields skipped, last value wins,
  a known field with the wrong wire type handled as unknown, strings validated
  as UTF-8.  A proto3 (no-presence) bytes field decodes through
  consumeBytesNoZero, append([]byte(nil), v...): an EMPTY value, even when it
  is on the wire, leaves the field nil -- so NymX / NymY of length 0 fail the
  common.go:52 nil check.
"""
import hashlib

from . import request as RQ

# FP256BN (x = -0x6882F5C030B0A801; pinned by tests/test_idemix.py against the
# reference's idemix fixtures)
Q = 0xFFFFFFFFFFFCF0CD46E5F25EEE71A49F0CDC65FB12980A82D3292DDBAED33013
N = 0xFFFFFFFFFFFCF0CD46E5F25EEE71A49E0CDC65FB1299921AF62D536CD10B500D
B = 3
G = (1, 2)
FIELD_BYTES = 32
SIGN_LABEL = b"sign"

OK = 0
ERR_OWNER = 9        # the owner identity does not deserialize
ERR_SIGNATURE = 10   # the signature does not unmarshal / pseudonym signature invalid
ERR_UNSUPPORTED = 11  # owner type handled in Go (HTLC script)
ERR_PANIC = 6


# ------------------------------------------------------------------ G1 (affine)
def on_curve(P):
    return P is None or (P[1] * P[1] - P[0] ** 3 - B) % Q == 0


def add(P, R):
    if P is None:
        return R
    if R is None:
        return P
    if P[0] == R[0]:
        if (P[1] + R[1]) % Q == 0:
            return None
        lam = 3 * P[0] * P[0] * pow(2 * P[1], -1, Q) % Q
    else:
        lam = (R[1] - P[1]) * pow(R[0] - P[0], -1, Q) % Q
    x = (lam * lam - P[0] - R[0]) % Q
    return (x, (lam * (P[0] - x) - P[1]) % Q)


def neg(P):
    return None if P is None else (P[0], (-P[1]) % Q)


def mul(P, k):
    k %= N
    acc, cur = None, P
    while k:
        if k & 1:
            acc = add(acc, cur)
        cur = add(cur, cur)
        k >>= 1
    return acc


def g1_bytes(P):
    """amcl ECP.ToBytes(b, false) as mathlib's G1.Bytes calls it: 65 bytes."""
    if P is None:
        return b"\x04" + bytes(32) + (1).to_bytes(32, "big")  # [EXT] infinity
    return b"\x04" + P[0].to_bytes(32, "big") + P[1].to_bytes(32, "big")


def hash_to_zr(data):
    return int.from_bytes(hashlib.sha256(data).digest(), "big") % N


# ------------------------------------------------------------------ protobuf
class PbError(Exception):
    pass


def _varint(b, i):
    v = 0
    for k in range(10):
        if i >= len(b):
            raise PbError("unexpected EOF")
        c = b[i]
        i += 1
        if k == 9 and c > 1:
            raise PbError("variable length integer overflow")
        v |= (c & 0x7F) << (7 * k)
        if c < 0x80:
            return v, i
    raise PbError("variable length integer overflow")


def _skip(b, i, num, wt, depth=0):
    if wt == 0:
        return _varint(b, i)[1]
    if wt == 1:
        if len(b) - i < 8:
            raise PbError("unexpected EOF")
        return i + 8
    if wt == 5:
        if len(b) - i < 4:
            raise PbError("unexpected EOF")
        return i + 4
    if wt == 2:
        n, i = _varint(b, i)
        if n > len(b) - i:
            raise PbError("unexpected EOF")
        return i + n
    if wt == 3:
        while True:
            if i >= len(b):
                raise PbError("unexpected EOF")
            tag, i = _varint(b, i)
            n2, w2 = tag >> 3, tag & 7
            if n2 < 1 or n2 > (1 << 29) - 1:
                raise PbError("invalid field number")
            if w2 == 4:
                if n2 != num:
                    raise PbError("mismatching end group marker")
                return i
            i = _skip(b, i, n2, w2, depth + 1)
    raise PbError("cannot parse reserved wire type")


def _utf8(v):
    try:
        v.decode("utf-8", errors="strict")
    except UnicodeDecodeError:
        raise PbError("string field contains invalid UTF-8")
    return v


def pb_decode(b, schema):
    """schema: {num: kind} with kind in 'bytes', 'string', 'enum', ('msg', schema),
    and a leading '*' for repeated.  Returns {num: value | [values]}."""
    out = {}
    i = 0
    while i < len(b):
        tag, i = _varint(b, i)
        num, wt = tag >> 3, tag & 7
        if num < 1 or num > (1 << 29) - 1:
            raise PbError("invalid field number")
        if wt == 4:
            raise PbError("unexpected end group")
        kind = schema.get(num)
        rep = isinstance(kind, str) and kind.startswith("*") or isinstance(kind, tuple) and kind[0] == "*msg"
        base = kind[1:] if isinstance(kind, str) and kind.startswith("*") else kind
        want = None if kind is None else (0 if base == "enum" else 2)
        if kind is None or wt != want:
            i = _skip(b, i, num, wt)
            continue
        if base == "enum":
            v, i = _varint(b, i)
            v &= 0xFFFFFFFF
            val = v - (1 << 32) if v >= 1 << 31 else v
        else:
            n, i = _varint(b, i)
            if n > len(b) - i:
                raise PbError("unexpected EOF")
            raw = bytes(b[i:i + n])
            i += n
            if base == "bytes":
                val = raw
            elif base == "string":
                val = _utf8(raw)
            else:  # message
                sub = base[1]
                val = pb_decode(raw, sub)
                if not rep and num in out:  # singular message seen twice: merge
                    merged = dict(out[num])
                    for k2, v2 in val.items():
                        if isinstance(v2, list):
                            merged[k2] = merged.get(k2, []) + v2
                        elif isinstance(v2, dict) and isinstance(merged.get(k2), dict):
                            m2 = dict(merged[k2])
                            m2.update(v2)
                            merged[k2] = m2
                        else:
                            merged[k2] = v2
                    val = merged
        if rep:
            out.setdefault(num, []).append(val)
        else:
            out[num] = val
    return out


def pb_field(num, wt, payload):
    """encoder for fixtures: one field"""
    def vi(v):
        o = bytearray()
        while True:
            c = v & 0x7F
            v >>= 7
            if v:
                o.append(c | 0x80)
            else:
                o.append(c)
                return bytes(o)
    if wt == 0:
        return vi(num << 3) + vi(payload)
    return vi((num << 3) | 2) + vi(len(payload)) + payload


ECP_S = {1: "bytes", 2: "bytes"}
ECP2_S = {1: "bytes", 2: "bytes", 3: "bytes", 4: "bytes"}
IPK_S = {1: "*string", 2: ("msg", ECP_S), 3: ("msg", ECP_S), 4: ("*msg", ECP_S), 5: ("msg", ECP2_S),
         6: ("msg", ECP_S), 7: ("msg", ECP_S), 8: "bytes", 9: "bytes", 10: "bytes"}
SERIALIZED_IDENTITY_S = {1: "string", 2: "bytes"}                          # msp.SerializedIdentity
SERIALIZED_IDEMIX_S = {1: "bytes", 2: "bytes", 3: "bytes", 4: "bytes", 5: "bytes"}  # NymX NymY Ou Role Proof
OU_S = {1: "string", 2: "string", 3: "bytes"}                                # msp.OrganizationUnit
ROLE_S = {1: "string", 2: "enum"}                                            # msp.MSPRole
NYMSIG_S = {1: "bytes", 2: "bytes", 3: "bytes", 4: "bytes"}                 # ProofC ProofSSk ProofSRNym Nonce


def from_bytes32(b):
    """amcl FromBytes: the first 32 bytes big-endian; a shorter slice panics."""
    if b is None or len(b) < 32:
        raise IndexError("index out of range")
    return int.from_bytes(b[:32], "big")


def ecp_from_bytes(x, y):
    """amcl NewECPbigs(FromBytes(x), FromBytes(y)): coordinates mod q, off-curve -> infinity."""
    P = (from_bytes32(x) % Q, from_bytes32(y) % Q)
    return P if on_curve(P) else None


class IssuerPK:
    def __init__(self, raw):
        m = pb_decode(raw, IPK_S)
        self.raw = raw
        self.hsk = ecp_from_bytes(m[2].get(1), m[2].get(2))
        self.hrand = ecp_from_bytes(m[3].get(1), m[3].get(2))
        self.hattrs = [ecp_from_bytes(e.get(1), e.get(2)) for e in m.get(4, [])]
        self.bar_g1 = ecp_from_bytes(m[6].get(1), m[6].get(2))
        self.bar_g2 = ecp_from_bytes(m[7].get(1), m[7].get(2))
        self.hash = m.get(10, b"")
        self.fields = m


# ------------------------------------------------------------------ G2 (issuer key proof)
# amcl FP256BN: Fp2 = Fp[i]/(i^2 + 1); G2 lives on the M-type sextic twist
# y^2 = x^3 + 3(1 + i) (every reference IssuerPublicKey W satisfies it).
B2 = (3, 3)
H2 = 2 * Q - N  # #E'(Fp2) / n for the BN sextic twist
# amcl ECP2_generator() (CURVE_Pxa, Pxb, Pya, Pyb).  amcl's ROM is not in the
# reference; the point is RECOVERED, not assumed: it is H2 * (1, y0) with x = 1
# the first twist abscissa, and of the two roots y0 exactly one makes
# issuer_key_check() accept all three reference IssuerPublicKey fixtures -- a
# SHA-256 match over 579 reference-held bytes, so a wrong generator could not
# pass (tests/test_idemix.py::test_issuer_key_proof_pins_g2_and_transcript).
GEN_G2 = ((0xFE0C3350B4C96C2028560F577C28913ACE1C539A12BF843CD22616B689C09EFB,
           0x4EA66057738AC054DB5AE1C637D813B924DD78E287D03589D269ED34A37E6A2B),
          (0x702046E7C542A3B376770D75124E3E51EFCB24758D615848E909B481BEDC27FF,
           0x0554E3BCD388C29042EEA649297EB29F8B4CBE80821A98B3E01281114AAD049B))


def _f2m(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % Q, (a[0] * b[1] + a[1] * b[0]) % Q)


def _f2a(a, b):
    return ((a[0] + b[0]) % Q, (a[1] + b[1]) % Q)


def _f2s(a, b):
    return ((a[0] - b[0]) % Q, (a[1] - b[1]) % Q)


def _f2i(a):
    d = pow((a[0] * a[0] + a[1] * a[1]) % Q, -1, Q)
    return (a[0] * d % Q, -a[1] * d % Q)


def g2_on_curve(P):
    return P is None or _f2s(_f2m(P[1], P[1]), _f2m(P[0], _f2m(P[0], P[0]))) == B2


def g2_add(P, R):
    if P is None:
        return R
    if R is None:
        return P
    if P[0] == R[0]:
        if _f2a(P[1], R[1]) == (0, 0):
            return None
        lam = _f2m(_f2m((3, 0), _f2m(P[0], P[0])), _f2i(_f2m((2, 0), P[1])))
    else:
        lam = _f2m(_f2s(R[1], P[1]), _f2i(_f2s(R[0], P[0])))
    x = _f2s(_f2s(_f2m(lam, lam), P[0]), R[0])
    return (x, _f2s(_f2m(lam, _f2s(P[0], x)), P[1]))


def g2_mul(P, k):
    acc = None
    for bit in bin(k)[2:] if k > 0 else "":
        acc = g2_add(acc, acc)
        if bit == "1":
            acc = g2_add(acc, P)
    return acc


def g2_bytes(P):
    """amcl ECP2.ToBytes as mathlib's G2.Bytes calls it: 128 bytes Xa||Xb||Ya||Yb
    (infinity as amcl's affine (0, 0) representative [EXT, unreached])."""
    (xa, xb), (ya, yb) = P if P is not None else ((0, 0), (0, 0))
    return b"".join(v.to_bytes(32, "big") for v in (xa, xb, ya, yb))


def ecp2_from_proto(e):
    """amcl NewECP2fp2s(FP2(FromBytes(Xa), FromBytes(Xb)), FP2(FromBytes(Ya), FromBytes(Yb))):
    off-curve -> infinity (as NewECPbigs in G1)."""
    P = ((from_bytes32(e.get(1)) % Q, from_bytes32(e.get(2)) % Q),
         (from_bytes32(e.get(3)) % Q, from_bytes32(e.get(4)) % Q))
    return P if g2_on_curve(P) else None


def issuer_key_check(raw):
    """IBM/idemix IssuerPublicKey.Check (run when the deserializer imports the
    issuer key, identity/msp/idemix/deserializer.go:59-75): the key's own
    Schnorr proof of knowledge of isk with W = g2^isk and BarG2 = BarG1^isk.
        t1 = g2^ProofS * W^-ProofC,  t2 = BarG1^ProofS * BarG2^-ProofC,
        ProofC == HashModOrder(t1 || t2 || g2 || BarG1 || W || BarG2)
    with G2 as 128 bytes, G1 as 65 bytes (0x04||X||Y), proofData of 18*32+3 bytes.
    Returns (ok, why)."""
    try:
        m = pb_decode(raw, IPK_S)
    except PbError as e:
        return False, "failed to unmarshal issuer public key: %s" % e
    if any(m.get(k) is None for k in (2, 3, 5, 6, 7)):
        return False, "some part of the public key is undefined"
    try:
        bar_g1 = ecp_from_bytes(m[6].get(1), m[6].get(2))
        bar_g2 = ecp_from_bytes(m[7].get(1), m[7].get(2))
        w = ecp2_from_proto(m[5])
        proof_c, proof_s = from_bytes32(m.get(8)), from_bytes32(m.get(9))
    except IndexError as e:
        return False, "failure [%s]" % e
    if bar_g1 is None or len(m.get(4, [])) < len(m.get(1, [])):
        return False, "some part of the public key is undefined"
    neg_c = (N - proof_c % N) % N
    t1 = g2_add(g2_mul(GEN_G2, proof_s % N), g2_mul(w, neg_c))
    t2 = add(mul(bar_g1, proof_s), mul(bar_g2, neg_c))
    data = (g2_bytes(t1) + g1_bytes(t2) + g2_bytes(GEN_G2) + g1_bytes(bar_g1) + g2_bytes(w) + g1_bytes(bar_g2))
    assert len(data) == 18 * FIELD_BYTES + 3
    if proof_c != hash_to_zr(data):
        return False, "zero knowledge proof in public key invalid"
    return True, ""


def issuer_key_check_bn254(raw):
    """The same IssuerPublicKey.Check for an issuer key on BN254 (IBM/idemix
    with mathlib's BN254 curve and gurvy translator, as cmd/tokengen's testdata
    key is): points decoded with gnark SetBytes from the proto's coordinates
    (G1: X||Y; G2: Xa||Xb||Ya||Yb = gnark RawBytes X.A1||X.A0||Y.A1||Y.A0),
    g2 = gnark's G2 generator, the proof data appended with mathlib's Bytes()
    (gnark RawBytes: G1 64, G2 128 bytes) into the 18*32+3-byte buffer (576
    bytes used, 3 zero bytes left) and HashToZr = SHA-256 mod r over all of it.
    This is the encoding and hash the zkatdlog transcripts use (bn254.g1_bytes,
    g2_bytes, hash_to_zr), so the key pins them.  Returns (ok, why)."""
    from . import bn254 as C
    try:
        m = pb_decode(raw, IPK_S)
    except PbError as e:
        return False, "failed to unmarshal issuer public key: %s" % e
    if any(m.get(k) is None for k in (2, 3, 5, 6, 7)):
        return False, "some part of the public key is undefined"
    try:
        bar_g1 = C.g1_from_bytes((m[6].get(1) or b"") + (m[6].get(2) or b""))
        bar_g2 = C.g1_from_bytes((m[7].get(1) or b"") + (m[7].get(2) or b""))
        w = C.g2_from_bytes(b"".join(m[5].get(k) or b"" for k in (1, 2, 3, 4)))
    except C.DecodeError as e:
        return False, "failure [%s]" % e
    proof_c = int.from_bytes(m.get(8) or b"", "big")
    proof_s = int.from_bytes(m.get(9) or b"", "big")
    neg_c = (-proof_c) % C.R
    t1 = C.g2_add(C.g2_mul(C.G2_GEN, proof_s % C.R), C.g2_mul(w, neg_c))
    t2 = C.g1_add(C.g1_mul(bar_g1, proof_s), C.g1_mul(bar_g2, neg_c))
    data = (C.g2_bytes(t1) + C.g1_bytes(t2) + C.g2_bytes(C.G2_GEN) + C.g1_bytes(bar_g1) + C.g2_bytes(w)
            + C.g1_bytes(bar_g2))
    data += bytes(18 * 32 + 3 - len(data))
    if proof_c != C.hash_to_zr(data):
        return False, "zero knowledge proof in public key invalid"
    return True, ""


# ------------------------------------------------------------------ ASN.1 RawOwner
def _printable(c, amp_star=True):
    return (ord("a") <= c <= ord("z") or ord("A") <= c <= ord("Z") or ord("0") <= c <= ord("9")
            or c in b" '()+,-./:=?" or (amp_star and c in b"*&"))


def _asn1_string(tag, body):
    """Go 1.18 encoding/asn1 parseField for a string-typed field."""
    if tag == 0x13:  # PrintableString
        if not all(_printable(c) for c in body):
            raise RQ.Asn1Error("PrintableString contains invalid character")
        return body.decode("latin-1")
    if tag == 0x16:  # IA5String
        if any(c >= 0x80 for c in body):
            raise RQ.Asn1Error("IA5String contains invalid character")
        return body.decode("latin-1")
    if tag in (0x14, 0x1B):  # T61String, GeneralString: bytes as-is
        return body.decode("latin-1")
    if tag == 0x0C:  # UTF8String
        try:
            return body.decode("utf-8", errors="strict")
        except UnicodeDecodeError:
            raise RQ.Asn1Error("invalid UTF-8 string")
    if tag == 0x12:  # NumericString
        if not all(ord("0") <= c <= ord("9") or c == 0x20 for c in body):
            raise RQ.Asn1Error("NumericString contains invalid character")
        return body.decode("latin-1")
    if tag == 0x1E:  # BMPString
        if len(body) % 2:
            raise RQ.Asn1Error("odd-length BMP string")
        if len(body) >= 2 and body[-1] == 0 and body[-2] == 0:
            body = body[:-2]
        return body.decode("utf-16-be", errors="replace")
    raise RQ.Asn1Error("tags don't match")


def _asn1_len(b, off):
    if off >= len(b):
        raise RQ.Asn1Error("truncated tag or length")
    c = b[off]
    off += 1
    if c & 0x80 == 0:
        n = c
    else:
        nb = c & 0x7F
        if nb == 0:
            raise RQ.Asn1Error("indefinite length found (not DER)")
        n = 0
        for _ in range(nb):
            if off >= len(b):
                raise RQ.Asn1Error("truncated tag or length")
            if n >= 1 << 23:
                raise RQ.Asn1Error("length too large")
            n = (n << 8) | b[off]
            off += 1
            if n == 0:
                raise RQ.Asn1Error("superfluous leading zeros in length")
        if n < 0x80:
            raise RQ.Asn1Error("non-minimal length")
    if n > len(b) - off:
        raise RQ.Asn1Error("data truncated")
    return n, off


def _asn1_tag(b, off):
    if off >= len(b):
        raise RQ.Asn1Error("sequence truncated")
    t = b[off]
    if t & 0x1F == 0x1F:  # high-tag-number form: no universal string / octet tag fits
        raise RQ.Asn1Error("tags don't match")
    return t, off + 1


def raw_owner_decode(raw):
    """identity.UnmarshallRawOwner (identity/owner.go:30-37): (Type, Identity)."""
    t, off = _asn1_tag(raw, 0)
    if t != 0x30:
        raise RQ.Asn1Error("tags don't match")
    n, off = _asn1_len(raw, off)
    body = raw[off:off + n]
    k = 0
    t, k = _asn1_tag(body, k)
    n1, k = _asn1_len(body, k)
    typ = _asn1_string(t, body[k:k + n1])
    k += n1
    t, k = _asn1_tag(body, k)
    if t != 0x04:
        raise RQ.Asn1Error("tags don't match")
    n2, k = _asn1_len(body, k)
    ident = bytes(body[k:k + n2])
    return typ, ident


def _der(tag, body):
    n = len(body)
    if n < 0x80:
        ln = bytes([n])
    else:
        nb = (n.bit_length() + 7) // 8
        ln = bytes([0x80 | nb]) + n.to_bytes(nb, "big")
    return bytes([tag]) + ln + body


def raw_owner_encode(typ, ident, string_tag=0x13):
    """asn1.Marshal(RawOwner{...}) (PrintableString for printable Type)."""
    return _der(0x30, _der(string_tag, typ) + _der(0x04, ident))


# ------------------------------------------------------------------ idemix
def make_nym(ipk, sk, r_nym):
    """Nym = HSk^sk * HRand^RNym (IBM/idemix MakeNym)"""
    return add(mul(ipk.hsk, sk), mul(ipk.hrand, r_nym))


def _proof_data(t, nym, ipk_hash, msg):
    d = bytearray(len(SIGN_LABEL) + 2 * (2 * FIELD_BYTES + 1) + FIELD_BYTES + len(msg))
    idx = 0
    d[idx:idx + 4] = SIGN_LABEL
    idx += 4
    d[idx:idx + 65] = g1_bytes(t)
    idx += 65
    d[idx:idx + 65] = g1_bytes(nym)
    idx += 65
    h = ipk_hash[:len(d) - idx]
    d[idx:idx + len(h)] = h  # copy(proofData[index:], ipk.Hash)
    idx += FIELD_BYTES
    d[idx:] = msg
    return bytes(d)


def nym_sign(ipk, sk, r_nym, nym, msg, r_sk, r_rnym, nonce):
    """IBM/idemix NewNymSignature with injected randomness (r_sk, r_rnym, nonce):
    the NymSignature proto bytes."""
    t = add(mul(ipk.hsk, r_sk), mul(ipk.hrand, r_rnym))
    c = hash_to_zr(_proof_data(t, nym, ipk.hash, msg))
    proof_c = hash_to_zr(c.to_bytes(32, "big") + nonce.to_bytes(32, "big"))
    s_sk = (r_sk + proof_c * sk) % N
    s_rnym = (r_rnym + proof_c * r_nym) % N
    return b"".join(pb_field(k + 1, 2, v.to_bytes(32, "big")) for k, v in enumerate((proof_c, s_sk, s_rnym, nonce)))


def nym_verify(ipk, nym, sig, msg):
    """IBM/idemix NymSignature.Ver behind the bridge's recover: (code, text)."""
    if len(sig) == 0:
        return ERR_SIGNATURE, "invalid signature, it must not be empty"
    try:
        m = pb_decode(sig, NYMSIG_S)
    except PbError as e:
        return ERR_SIGNATURE, "error unmarshalling signature: %s" % e
    try:
        proof_c, s_sk, s_rnym, nonce = (from_bytes32(m.get(k)) for k in (1, 2, 3, 4))
    except IndexError as e:
        return ERR_SIGNATURE, "failure [%s]" % e
    t = add(add(mul(ipk.hsk, s_sk), mul(ipk.hrand, s_rnym)), neg(mul(nym, proof_c)))
    c = hash_to_zr(_proof_data(t, nym, ipk.hash, msg))
    if proof_c != hash_to_zr(c.to_bytes(32, "big") + nonce.to_bytes(32, "big")):
        return ERR_SIGNATURE, "pseudonym signature invalid: zero-knowledge proof is invalid"
    return OK, ""


def deserialize_idemix_identity(raw):
    """common.go:40-117 Deserialize(raw, false): the nym point, or (code, text)."""
    try:
        si = pb_decode(raw, SERIALIZED_IDENTITY_S)
    except PbError:
        return None, (ERR_OWNER, "failed to unmarshal to msp.SerializedIdentity{}")
    try:
        ser = pb_decode(si.get(2, b""), SERIALIZED_IDEMIX_S)
    except PbError:
        return None, (ERR_OWNER, "could not deserialize a SerializedIdemixIdentity")
    if not ser.get(1) or not ser.get(2):  # absent OR empty: proto3 bytes decode to nil when empty
        return None, (ERR_OWNER, "unable to deserialize idemix identity: pseudonym is invalid")
    raw_nym = ser[1] + ser[2]
    half = len(raw_nym) // 2
    try:
        nym = ecp_from_bytes(raw_nym[:half], raw_nym[half:])
    except IndexError:
        return None, (ERR_OWNER, "failed to import nym public key")
    try:
        pb_decode(ser.get(3, b""), OU_S)
    except PbError:
        return None, (ERR_OWNER, "cannot deserialize the OU of the identity")
    try:
        pb_decode(ser.get(4, b""), ROLE_S)
    except PbError:
        return None, (ERR_OWNER, "cannot deserialize the role of the identity")
    return nym, None


def owner_verify(ipk, owner, msg, sig):
    """One input of TransferSignatureValidate: GetOwnerVerifier(tok.Owner) then
    verifier.Verify(msg, sigma).  (code, text)."""
    try:
        typ, ident = raw_owner_decode(owner)
    except RQ.Asn1Error:
        return ERR_OWNER, "failed to unmarshal RawOwner"
    if typ == "htlc":
        return ERR_UNSUPPORTED, "htlc script owner: verified in Go"
    if typ != "si":
        return ERR_OWNER, "failed to deserialize RawOwner: Unknown owner type %s" % typ
    nym, err = deserialize_idemix_identity(ident)
    if err:
        return err
    return nym_verify(ipk, nym, sig, msg)


def serialize_idemix_identity(nym, mspid="idemix", ou=b"", role=b"", proof=b"", nymx=None, nymy=None):
    """msp.SerializedIdentity{Mspid, IdBytes: SerializedIdemixIdentity{NymX, NymY, Ou, Role, Proof}}
    (identity/msp/idemix/id.go Serialize) for fixtures."""
    x = nym[0].to_bytes(32, "big") if nymx is None else nymx
    y = nym[1].to_bytes(32, "big") if nymy is None else nymy
    inner = pb_field(1, 2, x) + pb_field(2, 2, y) + pb_field(3, 2, ou) + pb_field(4, 2, role) + pb_field(5, 2, proof)
    return pb_field(1, 2, mspid.encode()) + pb_field(2, 2, inner)


# ------------------------------------------------------------------ auditor: owner match
# crypto/audit/auditor.go:252-274 InspectTokenOwner -> des.GetOwnerMatcher(
# token.Owner.OwnerInfo) = idemix DeserializeAuditInfo (identity/msp/idemix/
# audit.go:32-46, Go encoding/json) -> AuditInfo.Match(RawOwner.Identity)
# (audit.go:51-83): the msp protos, then CSP.Verify(ipk, serialized.Proof, nil,
# EidNymAuditOpts{EidIndex 2, EnrollmentID string(Attributes[2]), RNymEid}).
# [EXT] IBM/idemix (not vendored), restated:
#   AuditNymEid: sig = proto Signature(serialized.Proof); EidNym must be present;
#   Nym_eid = HAttrs[2]^HashToZr(EnrollmentID) * HRand^RNymEid; match iff
#   Nym_eid == sig.EidNym.Nym (ECP from its X, Y bytes as NewECPbigs reads them).
#   Signature proto: 1 a_prime, 2 a_bar, 3 b_prime (ECP), 4..9 proof bytes,
#   10 repeated proof_s_attrs, 11 nonce, 12 nym (ECP), 13 proof_s_r_nym,
#   14 revocation_epoch_pk (ECP2), 15 revocation_pk_sig, 16 epoch (int64),
#   17 non_revocation_proof {1 revocation_alg, 2 non_revocation_proof},
#   18 eid_nym {1 nym (ECP), 2 proof_s_eid}.
#   AuditInfo JSON: {"RNymEid": Zr, "EID": Zr (embedded *NymEIDAuditData),
#   "Attributes": [][]byte}; mathlib Zr as {"curve": FP256BN_AMCL = 0,
#   "element": base64(>= 32 bytes)}, another curve id panics on use.
ERR_AUDIT = 12   # Match failed: the owner does not match the audit info
EID_INDEX = 2
NONREV_S = {1: "enum", 2: "bytes"}
EIDNYM_S = {1: ("msg", ECP_S), 2: "bytes"}
SIGNATURE_S = {1: ("msg", ECP_S), 2: ("msg", ECP_S), 3: ("msg", ECP_S), 4: "bytes", 5: "bytes", 6: "bytes",
               7: "bytes", 8: "bytes", 9: "bytes", 10: "*bytes", 11: "bytes", 12: ("msg", ECP_S), 13: "bytes",
               14: ("msg", ECP2_S), 15: "bytes", 16: "enum", 17: ("msg", NONREV_S), 18: ("msg", EIDNYM_S)}
FP256BN_CURVE_ID = 0


class Panic(Exception):
    pass


def _zr_json(v):
    """mathlib Zr UnmarshalJSON on the FP256BN curve: None for JSON null / absent,
    "panic" for another curve id or an element shorter than 32 bytes."""
    from . import gojson as J
    if v is None or v[0] == "null":
        return None
    curve, raw = J.dec_elem(v)
    if curve != FP256BN_CURVE_ID or raw is None or len(raw) < 32:
        return "panic"
    return int.from_bytes(raw[:32], "big")


def audit_info_decode(raw):
    """DeserializeAuditInfo: (rnym_eid, attributes); raises GoJSONError (any
    decoding error, first) or Panic (a Zr of another curve / too short)."""
    from . import gojson as J
    v = J.parse(raw)
    if v[0] == "null":
        return None, None
    if v[0] != "obj":
        raise J.GoJSONError("cannot unmarshal into AuditInfo")
    rnym = _zr_json(J.field(v, "RNymEid"))
    eid = _zr_json(J.field(v, "EID"))
    attrs = J.dec_list(J.field(v, "Attributes"), J.dec_bytes)
    if "panic" in (rnym, eid):
        raise Panic("mathlib Zr of another curve")
    return rnym, attrs


def audit_owner_match(ipk, owner, audit_info):
    """InspectTokenOwner for one token: (code, text).  owner = token.Owner
    (ASN.1 RawOwner), audit_info = the owner's OwnerInfo (AuditInfo JSON)."""
    from . import gojson as J
    if len(owner) == 0:
        return ERR_OWNER, "token is a redeem token, cannot inspect ownership"
    if len(audit_info) == 0:
        return ERR_OWNER, "failed to inspect owner: owner info is nil"
    try:
        typ, ident = raw_owner_decode(owner)
    except RQ.Asn1Error:
        return ERR_OWNER, "owner cannot be unwrapped"
    if typ != "si":
        return ERR_UNSUPPORTED, "script owner: inspected in Go"
    try:
        rnym, attrs = audit_info_decode(audit_info)
    except J.GoJSONError:
        return ERR_OWNER, "failed to get owner matcher"
    except Panic as e:
        return ERR_PANIC, "panic: %s" % e
    # Match (audit.go:51-83)
    try:
        si = pb_decode(ident, SERIALIZED_IDENTITY_S)
    except PbError:
        return ERR_AUDIT, "failed to unmarshal to msp.SerializedIdentity{}"
    try:
        ser = pb_decode(si.get(2, b""), SERIALIZED_IDEMIX_S)
    except PbError:
        return ERR_AUDIT, "could not deserialize a SerializedIdemixIdentity"
    if attrs is None or len(attrs) <= EID_INDEX:
        return ERR_PANIC, "panic: index out of range"
    eid = attrs[EID_INDEX] or b""
    try:
        sig = pb_decode(ser.get(5, b""), SIGNATURE_S)
    except PbError as e:
        return ERR_AUDIT, "error while verifying the nym eid: %s" % e
    en = sig.get(18)
    if en is None or en.get(1) is None:
        return ERR_AUDIT, "error while verifying the nym eid: no EidNym provided"
    if len(ipk.hattrs) <= EID_INDEX:
        return ERR_AUDIT, "error while verifying the nym eid: could not access H_a_eid in array"
    if rnym is None:
        return ERR_PANIC, "panic: nil RNymEid"
    try:
        nym_eid = ecp_from_bytes(en[1].get(1), en[1].get(2))
    except IndexError:
        return ERR_PANIC, "panic: index out of range"
    want = add(mul(ipk.hattrs[EID_INDEX], hash_to_zr(eid)), mul(ipk.hrand, rnym))
    if want != nym_eid:
        return ERR_AUDIT, "error while verifying the nym eid: eid nym does not match"
    return OK, ""


def audit_info_encode(rnym, eid_zr, attrs, curve=FP256BN_CURVE_ID):
    """json.Marshal(AuditInfo) for fixtures (Zr as 32-byte big-endian elements)."""
    from . import gojson as J
    z = (lambda x: "null" if x is None else J.enc_elem(x.to_bytes(32, "big"), curve))
    return J.enc_struct([("RNymEid", z(rnym)), ("EID", z(eid_zr)),
                         ("Attributes", J.enc_list(attrs, J.enc_bytes))]).encode()


def signature_with_eid_nym(nym_eid, extra=b""):
    """an idemix Signature proto carrying eid_nym (and `extra` encoded fields) for fixtures"""
    ecp = pb_field(1, 2, nym_eid[0].to_bytes(32, "big")) + pb_field(2, 2, nym_eid[1].to_bytes(32, "big"))
    return extra + pb_field(18, 2, pb_field(1, 2, ecp) + pb_field(2, 2, bytes(32)))


# ------------------------------------------------------------------ BN254 (gurvy translator)
# The curve the reference DEPLOYS for idemix: cmd/pp/dlog/gen.go:117
# (crypto.Setup(..., math3.BN254)), integration/nwo/token/platform.go:56,
# fabric/fabric.go:81, orion/orion.go:72, the wallet's identity/msp/idemix/
# lm.go:153; identity/msp/idemix/deserializer.go:40-51 picks the translator
# by curve (math.BN254 -> amcl.Gurvy{C: curve}).  [EXT] IBM/idemix and
# IBM/mathlib (go.mod:6-7; gnark-crypto v0.6.0 underneath, go.mod:53) are not
# vendored; restated:
#  * Gurvy.G1FromProto(ECP{X, Y}): len(X) and len(Y) must both be FieldBytes
#    (32) -- else "invalid marshalled length" --, then mathlib NewG1FromBytes
#    (X || Y) = gnark G1Affine.SetBytes behind a recover (bn254.g1_from_bytes:
#    flags, mod-p coordinates, on-curve, (0,0) = infinity, compressed forms);
#  * the nym import (NymPublicKeyImporter -> User.NewPublicNymFromBytes ->
#    Translator.G1FromRawBytes): raw = NymX || NymY split at len/2 and read by
#    G1FromProto, so only a 64-byte total decodes; a decoding error is an
#    import error (amcl read an off-curve nym as infinity, gnark rejects it);
#  * Zr from bytes: big.Int SetBytes over the WHOLE slice (any length, empty =
#    0), no reduction; Equals compares the integers; G1 Mul by any big.Int = (k
#    mod r) P (gnark GLV: the lattice rounding error does not grow with k);
#    Zr.Bytes = common.BigToBytes, 32 bytes, and a value >= 2^256 panics there
#    (make with a negative length), recovered into "failure [...]";
#  * G1 Bytes = gnark RawBytes, 64 bytes (infinity = 64 zero bytes), while
#    NymSignature still sizes proofData for 65-byte G1s:
#    4 + 2*(2*32+1) + 32 + len(msg) bytes, filled as "sign" | t (64) | Nym (64)
#    | ipk.Hash at 132 | msg at 164, the last 2 bytes left zero -- the same
#    sizing the reference-held BN254 IssuerPublicKey proof has (18*32+3 bytes,
#    576 used; issuer_key_check_bn254 accepts both tokengen keys with it);
#  * HashToZr = SHA-256 mod r (pinned by those keys).
BN254_CURVE_ID = 1


def _bn():
    from . import bn254 as C
    return C


class G1ProtoError(Exception):
    pass


def bn_g1_from_proto(x, y):
    """Gurvy.G1FromProto(&ECP{X: x, Y: y}): the point (None = infinity) or G1ProtoError"""
    C = _bn()
    if x is None or y is None or len(x) != 32 or len(y) != 32:
        raise G1ProtoError("invalid marshalled length")
    try:
        return C.g1_from_bytes(bytes(x) + bytes(y))
    except C.DecodeError as e:
        raise G1ProtoError("failure [set bytes failed [%s]]" % e)


class IssuerPKBn254:
    """an IssuerPublicKey proto read with the Gurvy translator; bad HSk / HRand /
    HAttrs are None (the Go importer, IssuerPublicKey.Check, would refuse the key)"""

    def __init__(self, raw):
        m = pb_decode(raw, IPK_S)
        self.raw = raw
        self.fields = m

        def pt(e):
            try:
                return ("ok", bn_g1_from_proto((e or {}).get(1), (e or {}).get(2)))
            except G1ProtoError:
                return ("bad", None)
        self.hsk_s, self.hsk = pt(m.get(2))
        self.hrand_s, self.hrand = pt(m.get(3))
        self.hattrs_s = [pt(e) for e in m.get(4, [])]
        self.hattrs = [p for _, p in self.hattrs_s]
        self.hash = m.get(10, b"")


def bn_zr(b):
    """mathlib gurvy NewZrFromBytes: the whole slice big-endian, unreduced"""
    return int.from_bytes(b or b"", "big")


def bn_proof_data(t, nym, ipk_hash, msg):
    C = _bn()
    d = bytearray(len(SIGN_LABEL) + 2 * (2 * FIELD_BYTES + 1) + FIELD_BYTES + len(msg))
    d[0:4] = SIGN_LABEL
    d[4:68] = C.g1_bytes(t)
    d[68:132] = C.g1_bytes(nym)
    h = ipk_hash[:len(d) - 132]
    d[132:132 + len(h)] = h  # copy(proofData[index:], ipk.Hash)
    d[164:164 + len(msg)] = msg  # copy(proofData[index:], msg): 2 zero bytes stay at the end
    return bytes(d)


def bn_make_nym(ipk, sk, r_nym):
    C = _bn()
    return C.g1_add(C.g1_mul(ipk.hsk, sk), C.g1_mul(ipk.hrand, r_nym))


def bn_nym_sign(ipk, sk, r_nym, nym, msg, r_sk, r_rnym, nonce):
    """NewNymSignature on BN254 with injected randomness: the NymSignature proto"""
    C = _bn()
    t = C.g1_add(C.g1_mul(ipk.hsk, r_sk), C.g1_mul(ipk.hrand, r_rnym))
    c = C.hash_to_zr(bn_proof_data(t, nym, ipk.hash, msg))
    proof_c = C.hash_to_zr(c.to_bytes(32, "big") + nonce.to_bytes(32, "big"))
    s_sk = (r_sk + proof_c * sk) % C.R
    s_rnym = (r_rnym + proof_c * r_nym) % C.R
    return b"".join(pb_field(k + 1, 2, v.to_bytes(32, "big")) for k, v in enumerate((proof_c, s_sk, s_rnym, nonce)))


def bn_nym_verify(ipk, nym, sig, msg):
    """NymSignature.Ver on BN254 behind the bridge's recover: (code, text)"""
    C = _bn()
    if len(sig) == 0:
        return ERR_SIGNATURE, "invalid signature, it must not be empty"
    try:
        m = pb_decode(sig, NYMSIG_S)
    except PbError as e:
        return ERR_SIGNATURE, "error unmarshalling signature: %s" % e
    proof_c, s_sk, s_rnym, nonce = (bn_zr(m.get(k)) for k in (1, 2, 3, 4))
    t = C.g1_add(C.g1_add(C.g1_mul(ipk.hsk, s_sk), C.g1_mul(ipk.hrand, s_rnym)), C.g1_neg(C.g1_mul(nym, proof_c)))
    c = C.hash_to_zr(bn_proof_data(t, nym, ipk.hash, msg))
    if nonce >= 1 << 256:
        return ERR_SIGNATURE, "failure [runtime error: makeslice: len out of range]"
    if proof_c != C.hash_to_zr(c.to_bytes(32, "big") + nonce.to_bytes(32, "big")):
        return ERR_SIGNATURE, "pseudonym signature invalid: zero-knowledge proof is invalid"
    return OK, ""


def bn_deserialize_idemix_identity(raw):
    """common.go:40-117 Deserialize(raw, false) with the Gurvy translator"""
    try:
        si = pb_decode(raw, SERIALIZED_IDENTITY_S)
    except PbError:
        return None, (ERR_OWNER, "failed to unmarshal to msp.SerializedIdentity{}")
    try:
        ser = pb_decode(si.get(2, b""), SERIALIZED_IDEMIX_S)
    except PbError:
        return None, (ERR_OWNER, "could not deserialize a SerializedIdemixIdentity")
    if not ser.get(1) or not ser.get(2):
        return None, (ERR_OWNER, "unable to deserialize idemix identity: pseudonym is invalid")
    raw_nym = ser[1] + ser[2]
    half = len(raw_nym) // 2
    try:
        nym = bn_g1_from_proto(raw_nym[:half], raw_nym[half:])
    except G1ProtoError:
        return None, (ERR_OWNER, "failed to import nym public key")
    try:
        pb_decode(ser.get(3, b""), OU_S)
    except PbError:
        return None, (ERR_OWNER, "cannot deserialize the OU of the identity")
    try:
        pb_decode(ser.get(4, b""), ROLE_S)
    except PbError:
        return None, (ERR_OWNER, "cannot deserialize the role of the identity")
    return nym, None


def bn_owner_verify(ipk, owner, msg, sig):
    """one input of TransferSignatureValidate on a BN254 idemix deployment: (code, text)"""
    try:
        typ, ident = raw_owner_decode(owner)
    except RQ.Asn1Error:
        return ERR_OWNER, "failed to unmarshal RawOwner"
    if typ == "htlc":
        return ERR_UNSUPPORTED, "htlc script owner: verified in Go"
    if typ != "si":
        return ERR_OWNER, "failed to deserialize RawOwner: Unknown owner type %s" % typ
    nym, err = bn_deserialize_idemix_identity(ident)
    if err:
        return err
    return bn_nym_verify(ipk, nym, sig, msg)


def bn_serialize_idemix_identity(nym, **kw):
    """as serialize_idemix_identity, with the nym's gnark coordinates (infinity = zeros)"""
    C = _bn()
    raw = C.g1_bytes(nym)
    kw.setdefault("nymx", raw[:32])
    kw.setdefault("nymy", raw[32:])
    return serialize_idemix_identity((0, 0), **kw)


def _bn_zr_json(v):
    """mathlib Zr UnmarshalJSON on BN254: None for null / absent, "panic" for a
    Zr of another curve id (the gurvy driver's type assertion on use), else the
    raw integer of the element (any length)"""
    from . import gojson as J
    if v is None or v[0] == "null":
        return None
    curve, raw = J.dec_elem(v)
    if curve != BN254_CURVE_ID:
        return "panic"
    return bn_zr(raw)


def bn_audit_owner_match(ipk, owner, audit_info):
    """InspectTokenOwner for one token on a BN254 idemix deployment: (code, text).
    AuditNymEid order [EXT]: EidNym present, len(HAttrs) > 2, H_a_eid / HRand /
    EidNym through G1FromProto (an error is a Match error), then
    H_a_eid^HashToZr(eid) * HRand^RNymEid (a nil RNymEid panics here) == EidNym."""
    from . import gojson as J
    C = _bn()
    if len(owner) == 0:
        return ERR_OWNER, "token is a redeem token, cannot inspect ownership"
    if len(audit_info) == 0:
        return ERR_OWNER, "failed to inspect owner: owner info is nil"
    try:
        typ, ident = raw_owner_decode(owner)
    except RQ.Asn1Error:
        return ERR_OWNER, "owner cannot be unwrapped"
    if typ != "si":
        return ERR_UNSUPPORTED, "script owner: inspected in Go"
    try:
        v = J.parse(audit_info)
        if v[0] == "null":
            rnym, attrs = None, None
        elif v[0] != "obj":
            raise J.GoJSONError("cannot unmarshal into AuditInfo")
        else:
            rnym = _bn_zr_json(J.field(v, "RNymEid"))
            eid_zr = _bn_zr_json(J.field(v, "EID"))
            attrs = J.dec_list(J.field(v, "Attributes"), J.dec_bytes)
            if "panic" in (rnym, eid_zr):
                return ERR_PANIC, "panic: mathlib Zr of another curve"
    except J.GoJSONError:
        return ERR_OWNER, "failed to get owner matcher"
    try:
        si = pb_decode(ident, SERIALIZED_IDENTITY_S)
    except PbError:
        return ERR_AUDIT, "failed to unmarshal to msp.SerializedIdentity{}"
    try:
        ser = pb_decode(si.get(2, b""), SERIALIZED_IDEMIX_S)
    except PbError:
        return ERR_AUDIT, "could not deserialize a SerializedIdemixIdentity"
    if attrs is None or len(attrs) <= EID_INDEX:
        return ERR_PANIC, "panic: index out of range"
    eid = attrs[EID_INDEX] or b""
    try:
        sig = pb_decode(ser.get(5, b""), SIGNATURE_S)
    except PbError as e:
        return ERR_AUDIT, "error while verifying the nym eid: %s" % e
    en = sig.get(18)
    if en is None or en.get(1) is None:
        return ERR_AUDIT, "error while verifying the nym eid: no EidNym provided"
    if len(ipk.hattrs) <= EID_INDEX:
        return ERR_AUDIT, "error while verifying the nym eid: could not access H_a_eid in array"
    if ipk.hattrs_s[EID_INDEX][0] != "ok" or ipk.hrand_s != "ok":
        return ERR_AUDIT, "error while verifying the nym eid: could not deserialize H_a_eid / HRand"
    try:
        nym_eid = bn_g1_from_proto(en[1].get(1), en[1].get(2))
    except G1ProtoError:
        return ERR_AUDIT, "error while verifying the nym eid: could not deserialize EidNym"
    if rnym is None:
        return ERR_PANIC, "panic: nil RNymEid"
    want = C.g1_add(C.g1_mul(ipk.hattrs[EID_INDEX], C.hash_to_zr(eid)), C.g1_mul(ipk.hrand, rnym))
    if want != nym_eid:
        return ERR_AUDIT, "error while verifying the nym eid: eid nym does not match"
    return OK, ""


def bn_signature_with_eid_nym(nym_eid, extra=b""):
    """an idemix Signature proto carrying eid_nym (gnark coordinates) for fixtures"""
    C = _bn()
    raw = C.g1_bytes(nym_eid)
    ecp = pb_field(1, 2, raw[:32]) + pb_field(2, 2, raw[32:])
    return extra + pb_field(18, 2, pb_field(1, 2, ecp) + pb_field(2, 2, bytes(32)))

"""zkatdlog (nogh) proofs restated in Python (TEST INFRASTRUCTURE ONLY).

Function-by-function restatement of ``token/core/zkatdlog/crypto`` in the
reference (paths relative to /root/reference/token/core/zkatdlog/crypto):

    setup            setup.go:214-236, 168-184, 153-166; pssign/sign.go:43-119
    token commitment token/token.go:64-98
    Schnorr          common/schnorr.go:36-118
    transfer WF      transfer/wellformedness.go:131-240, 243-378
    range proof      range/proof.go:141-444
    membership/POK   sigproof/membership.go:112-305; sigproof/pok.go:160-204
    transfer         transfer/transfer.go:66-154
    issue            issue/issue.go:151-223; issue/wellformedness.go:74-265

The verifier reproduces the reference's accept/reject decision, including the
reject classes the reference's tests pin and the
panic paths (reported as ``ERR_PANIC``: the reference process would crash, the
batch verifier reports reject).

Randomness: the reference draws from crypto/rand; here every random scalar is
derived from (seed, tag) with SHA-256 so that a prover on any device can
reproduce the same proof bytes (see ``Rand``).
"""
import hashlib

from . import bn254 as C
from . import gojson as J

R = C.R

# verdict / error classes (mirrors include/ftsamd.h)
OK = 0
ERR_PARSE = 1         # json / base64 / element decoding failed
ERR_MALFORMED = 2     # structural check failed ("not well formed", nil fields)
ERR_WF = 3            # "invalid zero-knowledge transfer" / issue WF challenge mismatch
ERR_RANGE = 4         # "invalid range proof"
ERR_MEMBERSHIP = 5    # "invalid membership proof"
ERR_PANIC = 6         # the reference would panic (nil dereference, foreign curve)


# Parity tests only: a list here collects every challenge a verifier
# recomputes, as (class, HashToZr) in the order the checks run (see
# include/ftsamd.h ftz_batch_challenges for the device's side).
CHALLENGE_TRACE = None


def _traced(kind, h):
    if CHALLENGE_TRACE is not None:
        CHALLENGE_TRACE.append((kind, h))
    return h


class VerifyError(Exception):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


class Panic(VerifyError):
    def __init__(self, msg):
        super().__init__(ERR_PANIC, msg)


# ------------------------------------------------------------------ randomness
class Rand:
    """Deterministic scalar source: rand(tag) = SHA-256(seed||tag||0) ||
    SHA-256(seed||tag||1) read big-endian, mod r (512 bits -> negligible bias)."""

    def __init__(self, seed):
        self.seed = bytes(seed)

    def zr(self, tag):
        t = tag.encode() if isinstance(tag, str) else bytes(tag)
        h0 = hashlib.sha256(self.seed + t + b"\x00").digest()
        h1 = hashlib.sha256(self.seed + t + b"\x01").digest()
        return int.from_bytes(h0 + h1, "big") % R


# ------------------------------------------------------------------ elements
def enc_zr(z):
    return J.enc_elem(C.zr_bytes(z % R) if 0 <= z < (1 << 256) else None)


def enc_g1(p):
    return J.enc_elem(C.g1_bytes(p))


def enc_g2(p):
    return J.enc_elem(C.g2_bytes(p))


def dec_zr(v):
    """mathlib Zr.UnmarshalJSON: big.Int SetBytes, *no* reduction (Zr.Equals
    compares raw integers).  Foreign curve -> the reference panics on first
    use (driver type assertion), reported here as a panic at decode."""
    e = J.dec_elem(v)
    if e is None:
        return None
    curve, raw = e
    if curve != J.BN254:
        raise Panic("foreign curve id %d" % curve)
    return int.from_bytes(raw or b"", "big")


def dec_g1(v):
    e = J.dec_elem(v)
    if e is None:
        return None
    curve, raw = e
    if curve != J.BN254:
        raise Panic("foreign curve id %d" % curve)
    try:
        return ("pt", C.g1_from_bytes(raw))
    except C.DecodeError as ex:
        raise VerifyError(ERR_PARSE, "failure [%s]" % ex)


def dec_g2(v):
    e = J.dec_elem(v)
    if e is None:
        return None
    curve, raw = e
    if curve != J.BN254:
        raise Panic("foreign curve id %d" % curve)
    try:
        return ("pt", C.g2_from_bytes(raw))
    except C.DecodeError as ex:
        raise VerifyError(ERR_PARSE, "failure [%s]" % ex)


def pt(x):
    """Unwrap a decoded (non-nil) point."""
    return x[1]


# ------------------------------------------------------------------ public params
class PublicParams:
    """setup.go:25-54 PublicParams / RangeProofParams."""

    def __init__(self):
        self.label = "zkatdlog"
        self.curve = J.BN254
        self.ped_gen = None
        self.ped = []
        self.sign_pk = []
        self.signed_values = []      # list of (R, S)
        self.q = None
        self.exponent = 0
        self.idemix_curve = 0
        self.idemix_pk = None
        self.auditor = None
        self.issuers = None
        self.precision = 64

    @property
    def base(self):
        return len(self.signed_values)

    def to_json(self):
        """setup.go:119-128 Serialize: json.Marshal(pp) wrapped in
        driver.SerializedPublicParameters{Identifier, Raw}."""
        sig = lambda s: J.enc_struct([("R", enc_g1(s[0])), ("S", enc_g1(s[1]))])
        rpp = J.enc_struct([
            ("SignPK", J.enc_list(self.sign_pk, enc_g2)),
            ("SignedValues", J.enc_list(self.signed_values, sig)),
            ("Q", enc_g2(self.q)),
            ("Exponent", str(self.exponent)),
        ])
        raw = J.enc_struct([
            ("Label", J.enc_str(self.label)),
            ("Curve", str(self.curve)),
            ("PedGen", enc_g1(self.ped_gen)),
            ("PedParams", J.enc_list(self.ped, enc_g1)),
            ("RangeProofParams", rpp),
            ("IdemixCurveID", str(self.idemix_curve)),
            ("IdemixIssuerPK", J.enc_bytes(self.idemix_pk)),
            ("Auditor", J.enc_bytes(self.auditor)),
            ("Issuers", J.enc_list(self.issuers, J.enc_bytes)),
            ("QuantityPrecision", str(self.precision)),
        ])
        return J.enc_struct([("Identifier", J.enc_str(self.label)),
                             ("Raw", J.enc_bytes(raw.encode()))]).encode()

    @staticmethod
    def from_json(data, label="zkatdlog"):
        """setup.go:134-151 Deserialize."""
        outer = J.parse(data)
        ident = J.dec_string(J.field(outer, "Identifier"))
        if ident != label:
            raise ValueError("invalid identifier, expecting [%s], got [%s]" % (label, ident))
        raw = J.dec_bytes(J.field(outer, "Raw"))
        v = J.resolve(J.parse(raw), PP_SCHEMA)
        pp = PublicParams()
        pp.label = label
        pp.curve = J.dec_int(J.field(v, "Curve"))
        g = J.field(v, "PedGen")
        pp.ped_gen = pt(dec_g1(g)) if g is not None and g[0] != "null" else None
        pp.ped = [pt(dec_g1(x)) for x in J.field(v, "PedParams")[1]]
        rpp = J.field(v, "RangeProofParams")
        pp.sign_pk = [pt(dec_g2(x)) for x in J.field(rpp, "SignPK")[1]]
        pp.signed_values = [(pt(dec_g1(J.field(s, "R"))), pt(dec_g1(J.field(s, "S"))))
                            for s in J.field(rpp, "SignedValues")[1]]
        pp.q = pt(dec_g2(J.field(rpp, "Q")))
        pp.exponent = J.dec_int(J.field(rpp, "Exponent"))
        pp.idemix_curve = J.dec_int(J.field(v, "IdemixCurveID"))
        pp.idemix_pk = J.dec_bytes(J.field(v, "IdemixIssuerPK"))
        pp.precision = J.dec_int(J.field(v, "QuantityPrecision"))
        return pp


# struct-pointer / slice-of-struct-pointer fields, whose duplicate keys merge
# (gojson.resolve): setup.go:25-54 PublicParams / RangeProofParams /
# pssign.Signature; range/proof.go:25-57 RangeProof / EqualityProofs /
# MembershipProof -> sigproof/membership.go:19-33 MembershipProof -> Signature
PP_SCHEMA = {"RangeProofParams": (J.STRUCT, {"SignedValues": (J.SLICE, {})})}
RANGE_SCHEMA = {"EqualityProofs": (J.STRUCT, {}),
                "MembershipProofs": (J.SLICE, {"SignatureProofs": (J.SLICE, {"Signature": (J.STRUCT, {})})})}

MATHLIB_CURVES = 3  # [EXT] len(math.Curves) at IBM/mathlib 0a7378db6912: FP256BN_AMCL, BN254, FP256BN_AMCL_MIRACL


def validate_json(data, label="zkatdlog"):
    """setup.go:238-273 PublicParams.Validate (with RangeProofParams.Validate
    :56-80) after Deserialize (:134-151), on the serialized bytes.  Returns ""
    or the reference's error text.  Point encodings are not checked here (the
    device decoder checks them when a context is created)."""
    try:
        outer = J.parse(data)
        ident = J.dec_string(J.field(outer, "Identifier"))
        if ident != label:
            return "invalid identifier, expecting [%s], got [%s]" % (label, ident)
        raw = J.dec_bytes(J.field(outer, "Raw"))
        v = J.resolve(J.parse(raw if raw is not None else b""), PP_SCHEMA)
        curve = J.dec_int(J.field(v, "Curve"))
        idemix_curve = J.dec_int(J.field(v, "IdemixCurveID"))
        prec = J.dec_int(J.field(v, "QuantityPrecision"))
        if prec < 0:
            raise J.GoJSONError("cannot unmarshal number into uint64")
        ipk = J.dec_bytes(J.field(v, "IdemixIssuerPK"))
    except J.GoJSONError as e:
        return "failed unmarshalling public parameters: %s" % e

    def isnull(x):
        return x is None or x[0] == "null"

    def arr(x):
        return [] if isnull(x) else x[1]
    if curve > MATHLIB_CURVES - 1:
        return "invalid public parameters: invalid curveID [%d > %d]" % (curve, MATHLIB_CURVES - 1)
    if idemix_curve > MATHLIB_CURVES - 1:  # the reference prints pp.Curve here
        return "invalid public parameters: invalid idemix curveID [%d > %d]" % (curve, MATHLIB_CURVES - 1)
    if isnull(J.field(v, "PedGen")):
        return "invalid public parameters: nil Pedersen generator"
    ped = arr(J.field(v, "PedParams"))
    if len(ped) != 3:
        return "invalid public parameters: length mismatch in Pedersen parameters [%d vs. 3]" % len(ped)
    for i, x in enumerate(ped):
        if isnull(x):
            return "invalid public parameters: nil Pedersen parameter at index %d" % i
    rpp = J.field(v, "RangeProofParams")
    if isnull(rpp):
        return "invalid public parameters: nil range proof parameters"
    spk, sv = arr(J.field(rpp, "SignPK")), arr(J.field(rpp, "SignedValues"))
    w = "invalid public parameters: invalid range proof parameters: "
    if len(spk) != 3:
        return w + "signature public key should be 3, instead it is %d" % len(spk)
    if len(sv) < 2:
        return w + "signed values should be > 2"
    if isnull(J.field(rpp, "Q")):
        return w + "generator Q is nil"
    if J.dec_int(J.field(rpp, "Exponent")) == 0:
        return w + "exponent is 0"
    for i, x in enumerate(sv):
        if isnull(x):
            return w + "signed value at index %d is nil" % i
    for i, x in enumerate(spk):
        if isnull(x):
            return w + "public key at index %d is nil" % i
    if prec != 64:
        return "invalid public parameters: quantity precision should be 64 instead it is %d" % prec
    if not ipk:
        return "invalid public parameters: empty idemix issuer"
    return ""


def ps_hash(m):
    """pssign/sign.go:198-206 hashMessages for a single message."""
    return C.hash_to_zr(C.zr_bytes(m))


def setup(base, exponent, rnd, idemix_pk=b"idemix-issuer-pk", idemix_curve=0):
    """setup.go:214-236 SetupWithCustomLabel with pssign KeyGen(1)
    (pssign/sign.go:43-67) and GenerateRangeProofParameters (setup.go:168-184).
    Reproduces the Sign quirk of pssign/sign.go:97-98: R stays the G1 generator
    (``Mul`` returns a new point that is discarded)."""
    pp = PublicParams()
    pp.q = C.g2_mul(C.G2_GEN, rnd.zr("setup/Q"))
    sk = [rnd.zr("setup/sk/%d" % i) for i in range(3)]
    pp.sign_pk = [C.g2_mul(pp.q, s) for s in sk]
    pp.ped_gen = C.g1_mul(C.G1_GEN, rnd.zr("setup/pedgen"))
    pp.ped = [C.g1_mul(C.G1_GEN, rnd.zr("setup/ped/%d" % i)) for i in range(3)]
    for m in range(base):
        Rpt = C.G1_GEN
        e = (sk[0] + sk[1] * m + sk[2] * ps_hash(m)) % R
        pp.signed_values.append((Rpt, C.g1_mul(Rpt, e)))
    pp.exponent = exponent
    pp.idemix_pk = idemix_pk
    pp.idemix_curve = idemix_curve
    pp._sk = sk
    return pp


def type_hash(ttype):
    return C.hash_to_zr(ttype.encode())


def token_commitment(pp, ttype, value, bf):
    """token/token.go:64-76 computeTokens: H(type)*Ped0 + value*Ped1 + bf*Ped2."""
    return C.g1_sum([C.g1_mul(pp.ped[0], type_hash(ttype)),
                     C.g1_mul(pp.ped[1], value), C.g1_mul(pp.ped[2], bf)])


# ------------------------------------------------------------------ Schnorr helpers
def schnorr_recompute(bases, proof, statement, chal):
    """common/schnorr.go:78-104 RecomputeCommitment: sum_i bases[i]*proof[i] - chal*statement."""
    if chal is None:
        raise VerifyError(ERR_MALFORMED, "invalid zero-knowledge proof: nil challenge or statement")
    if len(proof) > len(bases):
        raise VerifyError(ERR_MALFORMED, "please initialize Pedersen parameters correctly")
    acc = None
    for b, s in zip(bases, proof):
        if s is None:
            raise VerifyError(ERR_MALFORMED, "invalid zero-knowledge proof: nil proof")
        acc = C.g1_add(acc, C.g1_mul(b, s))
    return C.g1_add(acc, C.g1_neg(C.g1_mul(statement, chal)))


def g1_array_bytes(points):
    """common/array.go:29-40 G1Array.Bytes."""
    return b"".join(C.g1_bytes(p) for p in points)


def g2_array_bytes(points):
    return b"".join(C.g2_bytes(p) for p in points)


# ------------------------------------------------------------------ membership
def sig_json(R_, S_):
    """json.Marshal(pssign.Signature{R,S}) -- hashed into the membership
    transcript (sigproof/membership.go:270)."""
    return J.enc_struct([("R", enc_g1(R_)), ("S", enc_g1(S_))]).encode()


def membership_transcript(pp, com_to_value, g1_com, gt_com, sig_R, sig_S):
    """sigproof/membership.go:260-277 computeChallenge input bytes."""
    return (g1_array_bytes([pp.ped[0], pp.ped[1], com_to_value, g1_com, pp.ped_gen])
            + g2_array_bytes(pp.sign_pk + [pp.q]) + C.gt_bytes(gt_com) + sig_json(sig_R, sig_S))


def membership_prove(pp, rnd, tag, sig, value, com_bf, commitment):
    """sigproof/membership.go:112-158 Prove (+ obfuscateSignature :196-222,
    computeCommitment :225-257)."""
    P_, Q_ = pp.ped_gen, pp.q
    blinding = rnd.zr(tag + "/sigbf")
    rr = rnd.zr(tag + "/randomize")
    Rp = C.g1_mul(sig[0], rr)
    Sp = C.g1_mul(sig[1], rr)
    obf_S = C.g1_add(Sp, C.g1_mul(P_, blinding))
    h = C.hash_to_zr(C.zr_bytes(value))
    rv = rnd.zr(tag + "/r_value")
    rh = rnd.zr(tag + "/r_hash")
    rsbf = rnd.zr(tag + "/r_sigbf")
    t = C.g2_add(C.g2_mul(pp.sign_pk[1], rv), C.g2_mul(pp.sign_pk[2], rh))
    gt = C.final_exp(C.miller_loop([(Rp, t), (C.g1_mul(P_, rsbf), Q_)]))
    rcb = rnd.zr(tag + "/r_combf")
    g1c = C.g1_add(C.g1_mul(pp.ped[0], rv), C.g1_mul(pp.ped[1], rcb))
    chal = C.hash_to_zr(membership_transcript(pp, commitment, g1c, gt, Rp, obf_S))
    return {
        "Challenge": chal,
        "Signature": (Rp, obf_S),
        "Value": (rv + chal * value) % R,
        "ComBlindingFactor": (rcb + chal * com_bf) % R,
        "SigBlindingFactor": (rsbf + chal * blinding) % R,
        "Hash": (rh + chal * h) % R,
        "Commitment": commitment,
    }


def enc_membership(mp):
    return J.enc_struct([
        ("Challenge", enc_zr(mp["Challenge"])),
        ("Signature", J.enc_struct([("R", enc_g1(mp["Signature"][0])), ("S", enc_g1(mp["Signature"][1]))])),
        ("Value", enc_zr(mp["Value"])),
        ("ComBlindingFactor", enc_zr(mp["ComBlindingFactor"])),
        ("SigBlindingFactor", enc_zr(mp["SigBlindingFactor"])),
        ("Hash", enc_zr(mp["Hash"])),
        ("Commitment", enc_g1(mp["Commitment"])),
    ])


def membership_verify(pp, com_to_value, proof):
    """sigproof/membership.go:162-180 Verify with recomputeCommitments
    (:281-305) and POKVerifier.recomputeCommitment (pok.go:160-204).
    ``com_to_value`` is MembershipProofs[k].Commitments[i] (Schnorr statement);
    the transcript uses the proof's own Commitment field (membership.go:170)."""
    if proof is None:
        raise Panic("nil membership proof")           # membership.go:285 p.Challenge on nil
    # pok.go:160-204
    if proof["Value"] is None:
        raise VerifyError(ERR_MALFORMED, "nil elements")
    if proof["Hash"] is None:
        raise VerifyError(ERR_MALFORMED, "nil hash")
    sig = proof["Signature"]
    if sig is None or sig[0] is None or sig[1] is None:
        raise VerifyError(ERR_MALFORMED, "nil elements")
    c = proof["Challenge"]
    if c is None or proof["SigBlindingFactor"] is None:
        raise VerifyError(ERR_MALFORMED, "nil elements")
    Rw, Sw = pt(sig[0]), pt(sig[1])
    t = C.g2_add(C.g2_mul(pp.sign_pk[1], proof["Value"]), C.g2_mul(pp.sign_pk[2], proof["Hash"]))
    neg_pk0 = C.g2_neg(pp.sign_pk[0])
    m1 = C.miller_loop([(C.g1_mul(Sw, c), pp.q), (C.g1_mul(Rw, c), neg_pk0)])
    m2 = C.miller_loop([(Rw, t), (C.g1_mul(pp.ped_gen, proof["SigBlindingFactor"]), pp.q)])
    gt = C.final_exp(C.f12_mul(C.f12_inv(m1), m2))
    # Schnorr on Commitments[k][i] (membership.go:297-299)
    if com_to_value is None:
        raise VerifyError(ERR_MALFORMED, "invalid zero-knowledge proof: nil challenge or statement")
    g1c = schnorr_recompute(pp.ped[:2], [proof["Value"], proof["ComBlindingFactor"]], pt(com_to_value), c)
    if proof["Commitment"] is None:
        raise VerifyError(ERR_MALFORMED, "failed to marshal array of G1")
    data = membership_transcript(pp, pt(proof["Commitment"]), g1c, gt, Rw, Sw)
    if _traced(ERR_MEMBERSHIP, C.hash_to_zr(data)) != c:
        raise VerifyError(ERR_MEMBERSHIP, "invalid membership proof")


def dec_membership(v):
    if v is None or v[0] == "null":
        return None
    sigv = J.field(v, "Signature")
    sig = None
    if sigv is not None and sigv[0] != "null":
        sig = (dec_g1(J.field(sigv, "R")), dec_g1(J.field(sigv, "S")))
    return {
        "Challenge": dec_zr(J.field(v, "Challenge")),
        "Signature": sig,
        "Value": dec_zr(J.field(v, "Value")),
        "ComBlindingFactor": dec_zr(J.field(v, "ComBlindingFactor")),
        "SigBlindingFactor": dec_zr(J.field(v, "SigBlindingFactor")),
        "Hash": dec_zr(J.field(v, "Hash")),
        "Commitment": dec_g1(J.field(v, "Commitment")),
    }


# ------------------------------------------------------------------ range proof
INT64_MIN = -(1 << 63)

# Counterfactual switch for the parity tests only: True weighs digit i by the
# exact integer base**i instead of the reference's int64(math.Pow(...)).
EXACT_WEIGHTS = False


def go_pow(x, n):
    """Go math.Pow(x, float64(n)) for an integer n >= 0 and a finite x >= 2
    (Go standard library src/math/pow.go, go1.18 per the reference's go.mod:3;
    amd64 has no assembly Pow, so this pure-Go path is what runs).  Special
    cases y == 0 / x == 1 -> 1 and y == 1 -> x, then yi = n, yf = 0:
    Frexp(x) = x1 * 2^xe, repeated squaring of the mantissa x1 (renormalised
    back to [0.5, 1) after each square), the set bits of n multiplied into a1
    with their exponents summed into ae, and Ldexp(a1, ae).  Every float64
    operation here is a single IEEE-754 round-to-nearest multiply or add (Go
    does not fuse them on amd64), which Python floats reproduce exactly."""
    import math
    x = float(x)
    if n == 0 or x == 1.0:
        return 1.0
    if n == 1:
        return x
    a1, ae = 1.0, 0
    x1, xe = math.frexp(x)
    i = n
    while i != 0:
        if xe < -(1 << 12) or (1 << 12) < xe:
            # catastrophic overflow: Ldexp handles it below
            ae += xe
            break
        if i & 1:
            a1 *= x1
            ae += xe
        x1 *= x1
        xe <<= 1
        if x1 < 0.5:
            x1 += x1
            xe -= 1
        i >>= 1
    try:
        return math.ldexp(a1, ae)
    except OverflowError:  # Go's Ldexp returns +Inf
        return float("inf")


def go_int64(f):
    """int64(f) for a float64 f as Go compiles it on amd64 (CVTTSD2SQ): the
    truncated value when it fits, else the "integer indefinite" 0x8000000000000000
    (= -2^63) for NaN, +-Inf and every out-of-range value.  [EXT] the Go spec
    leaves the out-of-range result implementation-defined; amd64 is the
    platform the reference's peers run on."""
    if f != f or not (-9223372036854775808.0 <= f < 9223372036854775808.0):
        return INT64_MIN
    return int(f)


def digit_weight(base, i):
    """The weight of digit i in the range proof: int64(math.Pow(float64(Base),
    float64(i))) (range/proof.go:428 verifier, :327 prover).  Equal to base**i
    only while base**i is a float64; e.g. 7^21 comes out as 7^21 + 25 and
    base^i >= 2^63 as -2^63.  As a Zr it is taken mod r (NewZrFromInt keeps the
    big.Int; scalar multiplication and ModMul/ModAdd reduce it mod r)."""
    if EXACT_WEIGHTS:
        return base ** i
    return go_int64(go_pow(base, i))


def _go_quo(a, b):
    """Go int64 a / b (truncated toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def _go_rem(a, b):
    """Go int64 a % b (sign of the dividend)."""
    return a - _go_quo(a, b) * b


def range_weights_exact(base, exponent):
    """True when every verifier weight int64(math.Pow(base, i)), i < exponent, is base**i."""
    return all(go_int64(go_pow(base, i)) == base ** i for i in range(max(exponent, 0)))


def digits(v, base, exponent):
    """range/proof.go:297-311 preProcess: the digits the reference's prover
    commits to.  v must be an int64 (Value.Int(), :299); v >= int64(math.Pow(
    Base, Exponent)) is refused (:303-305); values[0] = v % Base on the
    original v (:307), then for i = Exponent-1 .. 1 values[i] = v / w_i and
    v = v % w_i with w_i = int64(math.Pow(Base, i)) (:308-311).  With inexact
    weights the digits need not sum back to v (the reference's verifier then
    rejects its own prover's proof), and a digit >= Base indexes past
    Signatures (:326) -- a Go panic, raised here as ``Panic``.

    [EXT] extension: where int64(math.Pow(Base, Exponent)) overflows (e.g.
    PP-B, b = 16, e = 16: 2^64 -> -2^63) the reference refuses every value;
    this build then proves v < Base^Exponent (up to 2^64 - 1) with the exact
    base-Base digits, which the reference's verifier accepts whenever every
    weight below Exponent is exact (else refused here)."""
    if v < 0:
        raise ValueError("can't compute range proof: value of token outside authorized range")
    top = digit_weight(base, exponent)
    if top == INT64_MIN and not EXACT_WEIGHTS:
        if v >= base ** exponent or not range_weights_exact(base, exponent):
            raise ValueError("can't compute range proof: value of token outside authorized range")
        out = []
        for _ in range(exponent):
            out.append(v % base)
            v //= base
        return out
    if v >= (1 << 63) or v >= top:
        raise ValueError("can't compute range proof: value of token outside authorized range")
    out = [0] * exponent
    out[0] = _go_rem(v, base)
    for i in range(exponent - 1):
        w = digit_weight(base, exponent - 1 - i)
        out[exponent - 1 - i] = _go_quo(v, w)
        v = _go_rem(v, w)
    for d in out:
        if d >= base or d < 0:
            raise Panic("index out of range [%d] with length %d" % (d, base))
    return out


def range_transcript(pp, tokens, com_tokens, com_values, coms):
    """range/proof.go:371-389 computeChallenge input bytes."""
    data = g1_array_bytes([pp.ped_gen] + tokens + com_tokens + com_values + pp.ped)
    data += g2_array_bytes([pp.q] + pp.sign_pk)
    for row in coms:
        data += g1_array_bytes(row)
    return data


def range_prove(pp, rnd, tag, tokens, witnesses, ttype, digit_rows=None):
    """range/proof.go:141-209 Prove.  witnesses: list of (value, bf).
    digit_rows (test fixtures only): commit to these digits instead of
    preProcess's (a crafted proof, e.g. one the reference's prover refuses to
    make but its verifier accepts)."""
    base, e = pp.base, pp.exponent
    coms, mps, com_bfs = [], [], []
    for k, (v, bf) in enumerate(witnesses):
        ds = digits(v, base, e) if digit_rows is None else digit_rows[k]
        row, mrow, cbf = [], [], 0
        for i, d in enumerate(ds):
            dbf = rnd.zr("%s/digit/%d/%d/bf" % (tag, k, i))
            com = C.g1_add(C.g1_mul(pp.ped[0], d), C.g1_mul(pp.ped[1], dbf))
            row.append(com)
            mrow.append(membership_prove(pp, rnd, "%s/mp/%d/%d" % (tag, k, i),
                                         pp.signed_values[d], d, dbf, com))
            # commitmentBlindingFactor += bf * pow mod r (:327-329)
            cbf = (cbf + dbf * digit_weight(base, i)) % R
        coms.append(row)
        mps.append(mrow)
        com_bfs.append(cbf)
    rtype = rnd.zr(tag + "/r_type")
    rv = [rnd.zr("%s/r_value/%d" % (tag, k)) for k in range(len(tokens))]
    rcbf = [rnd.zr("%s/r_combf/%d" % (tag, k)) for k in range(len(tokens))]
    rtbf = [rnd.zr("%s/r_tokbf/%d" % (tag, k)) for k in range(len(tokens))]
    ctoks = [C.g1_sum([C.g1_mul(pp.ped[0], rtype), C.g1_mul(pp.ped[1], rv[k]),
                       C.g1_mul(pp.ped[2], rtbf[k])]) for k in range(len(tokens))]
    cvals = [C.g1_add(C.g1_mul(pp.ped[0], rv[k]), C.g1_mul(pp.ped[1], rcbf[k]))
             for k in range(len(tokens))]
    chal = C.hash_to_zr(range_transcript(pp, tokens, ctoks, cvals, coms))
    eq_val = [(rv[k] + chal * witnesses[k][0]) % R for k in range(len(tokens))]
    eq_tbf = [(rtbf[k] + chal * witnesses[k][1]) % R for k in range(len(tokens))]
    eq_cbf = [(rcbf[k] + chal * com_bfs[k]) % R for k in range(len(tokens))]
    eq_type = (rtype + chal * type_hash(ttype)) % R
    mp_json = J.enc_list(list(range(len(tokens))), lambda k: J.enc_struct([
        ("Commitments", J.enc_list(coms[k], enc_g1)),
        ("SignatureProofs", J.enc_list(mps[k], enc_membership))]))
    return J.enc_struct([
        ("Challenge", enc_zr(chal)),
        ("EqualityProofs", J.enc_struct([
            ("Type", enc_zr(eq_type)),
            ("Value", J.enc_list(eq_val, enc_zr)),
            ("TokenBlindingFactor", J.enc_list(eq_tbf, enc_zr)),
            ("CommitmentBlindingFactor", J.enc_list(eq_cbf, enc_zr))])),
        ("MembershipProofs", mp_json),
    ]).encode()


def range_verify(pp, tokens, raw):
    """range/proof.go:211-284 Verify (+ recomputeCommitments :393-444)."""
    try:
        v = J.parse(raw if raw is not None else b"")
    except J.GoJSONError as ex:
        raise VerifyError(ERR_PARSE, str(ex))
    if v[0] == "null":
        v = ("obj", [])
    v = J.resolve(v, RANGE_SCHEMA)
    chal = dec_zr(J.field(v, "Challenge"))
    eqv = J.field(v, "EqualityProofs")
    eq = None
    if eqv is not None and eqv[0] != "null":
        eq = {"Type": dec_zr(J.field(eqv, "Type")),
              "Value": J.dec_list(J.field(eqv, "Value"), dec_zr),
              "TokenBlindingFactor": J.dec_list(J.field(eqv, "TokenBlindingFactor"), dec_zr),
              "CommitmentBlindingFactor": J.dec_list(J.field(eqv, "CommitmentBlindingFactor"), dec_zr)}

    def dec_mp(x):
        if x is None or x[0] == "null":
            return None
        return {"Commitments": J.dec_list(J.field(x, "Commitments"), dec_g1),
                "SignatureProofs": J.dec_list(J.field(x, "SignatureProofs"), dec_membership)}

    mps = J.dec_list(J.field(v, "MembershipProofs"), dec_mp) or []
    if len(mps) != len(tokens):
        raise VerifyError(ERR_MALFORMED, "range proof not well formed")
    jobs = []
    for k in range(len(tokens)):
        if mps[k] is None:
            raise VerifyError(ERR_MALFORMED, "range proof not well formed")
        cs = mps[k]["Commitments"] or []
        sps = mps[k]["SignatureProofs"] or []
        if len(cs) != len(sps):
            raise VerifyError(ERR_MALFORMED, "range proof not well formed")
        for i in range(len(cs)):
            jobs.append((cs[i], sps[i]))
    # membership verifications run in goroutines: a nil proof panics the
    # process; otherwise the (deterministically: first) error is returned.
    for _, sp in jobs:
        if sp is None:
            raise Panic("nil membership proof")
    first_err = None
    for com, sp in jobs:
        try:
            membership_verify(pp, com, sp)
        except Panic:
            raise
        except VerifyError as ex:
            if first_err is None:
                first_err = ex
    if first_err is not None:
        raise first_err
    # recomputeCommitments (range/proof.go:393-444)
    if eq is None:
        raise VerifyError(ERR_MALFORMED, "range proof not well formed")
    n = len(tokens)
    for key in ("Value", "TokenBlindingFactor", "CommitmentBlindingFactor"):
        if len(eq[key] or []) != n:
            raise VerifyError(ERR_MALFORMED, "range proof not well formed")
    ctoks = [schnorr_recompute(pp.ped, [eq["Type"], eq["Value"][j], eq["TokenBlindingFactor"][j]],
                               tokens[j], chal) for j in range(n)]
    cvals = []
    for j in range(n):
        cs = mps[j]["Commitments"] or []
        if len(cs) != pp.exponent:
            raise VerifyError(ERR_MALFORMED, "range proof not well formed")
        com = None
        for i in range(pp.exponent):
            if cs[i] is None:
                raise Panic("nil commitment")
            com = C.g1_add(com, C.g1_mul(pt(cs[i]), digit_weight(pp.base, i) % R))
        cvals.append(schnorr_recompute(pp.ped[:2], [eq["Value"][j], eq["CommitmentBlindingFactor"][j]],
                                       com, chal))
    coms = [[pt(c) for c in mps[j]["Commitments"]] for j in range(n)]
    if _traced(ERR_RANGE, C.hash_to_zr(range_transcript(pp, tokens, ctoks, cvals, coms))) != chal:
        raise VerifyError(ERR_RANGE, "invalid range proof")


# ------------------------------------------------------------------ transfer WF
def wf_prove(pp, rnd, tag, ins, outs, in_w, out_w, ttype):
    """transfer/wellformedness.go:131-154 Prove, computeProof :243-304, computeCommitments :307-378,
    computeProof :397-458.  in_w/out_w: lists of (value, bf)."""
    ni, no = len(ins), len(outs)
    rt = rnd.zr(tag + "/r_type")
    Q = C.g1_mul(pp.ped[0], rt)
    riv = [rnd.zr("%s/r_inv/%d" % (tag, i)) for i in range(ni)]
    ribf = [rnd.zr("%s/r_inbf/%d" % (tag, i)) for i in range(ni)]
    rs = rnd.zr(tag + "/r_sum")
    rov = [rnd.zr("%s/r_outv/%d" % (tag, i)) for i in range(no)]
    robf = [rnd.zr("%s/r_outbf/%d" % (tag, i)) for i in range(no)]
    cin, cout = [], []
    insum = None
    for i in range(ni):
        Pp = C.g1_mul(pp.ped[2], ribf[i])
        cin.append(C.g1_sum([C.g1_mul(pp.ped[1], riv[i]), Q, Pp]))
        insum = C.g1_add(insum, Pp)
    insum = C.g1_add(insum, C.g1_mul(pp.ped[1], rs))
    insum = C.g1_add(insum, C.g1_mul(Q, ni))
    outsum = C.g1_add(C.g1_mul(pp.ped[1], rs), C.g1_mul(Q, no))
    for i in range(no):
        Pp = C.g1_mul(pp.ped[2], robf[i])
        cout.append(C.g1_sum([C.g1_mul(pp.ped[1], rov[i]), Q, Pp]))
        outsum = C.g1_add(outsum, Pp)
    chal = C.hash_to_zr(g1_array_bytes(cin + [insum] + cout + [outsum] + ins + outs))
    resp = lambda r_, w: (r_ + chal * w) % R
    fields = [
        ("InputBlindingFactors", J.enc_list([resp(ribf[i], in_w[i][1]) for i in range(ni)], enc_zr)),
        ("OutputBlindingFactors", J.enc_list([resp(robf[i], out_w[i][1]) for i in range(no)], enc_zr)),
        ("InputValues", J.enc_list([resp(riv[i], in_w[i][0]) for i in range(ni)], enc_zr)),
        ("OutputValues", J.enc_list([resp(rov[i], out_w[i][0]) for i in range(no)], enc_zr)),
        ("Type", enc_zr(resp(rt, type_hash(ttype)))),
        ("Sum", enc_zr(resp(rs, sum(w[0] for w in in_w) % R))),
        ("Challenge", enc_zr(chal)),
    ]
    return J.enc_struct(fields).encode()


def wf_verify(pp, ins, outs, raw):
    """transfer/wellformedness.go:157-197 Verify with parseProof :200-240."""
    try:
        v = J.parse(raw if raw is not None else b"")
    except J.GoJSONError as ex:
        raise VerifyError(ERR_PARSE, "invalid transfer proof: cannot parse proof")
    if v[0] == "null":
        v = ("obj", [])
    if v[0] != "obj":
        raise VerifyError(ERR_PARSE, "invalid transfer proof: cannot parse proof")
    wf = {k: J.dec_list(J.field(v, k), dec_zr) for k in
          ("InputBlindingFactors", "OutputBlindingFactors", "InputValues", "OutputValues")}
    for k in ("Type", "Sum", "Challenge"):
        wf[k] = dec_zr(J.field(v, k))

    def parse_proof(tokens, values, bfs):
        values, bfs = values or [], bfs or []
        if len(values) != len(tokens) or len(bfs) != len(tokens):
            raise VerifyError(ERR_MALFORMED, "failed to parse wellformedness proof")
        # ModMul(ttype, n) dereferences ttype: nil Type panics (wellformedness.go:227)
        zk = []
        agg = None
        for i, t in enumerate(tokens):
            zk.append(([wf["Type"], values[i], bfs[i]], t))
            agg = C.g1_add(agg, t)
        if wf["Type"] is None:
            raise Panic("nil Type in ModMul")
        for b in bfs:
            if b is None:
                raise VerifyError(ERR_MALFORMED, "invalid wellformedness proof")
        zk.append(([(wf["Type"] * len(tokens)) % R, wf["Sum"], sum(bfs) % R], agg))
        return zk

    zin = parse_proof(ins, wf["InputValues"], wf["InputBlindingFactors"])
    cin = [schnorr_recompute(pp.ped, p, s, wf["Challenge"]) for p, s in zin]
    zout = parse_proof(outs, wf["OutputValues"], wf["OutputBlindingFactors"])
    cout = [schnorr_recompute(pp.ped, p, s, wf["Challenge"]) for p, s in zout]
    if _traced(ERR_WF, C.hash_to_zr(g1_array_bytes(cin + cout + ins + outs))) != wf["Challenge"]:
        raise VerifyError(ERR_WF, "invalid zero-knowledge transfer")


# ------------------------------------------------------------------ transfer
def transfer_prove(pp, rnd, ins, outs, in_w, out_w, ttype, tag="tx", digit_rows=None):
    """transfer/transfer.go:89-121 Prove -> json.Marshal(Proof{WF, Range}).
    digit_rows: see range_prove (crafted fixtures only)."""
    rc = None
    if not (len(ins) == 1 and len(outs) == 1):
        rc = range_prove(pp, rnd, tag + "/range", outs, out_w, ttype, digit_rows)
    wf = wf_prove(pp, rnd, tag + "/wf", ins, outs, in_w, out_w, ttype)
    return J.enc_struct([("WellFormedness", J.enc_bytes(wf)),
                         ("RangeCorrectness", J.enc_bytes(rc))]).encode()


def transfer_verify(pp, ins, outs, proof):
    """transfer/transfer.go:66-77 NewVerifier + :124-154 Verify.
    Returns (accepted, code, message)."""
    try:
        try:
            v = J.parse(proof)
            if v[0] == "null":
                v = ("obj", [])
            wfb = J.dec_bytes(J.field(v, "WellFormedness"))
            rcb = J.dec_bytes(J.field(v, "RangeCorrectness"))
        except J.GoJSONError as ex:
            raise VerifyError(ERR_PARSE, "invalid transfer proof")
        wf_err = None
        try:
            wf_verify(pp, ins, outs, wfb)
        except Panic:
            raise
        except VerifyError as ex:
            wf_err = ex
        except J.GoJSONError:
            wf_err = VerifyError(ERR_PARSE, "invalid transfer proof: cannot parse proof")
        rng_err = None
        if not (len(ins) == 1 and len(outs) == 1):
            try:
                range_verify(pp, outs, rcb)
            except Panic:
                raise
            except VerifyError as ex:
                rng_err = ex
            except J.GoJSONError as ex:
                rng_err = VerifyError(ERR_PARSE, str(ex))
        if wf_err is not None:
            raise wf_err
        if rng_err is not None:
            raise rng_err
        return True, OK, ""
    except VerifyError as ex:
        return False, ex.code, str(ex)


# ------------------------------------------------------------------ issue
def issue_wf_prove(pp, rnd, tag, tokens, wit, ttype, anonymous=False):
    """issue/wellformedness.go:74-184 (non-anonymous unless ``anonymous``)."""
    Q = None
    rt = None
    if anonymous:
        rt = rnd.zr(tag + "/r_type")
        Q = C.g1_mul(pp.ped[0], rt)
    rv, rbf, coms = [], [], []
    for i in range(len(tokens)):
        rv.append(rnd.zr("%s/r_value/%d" % (tag, i)))
        rbf.append(rnd.zr("%s/r_bf/%d" % (tag, i)))
        coms.append(C.g1_sum([C.g1_mul(pp.ped[1], rv[i]), C.g1_mul(pp.ped[2], rbf[i]), Q]))
    chal = C.hash_to_zr(g1_array_bytes(coms + tokens))
    fields = [("Type", enc_zr((rt + chal * type_hash(ttype)) % R) if anonymous else "null"),
              ("Values", J.enc_list([(rv[i] + chal * wit[i][0]) % R for i in range(len(tokens))], enc_zr)),
              ("BlindingFactors", J.enc_list([(rbf[i] + chal * wit[i][1]) % R for i in range(len(tokens))], enc_zr)),
              ("TypeInTheClear", J.enc_str("" if anonymous else ttype)),
              ("Challenge", enc_zr(chal))]
    return J.enc_struct(fields).encode()


def issue_prove(pp, rnd, tokens, wit, ttype, anonymous=False, tag="issue", digit_rows=None):
    """issue/issue.go:162-184 Prove (digit_rows: see range_prove)."""
    wf = issue_wf_prove(pp, rnd, tag + "/wf", tokens, wit, ttype, anonymous)
    rc = range_prove(pp, rnd, tag + "/range", tokens, wit, ttype, digit_rows)
    return J.enc_struct([("WellFormedness", J.enc_bytes(wf)),
                         ("RangeCorrectness", J.enc_bytes(rc))]).encode()


def issue_wf_verify(pp, tokens, anonymous, raw):
    """issue/wellformedness.go:206-265."""
    # wf.Deserialize (json.Unmarshal) covers the syntax and every field's
    # decoding: any error there is "failed to verify well-formedness proof"
    try:
        v = J.parse(raw if raw is not None else b"")
        if v[0] == "null":
            v = ("obj", [])
        wf = {"Type": dec_zr(J.field(v, "Type")),
              "Values": J.dec_list(J.field(v, "Values"), dec_zr),
              "BlindingFactors": J.dec_list(J.field(v, "BlindingFactors"), dec_zr),
              "TypeInTheClear": J.dec_string(J.field(v, "TypeInTheClear")),
              "Challenge": dec_zr(J.field(v, "Challenge"))}
    except J.GoJSONError:
        raise VerifyError(ERR_PARSE, "failed to verify well-formedness proof")
    c = wf["Challenge"]
    if c is None:
        raise VerifyError(ERR_MALFORMED, "failed to verify well-formedness proof: invalid public parameters")
    if not anonymous:
        wf["Type"] = (c * type_hash(wf["TypeInTheClear"])) % R
    vals, bfs = wf["Values"] or [], wf["BlindingFactors"] or []
    if len(vals) != len(tokens) or len(bfs) != len(tokens):
        raise VerifyError(ERR_MALFORMED, "well-formedness proof is not well formed: length mismatch")
    coms = [schnorr_recompute(pp.ped, [wf["Type"], vals[i], bfs[i]], tokens[i], c)
            for i in range(len(tokens))]
    if _traced(ERR_WF, C.hash_to_zr(g1_array_bytes(coms + tokens))) != c:
        raise VerifyError(ERR_WF, "invalid well-formedness proof")


def issue_verify(pp, tokens, proof, anonymous=False):
    """issue/issue.go:194-223 Verify (WF then range, sequential)."""
    try:
        try:
            v = J.parse(proof)
            if v[0] == "null":
                v = ("obj", [])
            wfb = J.dec_bytes(J.field(v, "WellFormedness"))
            rcb = J.dec_bytes(J.field(v, "RangeCorrectness"))
        except J.GoJSONError:
            raise VerifyError(ERR_PARSE, "invalid issue proof")
        issue_wf_verify(pp, tokens, anonymous, wfb)
        try:
            range_verify(pp, tokens, rcb)
        except J.GoJSONError as ex:
            raise VerifyError(ERR_PARSE, str(ex))
        return True, OK, ""
    except VerifyError as ex:
        return False, ex.code, str(ex)

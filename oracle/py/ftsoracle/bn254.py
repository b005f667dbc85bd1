"""BN254 arithmetic restated in plain Python integers (TEST INFRASTRUCTURE ONLY).

Restates what the reference obtains from ``github.com/IBM/mathlib`` (driver
``gurvy``) on top of ``consensys/gnark-crypto v0.6.0 ecc/bn254`` -- both absent
from /root/reference, see SURVEY.md section 8c and Appendix C:

* curve constants,
* the gnark tower Fp2 = Fp[u]/(u^2+1), Fp6 = Fp2[v]/(v^3-(9+u)),
  Fp12 = Fp6[w]/(w^2-v), twist E': y^2 = x^3 + 3/(9+u) (D-type),
* optimal-ate Miller loop (loop count 6x+2, two Frobenius lines) -- the value
  after final exponentiation does not depend on line scaling,
* final exponentiation  f^((p^6-1)(p^2+1) * H) where the hard exponent H is
  selectable: ``FE_EXACT`` (default, H = (p^4-p^2+1)/r: gnark-crypto v0.6.0,
  the version IBM/mathlib 0a7378db6912 pins (reference go.mod:7,53), computes
  it with the Scott et al. ePrint 2008/490 chain) or ``FE_FUENTES`` (H =
  2x(6x^2+3x+1)(p^4-p^2+1)/r, the Fuentes-Castaneda et al. chain of later
  gnark-crypto releases).  [EXT] unpinned -- see DESIGN.md section 4.
* encodings: G1 RawBytes (64 B X||Y), G2 RawBytes (X.A1|X.A0|Y.A1|Y.A0),
  E12.Bytes (C1.B2.A1 first ... C0.B0.A0 last), HashToZr = SHA-256 mod r.

Reference call sites: Pairing2 ``sigproof/pok.go:199,201``; FExp
``sigproof/pok.go:203``; HashToZr ``transfer/wellformedness.go:193`` etc.
Everything here is written for clarity, not speed.
"""
import hashlib

P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
X = 4965661367192848881          # BN parameter (positive for bn254)
ATE = 6 * X + 2                  # optimal-ate loop count

FE_FUENTES = "fuentes"
FE_EXACT = "exact"
FE_VARIANT = FE_EXACT            # default [EXT] assumption, see module doc

# ---------------------------------------------------------------- Fp2
def f2(a0, a1=0):
    return (a0 % P, a1 % P)

F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2_sqr(a):
    return f2_mul(a, a)


def f2_muls(a, s):
    return ((a[0] * s) % P, (a[1] * s) % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    n = (a[0] * a[0] + a[1] * a[1]) % P
    ni = pow(n, P - 2, P)
    return ((a[0] * ni) % P, (-a[1] * ni) % P)


def f2_mul_xi(a):
    # (a0 + a1 u)(9 + u) = 9a0 - a1 + (a0 + 9a1) u
    return ((9 * a[0] - a[1]) % P, (a[0] + 9 * a[1]) % P)


def f2_pow(a, e):
    res = F2_ONE
    base = a
    while e:
        if e & 1:
            res = f2_mul(res, base)
        base = f2_sqr(base)
        e >>= 1
    return res


XI = (9, 1)

# ---------------------------------------------------------------- Fp6
F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)


def f6_add(a, b):
    return (f2_add(a[0], b[0]), f2_add(a[1], b[1]), f2_add(a[2], b[2]))


def f6_sub(a, b):
    return (f2_sub(a[0], b[0]), f2_sub(a[1], b[1]), f2_sub(a[2], b[2]))


def f6_neg(a):
    return (f2_neg(a[0]), f2_neg(a[1]), f2_neg(a[2]))


def f6_mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    c0 = f2_add(f2_mul(a0, b0), f2_mul_xi(f2_add(f2_mul(a1, b2), f2_mul(a2, b1))))
    c1 = f2_add(f2_add(f2_mul(a0, b1), f2_mul(a1, b0)), f2_mul_xi(f2_mul(a2, b2)))
    c2 = f2_add(f2_add(f2_mul(a0, b2), f2_mul(a1, b1)), f2_mul(a2, b0))
    return (c0, c1, c2)


def f6_mul_v(a):
    return (f2_mul_xi(a[2]), a[0], a[1])


def f6_inv(a):
    a0, a1, a2 = a
    t0 = f2_sub(f2_sqr(a0), f2_mul_xi(f2_mul(a1, a2)))
    t1 = f2_sub(f2_mul_xi(f2_sqr(a2)), f2_mul(a0, a1))
    t2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    den = f2_add(f2_mul(a0, t0), f2_mul_xi(f2_add(f2_mul(a2, t1), f2_mul(a1, t2))))
    di = f2_inv(den)
    return (f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di))


# ---------------------------------------------------------------- Fp12
F12_ONE = (F6_ONE, F6_ZERO)


def f12_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0 = f6_mul(a0, b0)
    t1 = f6_mul(a1, b1)
    c0 = f6_add(t0, f6_mul_v(t1))
    c1 = f6_add(f6_mul(a0, b1), f6_mul(a1, b0))
    return (c0, c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    a0, a1 = a
    den = f6_sub(f6_mul(a0, a0), f6_mul_v(f6_mul(a1, a1)))
    di = f6_inv(den)
    return (f6_mul(a0, di), f6_neg(f6_mul(a1, di)))


def f12_pow(a, e):
    if e < 0:
        return f12_pow(f12_inv(a), -e)
    res = F12_ONE
    for bit in bin(e)[2:]:
        res = f12_sqr(res)
        if bit == "1":
            res = f12_mul(res, a)
    return res


def f12_eq(a, b):
    return a == b


def _to_w(a):
    """Tower -> coefficients of 1, w, w^2, ..., w^5 (w^2 = v, w^6 = xi)."""
    (b00, b01, b02), (b10, b11, b12) = a
    return [b00, b10, b01, b11, b02, b12]


def _from_w(c):
    return ((c[0], c[2], c[4]), (c[1], c[3], c[5]))


# gamma_k = xi^(k(p-1)/6): w^p = gamma_1 * w
_GAMMA1 = [f2_pow(XI, k * (P - 1) // 6) for k in range(6)]


def f12_frob(a, n=1):
    for _ in range(n):
        c = _to_w(a)
        c = [f2_mul(f2_conj(c[k]), _GAMMA1[k]) for k in range(6)]
        a = _from_w(c)
    return a


# ---------------------------------------------------------------- G1
B1 = 3
G1_GEN = (1, 2)
G1_INF = None


def g1_on_curve(pt):
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - B1) % P == 0


def g1_neg(pt):
    if pt is None:
        return None
    return (pt[0], (-pt[1]) % P)


def g1_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    if a[0] == b[0]:
        if (a[1] + b[1]) % P == 0:
            return None
        lam = (3 * a[0] * a[0]) * pow(2 * a[1], P - 2, P) % P
    else:
        lam = (b[1] - a[1]) * pow(b[0] - a[0], P - 2, P) % P
    x3 = (lam * lam - a[0] - b[0]) % P
    y3 = (lam * (a[0] - x3) - a[1]) % P
    return (x3, y3)


def _jac_dbl(Pj):
    X1, Y1, Z1 = Pj
    if Z1 == 0:
        return Pj
    A = X1 * X1 % P
    B = Y1 * Y1 % P
    C = B * B % P
    D = 2 * ((X1 + B) ** 2 - A - C) % P
    E = 3 * A % P
    F = E * E % P
    X3 = (F - 2 * D) % P
    Y3 = (E * (D - X3) - 8 * C) % P
    Z3 = 2 * Y1 * Z1 % P
    return (X3, Y3, Z3)


def _jac_add_aff(Pj, q):
    X1, Y1, Z1 = Pj
    if Z1 == 0:
        return (q[0], q[1], 1)
    Z1Z1 = Z1 * Z1 % P
    U2 = q[0] * Z1Z1 % P
    S2 = q[1] * Z1 * Z1Z1 % P
    H = (U2 - X1) % P
    rr = (S2 - Y1) % P
    if H == 0:
        if rr == 0:
            return _jac_dbl(Pj)
        return (1, 1, 0)
    HH = H * H % P
    HHH = H * HH % P
    V = X1 * HH % P
    X3 = (rr * rr - HHH - 2 * V) % P
    Y3 = (rr * (V - X3) - Y1 * HHH) % P
    Z3 = Z1 * H % P
    return (X3, Y3, Z3)


def _jac_to_aff(Pj):
    X1, Y1, Z1 = Pj
    if Z1 == 0:
        return None
    zi = pow(Z1, P - 2, P)
    zi2 = zi * zi % P
    return (X1 * zi2 % P, Y1 * zi2 * zi % P)


def g1_mul(pt, k):
    """Scalar multiplication; k taken mod r (every on-curve G1 point has order r:
    cofactor 1), matching gnark's GLV ScalarMultiplication for any big.Int."""
    k %= R
    if pt is None or k == 0:
        return None
    acc = (1, 1, 0)
    for bit in bin(k)[2:]:
        acc = _jac_dbl(acc)
        if bit == "1":
            acc = _jac_add_aff(acc, pt)
    return _jac_to_aff(acc)


def g1_sum(points):
    acc = None
    for q in points:
        acc = g1_add(acc, q)
    return acc


def g1_msm(points, scalars):
    """sum_i k_i P_i: the group element gnark-crypto v0.6.0 G1Jac.MultiExp
    returns (ecc/bn254/multiexp.go [EXT], the MSM mathlib wraps for the
    BASELINE configs[2] benchmark); scalars taken mod r.  TEST-ONLY checker."""
    return g1_sum(g1_mul(pt, k) for pt, k in zip(points, scalars))


# ---------------------------------------------------------------- G2 (twist)
B2 = f2_mul((3, 0), f2_inv(XI))
G2_GEN = (
    (10857046999023057135944570762232829481370756359578518086990519993285655852781,
     11559732032986387107991004021392285783925812861821192530917403151452391805634),
    (8495653923123431417604973247489272438418190587263600148770280649306958101930,
     4082367875863433681332203403145435568316851327593401208105741076214120093531),
)


def g2_on_curve(pt):
    if pt is None:
        return True
    x, y = pt
    return f2_sub(f2_sqr(y), f2_add(f2_mul(f2_sqr(x), x), B2)) == F2_ZERO


def g2_neg(pt):
    if pt is None:
        return None
    return (pt[0], f2_neg(pt[1]))


def g2_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    if a[0] == b[0]:
        if f2_add(a[1], b[1]) == F2_ZERO:
            return None
        lam = f2_mul(f2_muls(f2_sqr(a[0]), 3), f2_inv(f2_muls(a[1], 2)))
    else:
        lam = f2_mul(f2_sub(b[1], a[1]), f2_inv(f2_sub(b[0], a[0])))
    x3 = f2_sub(f2_sub(f2_sqr(lam), a[0]), b[0])
    y3 = f2_sub(f2_mul(lam, f2_sub(a[0], x3)), a[1])
    return (x3, y3)


def g2_mul(pt, k):
    k %= R
    res = None
    add = pt
    while k:
        if k & 1:
            res = g2_add(res, add)
        add = g2_add(add, add)
        k >>= 1
    return res


def g2_frob(pt):
    """Untwist-Frobenius-twist endomorphism pi on E'."""
    if pt is None:
        return None
    x, y = pt
    gx = f2_pow(XI, (P - 1) // 3)
    gy = f2_pow(XI, (P - 1) // 2)
    return (f2_mul(f2_conj(x), gx), f2_mul(f2_conj(y), gy))


# ---------------------------------------------------------------- pairing
def _line(T, Q, Pp):
    """Line through T and Q (tangent if T == Q) evaluated at P, as Fp12.

    With psi(x', y') = (x' w^2, y' w^3) and slope lambda = lambda' w:
    l(P) = yP - lambda' xP w + (lambda' x'T - y'T) w^3.
    Returns (value, T + Q)."""
    xP, yP = Pp
    if T[0] == Q[0] and T[1] == Q[1]:
        lam = f2_mul(f2_muls(f2_sqr(T[0]), 3), f2_inv(f2_muls(T[1], 2)))
    elif T[0] == Q[0]:
        # vertical line x - x'T w^2 : lies in Fp6, killed by the final exponentiation
        val = (((xP, 0), f2_neg(T[0]), F2_ZERO), F6_ZERO)
        return val, None
    else:
        lam = f2_mul(f2_sub(Q[1], T[1]), f2_inv(f2_sub(Q[0], T[0])))
    c1_0 = f2_neg(f2_muls(lam, xP))                 # coefficient of w
    c1_1 = f2_sub(f2_mul(lam, T[0]), T[1])          # coefficient of w^3 = v w
    val = (((yP, 0), F2_ZERO, F2_ZERO), (c1_0, c1_1, F2_ZERO))
    x3 = f2_sub(f2_sub(f2_sqr(lam), T[0]), Q[0])
    y3 = f2_sub(f2_mul(lam, f2_sub(T[0], x3)), T[1])
    return val, (x3, y3)


def miller_loop(pairs):
    """Product over (P in G1, Q in G2) of the optimal-ate Miller function
    f_{6x+2,Q}(P) * l_{T,piQ}(P) * l_{T',-pi^2 Q}(P).  Pairs with an infinity
    point are skipped (gnark MillerLoop)."""
    f = F12_ONE
    for Pp, Q in pairs:
        if Pp is None or Q is None:
            continue
        g = F12_ONE
        T = Q
        bits = bin(ATE)[3:]
        for bit in bits:
            g = f12_sqr(g)
            l, T = _line(T, T, Pp)
            g = f12_mul(g, l)
            if bit == "1":
                l, T = _line(T, Q, Pp)
                g = f12_mul(g, l)
        Q1 = g2_frob(Q)
        Q2 = g2_neg(g2_frob(Q1))
        l, T = _line(T, Q1, Pp)
        g = f12_mul(g, l)
        l, T = _line(T, Q2, Pp)
        g = f12_mul(g, l)
        f = f12_mul(f, g)
    return f


PHI12 = P ** 4 - P ** 2 + 1
assert PHI12 % R == 0
HARD_EXACT = PHI12 // R
HARD_FUENTES = 2 * X * (6 * X * X + 3 * X + 1) * HARD_EXACT


def final_exp(f, variant=None):
    variant = variant or FE_VARIANT
    # easy part: f^((p^6-1)(p^2+1))
    t = f12_mul(f12_conj(f), f12_inv(f))
    t = f12_mul(f12_frob(t, 2), t)
    h = HARD_FUENTES if variant == FE_FUENTES else HARD_EXACT
    return f12_pow(t, h)


def pairing(Pp, Q, variant=None):
    return final_exp(miller_loop([(Pp, Q)]), variant)


# ---------------------------------------------------------------- encodings
def fp_bytes(a):
    return (a % P).to_bytes(32, "big")


def g1_bytes(pt):
    """gnark G1Affine.RawBytes: X||Y big-endian.  Infinity: 64 zero bytes
    ([EXT]: bn254 has no uncompressed-infinity flag; mUncompressed = 0b00)."""
    if pt is None:
        return bytes(64)
    return fp_bytes(pt[0]) + fp_bytes(pt[1])


def g2_bytes(pt):
    """gnark G2Affine.RawBytes: X.A1 | X.A0 | Y.A1 | Y.A0."""
    if pt is None:
        return bytes(128)
    (x0, x1), (y0, y1) = pt
    return fp_bytes(x1) + fp_bytes(x0) + fp_bytes(y1) + fp_bytes(y0)


def gt_bytes(f):
    """gnark E12.Bytes: C1.B2.A1 | C1.B2.A0 | ... | C0.B0.A1 | C0.B0.A0."""
    out = b""
    for c in (f[1], f[0]):
        for b in (c[2], c[1], c[0]):
            out += fp_bytes(b[1]) + fp_bytes(b[0])
    return out


class DecodeError(Exception):
    pass


def g1_from_bytes(b):
    """gnark G1Affine.SetBytes (via mathlib NewG1FromBytes, recover->error).
    Uncompressed (flags 00): coordinates are reduced mod p (fp.SetBytes) and
    the point must lie on the curve; (0,0) is the point at infinity.
    Compressed-infinity (flags 01) -> infinity.  Compressed (10/11): X then
    the smallest/largest square root."""
    if b is None or len(b) < 32:
        raise DecodeError("short buffer")
    m = b[0] & 0xC0
    if m == 0x40:
        return None
    if m == 0x00:
        if len(b) < 64:
            raise DecodeError("short buffer")
        x = int.from_bytes(b[:32], "big") % P
        y = int.from_bytes(b[32:64], "big") % P
        if x == 0 and y == 0:
            return None
        if not g1_on_curve((x, y)):
            raise DecodeError("invalid point: subgroup check failed")
        return (x, y)
    x = int.from_bytes(bytes([b[0] & 0x3F]) + b[1:32], "big")
    if x >= P:
        raise DecodeError("invalid X")
    rhs = (x * x * x + B1) % P
    y = pow(rhs, (P + 1) // 4, P)
    if y * y % P != rhs:
        raise DecodeError("invalid compressed coordinate: square root doesn't exist")
    ny = (-y) % P
    lexi_largest = y > ny                       # gnark LexicographicallyLargest
    if (m == 0xC0) != lexi_largest:
        y = ny
    return (x, y)


def g2_from_bytes(b):
    if b is None or len(b) < 128:
        raise DecodeError("short buffer")
    if b[0] & 0xC0 == 0x40:
        return None
    if b[0] & 0xC0 != 0:
        raise DecodeError("compressed G2 not supported by this oracle")
    x1 = int.from_bytes(b[0:32], "big") % P
    x0 = int.from_bytes(b[32:64], "big") % P
    y1 = int.from_bytes(b[64:96], "big") % P
    y0 = int.from_bytes(b[96:128], "big") % P
    pt = ((x0, x1), (y0, y1))
    if pt == ((0, 0), (0, 0)):
        return None
    if not g2_on_curve(pt):
        raise DecodeError("invalid G2 point")
    return pt


def hash_to_zr(data):
    """mathlib HashToZr: SHA-256 digest as a big-endian integer, mod r."""
    return int.from_bytes(hashlib.sha256(data).digest(), "big") % R


def zr_bytes(z):
    """mathlib Zr.Bytes: 32-byte big-endian (common.BigToBytes)."""
    return int(z).to_bytes(32, "big")

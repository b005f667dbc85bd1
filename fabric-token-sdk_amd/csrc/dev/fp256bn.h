// FP256BN (AMCL) base field and G1, the curve of the idemix owner identities
// (IBM/mathlib math.FP256BN_AMCL).  One field element per
// lane, Montgomery form with R = 2^256 and 8 x 32-bit limbs, like dev/fp.h --
// but q > 2^255, so a + b and the Montgomery product's pre-subtraction value
// may carry out of 8 limbs: every operation here keeps that carry (CIOS with a
// ninth word, add/sub with carry-out), and all values stay fully reduced in
// [0, q).  The G1 group law is curve.h's (y^2 = x^3 + 3, a = 0, written once
// over the coordinate field): this header supplies the field functions it calls.
//
// Replaces the amcl FP256BN FP/ECP arithmetic mathlib's Fp256bn driver uses
// (NewECPbigs, ECP.Mul/Mul2/Sub, ECP.ToBytes) -- [EXT], IBM/mathlib
// v0.0.0-20220112091634-0a7378db6912 / hyperledger fabric-amcl, not vendored.
#pragma once
#include "curve.h"
#include "fp256bn_const.h"

namespace fts {

struct fq {
  uint32_t v[8];
};

FTS_HD fq fq_const(const uint32_t* c) {
  fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = c[i];
  return r;
}

// a >= q as plain integers
FTS_HD bool fq_geq(const uint32_t a[8]) {
  uint32_t t[8];
  uint32_t mm[8];
#pragma unroll
  for (int i = 0; i < 8; i++) mm[i] = Q_MOD[i];
  return sub8(t, a, mm) == 0;
}

FTS_HD fq operator+(const fq& a, const fq& b) {
  fq s, t;
  uint32_t c = add8(s.v, a.v, b.v);
  uint32_t mm[8];
#pragma unroll
  for (int i = 0; i < 8; i++) mm[i] = Q_MOD[i];
  uint32_t br = sub8(t.v, s.v, mm);
  // s + c 2^256 >= q  <=>  carry out, or no borrow from s - q
  return (c | (br ^ 1u)) ? t : s;
}

FTS_HD fq operator-(const fq& a, const fq& b) {
  fq d, t;
  uint32_t br = sub8(d.v, a.v, b.v);
  uint32_t mm[8];
#pragma unroll
  for (int i = 0; i < 8; i++) mm[i] = Q_MOD[i];
  add8(t.v, d.v, mm);  // d + q - 2^256 when a < b
  return br ? t : d;
}

// Montgomery product (CIOS, 32-bit limbs); a, b < q, result < q.  The running
// value stays below 2q < 2^257: t[8] holds the 2^256 bit.
FTS_HD fq operator*(const fq& a, const fq& b) {
  FTS_COUNT_MUL();
  uint32_t t[10];
#pragma unroll
  for (int i = 0; i < 10; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      c = (uint64_t)a.v[j] * b.v[i] + t[j] + (c >> 32);
      t[j] = (uint32_t)c;
    }
    uint64_t s = (uint64_t)t[8] + (c >> 32);
    t[8] = (uint32_t)s;
    t[9] = (uint32_t)(s >> 32);
    uint32_t m = t[0] * Q_INV;
    c = (uint64_t)m * Q_MOD[0] + t[0];
#pragma unroll
    for (int j = 1; j < 8; j++) {
      c = (uint64_t)m * Q_MOD[j] + t[j] + (c >> 32);
      t[j - 1] = (uint32_t)c;
    }
    s = (uint64_t)t[8] + (c >> 32);
    t[7] = (uint32_t)s;
    t[8] = t[9] + (uint32_t)(s >> 32);
  }
  fq r, u;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  uint32_t mm[8];
#pragma unroll
  for (int i = 0; i < 8; i++) mm[i] = Q_MOD[i];
  uint32_t br = sub8(u.v, r.v, mm);
  return (t[8] | (br ^ 1u)) ? u : r;
}

// field functions curve.h's templates call
FTS_HD fq sqr(const fq& a) { return a * a; }
FTS_HD fq neg(const fq& a) {
  fq z;
#pragma unroll
  for (int i = 0; i < 8; i++) z.v[i] = 0;
  return z - a;
}
FTS_HD bool is_zero(const fq& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= a.v[i];
  return o == 0;
}
FTS_HD bool eqf(const fq& a, const fq& b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= a.v[i] ^ b.v[i];
  return o == 0;
}
// a^(q-2) (Fermat; a != 0), 4-bit fixed windows: 252 squarings + 63 products
FTS_HDN fq fq_inv(const fq& a) {
  fq tab[16];
  tab[0] = fq_const(Q_ONE);
#pragma nounroll
  for (int i = 1; i < 16; i++) tab[i] = tab[i - 1] * a;
  fq r = fq_const(Q_ONE);
#pragma nounroll
  for (int w = 63; w >= 0; w--) {
    r = sqr(r);
    r = sqr(r);
    r = sqr(r);
    r = sqr(r);
    uint32_t d = (Q_MINUS_2[w >> 3] >> ((w & 7) * 4)) & 15;
    if (d) r = r * tab[d];
  }
  return r;
}
FTS_HD fq inv(const fq& a) { return fq_inv(a); }
template <>
FTS_HD fq zero_of<fq>() {
  fq z;
#pragma unroll
  for (int i = 0; i < 8; i++) z.v[i] = 0;
  return z;
}
template <>
FTS_HD fq one_of<fq>() {
  return fq_const(Q_ONE);
}

typedef Aff<fq> q1a;
typedef Jac<fq> q1j;

// canonical 256-bit integer (any value) -> Montgomery form of (x mod q):
// amcl NewFPbig reduces its BIG argument mod q (x < 2^256 < 2q: one subtraction)
FTS_HD fq fq_from_int(const uint32_t a[8]) {
  fq x;
#pragma unroll
  for (int i = 0; i < 8; i++) x.v[i] = a[i];
  if (fq_geq(x.v)) {
    uint32_t mm[8];
#pragma unroll
    for (int i = 0; i < 8; i++) mm[i] = Q_MOD[i];
    sub8(x.v, x.v, mm);
  }
  return x * fq_const(Q_R2);
}

FTS_HD void fq_to_int(uint32_t out[8], const fq& a) {
  fq one;
#pragma unroll
  for (int i = 0; i < 8; i++) one.v[i] = (i == 0);
  fq r = a * one;
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = r.v[i];
}

FTS_HD bool q1_on_curve(const q1a& a) {
  fq rhs = sqr(a.x) * a.x + fq_const(Q_B);
  return eqf(sqr(a.y), rhs);
}

// HashToZr for FP256BN (mathlib Fp256bn.HashToZr: FromBytes(SHA-256) mod n):
// the digest is < 2^256 < 2n, so at most one subtraction
FTS_HD void digest_mod_n(uint32_t out[8], const uint8_t d[32]) {
  uint32_t x[8], t[8], mm[8];
  be32_to_limbs(x, d);
#pragma unroll
  for (int i = 0; i < 8; i++) mm[i] = N_MOD[i];
  uint32_t br = sub8(t, x, mm);
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = br ? x[i] : t[i];
}

}  // namespace fts

// Extension-field tower of BN254 as used by gnark bn254:
//   Fp2 = Fp[u]/(u^2 + 1), Fp6 = Fp2[v]/(v^3 - xi), xi = 9 + u,
//   Fp12 = Fp6[w]/(w^2 - v).
// Element layout matches gnark's E2/E6/E12 so E12.Bytes ordering
// (C1.B2.A1 ... C0.B0.A0) is a plain walk.
#pragma once
#include "fp.h"

namespace fts {

struct fp2 {
  fp c0, c1;
};
struct fp6 {
  fp2 c0, c1, c2;
};
struct fp12 {
  fp6 c0, c1;
};

// ----------------------------------------------------------------- Fp2
FTS_HD fp2 f2_zero() { return {fe_zero<ModP>(), fe_zero<ModP>()}; }
FTS_HD fp2 f2_one() { return {fe_one<ModP>(), fe_zero<ModP>()}; }
FTS_HD fp2 f2_const(const uint32_t c[2][8]) { return {fe_const<ModP>(c[0]), fe_const<ModP>(c[1])}; }
FTS_HD fp2 operator+(const fp2& a, const fp2& b) { return {a.c0 + b.c0, a.c1 + b.c1}; }
FTS_HD fp2 operator-(const fp2& a, const fp2& b) { return {a.c0 - b.c0, a.c1 - b.c1}; }
FTS_HD fp2 f2_neg(const fp2& a) { return {fe_neg(a.c0), fe_neg(a.c1)}; }
FTS_HD fp2 f2_dbl(const fp2& a) { return {a.c0 + a.c0, a.c1 + a.c1}; }
FTS_HD fp2 f2_conj(const fp2& a) { return {a.c0, fe_neg(a.c1)}; }
FTS_HD bool f2_is_zero(const fp2& a) { return fe_is_zero(a.c0) && fe_is_zero(a.c1); }
FTS_HD bool f2_eq(const fp2& a, const fp2& b) { return fe_eq(a.c0, b.c0) && fe_eq(a.c1, b.c1); }

// Karatsuba: 3 Fp multiplications
FTS_HD fp2 operator*(const fp2& a, const fp2& b) {
  fp t0 = a.c0 * b.c0;
  fp t1 = a.c1 * b.c1;
  fp t2 = (a.c0 + a.c1) * (b.c0 + b.c1);
  return {t0 - t1, t2 - t0 - t1};
}

// (a0 + a1 u)^2 = (a0 + a1)(a0 - a1) + 2 a0 a1 u
FTS_HD fp2 f2_sqr(const fp2& a) {
  fp t = a.c0 * a.c1;
  return {(a.c0 + a.c1) * (a.c0 - a.c1), t + t};
}

FTS_HD fp2 f2_mul_fp(const fp2& a, const fp& s) { return {a.c0 * s, a.c1 * s}; }

// multiply by xi = 9 + u: (9a0 - a1) + (a0 + 9a1) u
FTS_HD fp2 f2_mul_xi(const fp2& a) {
  fp a0_2 = a.c0 + a.c0, a0_4 = a0_2 + a0_2, a0_8 = a0_4 + a0_4, a0_9 = a0_8 + a.c0;
  fp a1_2 = a.c1 + a.c1, a1_4 = a1_2 + a1_2, a1_8 = a1_4 + a1_4, a1_9 = a1_8 + a.c1;
  return {a0_9 - a.c1, a.c0 + a1_9};
}

FTS_HD fp2 f2_inv_inl(const fp2& a) {
  fp n = fe_sqr(a.c0) + fe_sqr(a.c1);
  fp ni = fp_inv_var(n);  // variable time: every value inverted on this path is public
  return {a.c0 * ni, fe_neg(a.c1 * ni)};
}
// out of line where the caller's registers are tight (a call frame instead of spills)
FTS_HDN fp2 f2_inv(const fp2& a) { return f2_inv_inl(a); }

// ----------------------------------------------------------------- Fp6
FTS_HD fp6 f6_zero() { return {f2_zero(), f2_zero(), f2_zero()}; }
FTS_HD fp6 f6_one() { return {f2_one(), f2_zero(), f2_zero()}; }
FTS_HD fp6 operator+(const fp6& a, const fp6& b) { return {a.c0 + b.c0, a.c1 + b.c1, a.c2 + b.c2}; }
FTS_HD fp6 operator-(const fp6& a, const fp6& b) { return {a.c0 - b.c0, a.c1 - b.c1, a.c2 - b.c2}; }
FTS_HD fp6 f6_neg(const fp6& a) { return {f2_neg(a.c0), f2_neg(a.c1), f2_neg(a.c2)}; }

// Karatsuba-style: 6 Fp2 multiplications
FTS_HDN fp6 operator*(const fp6& a, const fp6& b) {
  fp2 t0 = a.c0 * b.c0;
  fp2 t1 = a.c1 * b.c1;
  fp2 t2 = a.c2 * b.c2;
  fp2 c0 = (a.c1 + a.c2) * (b.c1 + b.c2) - t1 - t2;
  c0 = f2_mul_xi(c0) + t0;
  fp2 c1 = (a.c0 + a.c1) * (b.c0 + b.c1) - t0 - t1 + f2_mul_xi(t2);
  fp2 c2 = (a.c0 + a.c2) * (b.c0 + b.c2) - t0 - t2 + t1;
  return {c0, c1, c2};
}

FTS_HD fp6 f6_sqr(const fp6& a) { return a * a; }

// a * v = (xi a2, a0, a1)
FTS_HD fp6 f6_mul_v(const fp6& a) { return {f2_mul_xi(a.c2), a.c0, a.c1}; }

FTS_HD fp6 f6_mul_f2(const fp6& a, const fp2& s) { return {a.c0 * s, a.c1 * s, a.c2 * s}; }

// a * (b0 + b1 v)
FTS_HDN fp6 f6_mul_01(const fp6& a, const fp2& b0, const fp2& b1) {
  fp2 t0 = a.c0 * b0;
  fp2 t1 = a.c1 * b1;
  fp2 c0 = f2_mul_xi((a.c1 + a.c2) * b1 - t1) + t0;
  fp2 c1 = (a.c0 + a.c1) * (b0 + b1) - t0 - t1;
  fp2 c2 = (a.c0 + a.c2) * b0 - t0 + t1;
  return {c0, c1, c2};
}

FTS_HDN fp6 f6_inv(const fp6& a) {
  fp2 t0 = f2_sqr(a.c0) - f2_mul_xi(a.c1 * a.c2);
  fp2 t1 = f2_mul_xi(f2_sqr(a.c2)) - a.c0 * a.c1;
  fp2 t2 = f2_sqr(a.c1) - a.c0 * a.c2;
  fp2 den = a.c0 * t0 + f2_mul_xi(a.c2 * t1 + a.c1 * t2);
  fp2 di = f2_inv(den);
  return {t0 * di, t1 * di, t2 * di};
}

// ----------------------------------------------------------------- Fp12
FTS_HD fp12 f12_one() { return {f6_one(), f6_zero()}; }

FTS_HDN fp12 operator*(const fp12& a, const fp12& b) {
  fp6 t0 = a.c0 * b.c0;
  fp6 t1 = a.c1 * b.c1;
  fp6 c1 = (a.c0 + a.c1) * (b.c0 + b.c1) - t0 - t1;
  fp6 c0 = t0 + f6_mul_v(t1);
  return {c0, c1};
}

// complex squaring: 2 Fp6 multiplications
FTS_HDN fp12 f12_sqr(const fp12& a) {
  fp6 ab = a.c0 * a.c1;
  fp6 c0 = (a.c0 + a.c1) * (a.c0 + f6_mul_v(a.c1)) - ab - f6_mul_v(ab);
  return {c0, ab + ab};
}

FTS_HD fp12 f12_conj(const fp12& a) { return {a.c0, f6_neg(a.c1)}; }

FTS_HDN fp12 f12_inv(const fp12& a) {
  fp6 den = f6_sqr(a.c0) - f6_mul_v(f6_sqr(a.c1));
  fp6 di = f6_inv(den);
  return {a.c0 * di, f6_neg(a.c1 * di)};
}

FTS_HD bool f12_eq(const fp12& a, const fp12& b) {
  return f2_eq(a.c0.c0, b.c0.c0) && f2_eq(a.c0.c1, b.c0.c1) && f2_eq(a.c0.c2, b.c0.c2) &&
         f2_eq(a.c1.c0, b.c1.c0) && f2_eq(a.c1.c1, b.c1.c1) && f2_eq(a.c1.c2, b.c1.c2);
}

// f * (c0 + c3 w + c4 v w): sparse line multiplication (gnark "MulBy034")
FTS_HDN fp12 f12_mul_034(const fp12& f, const fp2& c0, const fp2& c3, const fp2& c4) {
  fp6 a = f6_mul_f2(f.c0, c0);
  fp6 b = f6_mul_01(f.c1, c3, c4);
  fp2 d0 = c0 + c3;
  fp6 e = f6_mul_01(f.c0 + f.c1, d0, c4);
  fp6 r1 = e - a - b;
  fp6 r0 = f6_mul_v(b) + a;
  return {r0, r1};
}

// Frobenius maps: coefficient of w^k (k = 2i + j for v^i w^j) scaled by gamma_{n,k}
FTS_HDN fp12 f12_frob(const fp12& a) {
  fp12 r;
  r.c0.c0 = f2_conj(a.c0.c0);
  r.c0.c1 = f2_conj(a.c0.c1) * f2_const(FROB1[2]);
  r.c0.c2 = f2_conj(a.c0.c2) * f2_const(FROB1[4]);
  r.c1.c0 = f2_conj(a.c1.c0) * f2_const(FROB1[1]);
  r.c1.c1 = f2_conj(a.c1.c1) * f2_const(FROB1[3]);
  r.c1.c2 = f2_conj(a.c1.c2) * f2_const(FROB1[5]);
  return r;
}

FTS_HDN fp12 f12_frob2(const fp12& a) {
  fp12 r;
  r.c0.c0 = a.c0.c0;
  r.c0.c1 = f2_mul_fp(a.c0.c1, fe_const<ModP>(FROB2[2][0]));
  r.c0.c2 = f2_mul_fp(a.c0.c2, fe_const<ModP>(FROB2[4][0]));
  r.c1.c0 = f2_mul_fp(a.c1.c0, fe_const<ModP>(FROB2[1][0]));
  r.c1.c1 = f2_mul_fp(a.c1.c1, fe_const<ModP>(FROB2[3][0]));
  r.c1.c2 = f2_mul_fp(a.c1.c2, fe_const<ModP>(FROB2[5][0]));
  return r;
}

FTS_HDN fp12 f12_frob3(const fp12& a) {
  fp12 r;
  r.c0.c0 = f2_conj(a.c0.c0);
  r.c0.c1 = f2_conj(a.c0.c1) * f2_const(FROB3[2]);
  r.c0.c2 = f2_conj(a.c0.c2) * f2_const(FROB3[4]);
  r.c1.c0 = f2_conj(a.c1.c0) * f2_const(FROB3[1]);
  r.c1.c1 = f2_conj(a.c1.c1) * f2_const(FROB3[3]);
  r.c1.c2 = f2_conj(a.c1.c2) * f2_const(FROB3[5]);
  return r;
}

// gnark E12.Bytes(): 12 canonical big-endian Fp words, C1.B2.A1 first.
FTS_HDN void f12_to_bytes(uint8_t* out, const fp12& a) {
  const fp2* cs[6] = {&a.c1.c2, &a.c1.c1, &a.c1.c0, &a.c0.c2, &a.c0.c1, &a.c0.c0};
  for (int k = 0; k < 6; k++) {
    uint32_t t[8];
    fe_to_int(t, cs[k]->c1);
    limbs_to_be32(out + 64 * k, t);
    fe_to_int(t, cs[k]->c0);
    limbs_to_be32(out + 64 * k + 32, t);
  }
}

}  // namespace fts

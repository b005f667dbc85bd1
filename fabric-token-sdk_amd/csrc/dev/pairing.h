// Optimal-ate pairing on BN254 (loop 6x+2 in NAF, two Frobenius lines) and the
// final exponentiation, per lane.  Replaces mathlib Curve.Pairing2 / FExp
// (gnark bn254 MillerLoop / FinalExponentiation), reference call sites
// sigproof/pok.go:199-203, sigproof/membership.go:246-247.
//
// Line formulas: homogeneous projective doubling / mixed addition on the
// D-type twist; the line through T (and Q) evaluated at P is
//   l(P) = r0*yP + (r1*xP) w + r2 v w        (sparse "034" element)
// which differs from the affine line by an Fp2 factor -- annihilated by the
// final exponentiation, so the reduced pairing is exactly gnark's.
#pragma once
#include "curve.h"

namespace fts {

struct LineCoef {
  fp2 r0, r1, r2;
};

struct g2p {
  fp2 x, y, z;  // homogeneous projective point on E'
};

FTS_HD fp fp_half(const fp& a) {
  uint32_t t[8], mm[8];
  uint32_t odd = a.v[0] & 1;
#pragma unroll
  for (int i = 0; i < 8; i++) mm[i] = odd ? P_MOD[i] : 0u;
  uint32_t top = add8(t, a.v, mm);
  fp r;
#pragma unroll
  for (int i = 0; i < 7; i++) r.v[i] = (t[i] >> 1) | (t[i + 1] << 31);
  r.v[7] = (t[7] >> 1) | (top << 31);
  return r;
}
FTS_HD fp2 f2_half(const fp2& a) { return {fp_half(a.c0), fp_half(a.c1)}; }

// T <- 2T; returns the tangent line coefficients (inline form: the one-lane
// line stage, whose loop would otherwise keep T and the coefficients in a call
// frame in scratch memory)
FTS_HD LineCoef dbl_step_inl(g2p& T) {
  fp2 A = f2_half(T.x * T.y);
  fp2 B = f2_sqr(T.y);
  fp2 C = f2_sqr(T.z);
  fp2 E = (C + C + C) * f2_const(TWIST_B);  // 3 b' Z^2
  fp2 F = E + E + E;
  fp2 G = f2_half(B + F);
  fp2 H = f2_sqr(T.y + T.z) - (B + C);
  fp2 I = E - B;
  fp2 J = f2_sqr(T.x);
  fp2 EE = f2_sqr(E);
  fp2 K = EE + EE + EE;
  T.x = A * (B - F);
  T.y = f2_sqr(G) - K;
  T.z = B * H;
  LineCoef l;
  l.r0 = f2_neg(H);
  l.r1 = J + J + J;
  l.r2 = I;
  return l;
}
FTS_HDN LineCoef dbl_step(g2p& T) { return dbl_step_inl(T); }

// T <- T + Q (Q affine); returns the chord line coefficients
FTS_HD LineCoef add_step_inl(g2p& T, const g2a& Q) {
  fp2 O = T.y - Q.y * T.z;
  fp2 L = T.x - Q.x * T.z;
  fp2 C = f2_sqr(O);
  fp2 D = f2_sqr(L);
  fp2 E = L * D;
  fp2 F = T.z * C;
  fp2 G = T.x * D;
  fp2 H = E + F - (G + G);
  fp2 t1 = T.y * E;
  T.x = L * H;
  T.y = (G - H) * O - t1;
  T.z = E * T.z;
  LineCoef l;
  l.r0 = L;
  l.r1 = f2_neg(O);
  l.r2 = Q.x * O - L * Q.y;
  return l;
}
FTS_HDN LineCoef add_step(g2p& T, const g2a& Q) { return add_step_inl(T, Q); }

FTS_HDN fp12 line_mul(const fp12& f, const LineCoef& l, const g1a& P) {
  return f12_mul_034(f, f2_mul_fp(l.r0, P.y), f2_mul_fp(l.r1, P.x), l.r2);
}

// pi(Q) and -pi^2(Q) on the twist
FTS_HD g2a tw_frob(const g2a& q) {
  g2a r;
  r.x = f2_conj(q.x) * f2_const(TW_FROB_X);
  r.y = f2_conj(q.y) * f2_const(TW_FROB_Y);
  r.inf = q.inf;
  return r;
}
FTS_HD g2a tw_frob2_neg(const g2a& q) {
  g2a r;
  r.x = f2_mul_fp(q.x, fe_const<ModP>(TW_FROB2_X));
  r.y = f2_neg(f2_mul_fp(q.y, fe_const<ModP>(TW_FROB2_Y)));
  r.inf = q.inf;
  return r;
}

FTS_HD int naf_digit(int i) {
  if (i >= 64) return 0;  // position 64: the leading digit, consumed by T = Q
  if ((ATE_NAF_POS >> i) & 1) return 1;
  if ((ATE_NAF_NEG >> i) & 1) return -1;
  return 0;
}

static constexpr int MILLER_LINES = 65 + 21 + 2;  // doublings + NAF additions + 2 Frobenius lines

// The Miller loop's step sequence (precompute_lines order): for i = 64..0 a
// doubling, then an addition of Q / -Q where the ate NAF digit is +1 / -1;
// then the additions of pi(Q) and -pi^2(Q).
enum : uint8_t { STEP_DBL = 0, STEP_ADD = 1, STEP_SUB = 2, STEP_FROB1 = 3, STEP_FROB2 = 4 };
struct MillerSteps {
  uint8_t t[MILLER_LINES];
};
constexpr MillerSteps miller_steps() {
  MillerSteps m{};
  int n = 0;
  for (int i = 64; i >= 0; i--) {
    m.t[n++] = STEP_DBL;
    bool pos = i < 64 && ((ATE_NAF_POS >> i) & 1), neg = i < 64 && ((ATE_NAF_NEG >> i) & 1);
    if (pos) m.t[n++] = STEP_ADD;
    if (neg) m.t[n++] = STEP_SUB;
  }
  m.t[n++] = STEP_FROB1;
  m.t[n++] = STEP_FROB2;
  return m;
}
static constexpr MillerSteps MILLER_STEPS = miller_steps();

// Line coefficients of a fixed G2 point, in consumption order (host precompute
// at context creation; consumed by miller_2 for the PP generator Q).
FTS_HDN int precompute_lines(LineCoef* out, const g2a& Q) {
  g2p T = {Q.x, Q.y, f2_one()};
  g2a Qn = aff_neg(Q);
  int n = 0;
#pragma nounroll
  for (int i = 64; i >= 0; i--) {
    out[n++] = dbl_step(T);
    int d = naf_digit(i);
    if (d == 1) out[n++] = add_step(T, Q);
    if (d == -1) out[n++] = add_step(T, Qn);
  }
  out[n++] = add_step(T, tw_frob(Q));
  out[n++] = add_step(T, tw_frob2_neg(Q));
  return n;
}

// Miller loop of the 2-pair product  f(P1, Qfix) * f(P2, Q2)  where Qfix is
// given by precomputed lines.  Pairs with an infinity point contribute 1
// (gnark MillerLoop skips them).
template <class LinePtr>
FTS_HDN fp12 miller_2(const LinePtr qlines, const g1a& P1, const g1a& P2, const g2a& Q2) {
  fp12 f = f12_one();
  bool use1 = !P1.inf;
  bool use2 = !(P2.inf || Q2.inf);
  g2p T = {Q2.x, Q2.y, f2_one()};
  g2a Qn = aff_neg(Q2);
  int n = 0;
#pragma nounroll
  for (int i = 64; i >= 0; i--) {
    if (i != 64) f = f12_sqr(f);
    if (use1) f = line_mul(f, qlines[n], P1);
    n++;
    if (use2) f = line_mul(f, dbl_step(T), P2);
    int d = naf_digit(i);
    if (d != 0) {
      if (use1) f = line_mul(f, qlines[n], P1);
      n++;
      if (use2) f = line_mul(f, add_step(T, d == 1 ? Q2 : Qn), P2);
    }
  }
  if (use1) {
    f = line_mul(f, qlines[n], P1);
    f = line_mul(f, qlines[n + 1], P1);
  }
  if (use2) {
    f = line_mul(f, add_step(T, tw_frob(Q2)), P2);
    f = line_mul(f, add_step(T, tw_frob2_neg(Q2)), P2);
  }
  return f;
}

// Miller loop of three pairs with precomputed lines each (the prover's
// fixed-pair membership commitment on the host: Q, PK1, PK2 all fixed)
template <class LinePtr>
FTS_HDN fp12 miller_fixed3(const LinePtr l0, const g1a& P0, const LinePtr l1, const g1a& P1, const LinePtr l2,
                           const g1a& P2) {
  fp12 f = f12_one();
  const LinePtr L[3] = {l0, l1, l2};
  const g1a* P[3] = {&P0, &P1, &P2};
  int n = 0;
#pragma nounroll
  for (int i = 64; i >= 0; i--) {
    if (i != 64) f = f12_sqr(f);
    for (int t = 0; t < 3; t++)
      if (!P[t]->inf) f = line_mul(f, L[t][n], *P[t]);
    n++;
    if (naf_digit(i) != 0) {
      for (int t = 0; t < 3; t++)
        if (!P[t]->inf) f = line_mul(f, L[t][n], *P[t]);
      n++;
    }
  }
  for (int e = 0; e < 2; e++, n++)
    for (int t = 0; t < 3; t++)
      if (!P[t]->inf) f = line_mul(f, L[t][n], *P[t]);
  return f;
}

// Miller loop for one pair with on-the-fly lines (used for tests / prover).
FTS_HDN fp12 miller_1(const g1a& P, const g2a& Q) {
  fp12 f = f12_one();
  if (P.inf || Q.inf) return f;
  g2p T = {Q.x, Q.y, f2_one()};
  g2a Qn = aff_neg(Q);
#pragma nounroll
  for (int i = 64; i >= 0; i--) {
    if (i != 64) f = f12_sqr(f);
    f = line_mul(f, dbl_step(T), P);
    int d = naf_digit(i);
    if (d == 1) f = line_mul(f, add_step(T, Q), P);
    if (d == -1) f = line_mul(f, add_step(T, Qn), P);
  }
  f = line_mul(f, add_step(T, tw_frob(Q)), P);
  f = line_mul(f, add_step(T, tw_frob2_neg(Q)), P);
  return f;
}

// Cyclotomic-subgroup squaring (Granger-Scott, ePrint 2009/565 section 3.2):
// valid only for elements of order dividing p^4 - p^2 + 1 (after the easy
// part of the final exponentiation).  9 Fp2 squarings instead of 12 Fp2
// multiplications.  Viewing Fp12 as three Fp4 = Fp2[t]/(t^2 - xi) pairs
// (c0.c0, c1.c1), (c1.c0, c0.c2), (c0.c1, c1.c2).
FTS_HDN fp12 f12_cyclo_sqr(const fp12& x) {
  fp2 t0 = f2_sqr(x.c1.c1);
  fp2 t1 = f2_sqr(x.c0.c0);
  fp2 t6 = f2_sqr(x.c1.c1 + x.c0.c0) - t0 - t1;  // 2 x4 x0
  fp2 t2 = f2_sqr(x.c0.c2);
  fp2 t3 = f2_sqr(x.c1.c0);
  fp2 t7 = f2_sqr(x.c0.c2 + x.c1.c0) - t2 - t3;  // 2 x2 x3
  fp2 t4 = f2_sqr(x.c1.c2);
  fp2 t5 = f2_sqr(x.c0.c1);
  fp2 t8 = f2_mul_xi(f2_sqr(x.c1.c2 + x.c0.c1) - t4 - t5);  // 2 x5 x1 xi
  t0 = f2_mul_xi(t0) + t1;  // x4^2 xi + x0^2
  t2 = f2_mul_xi(t2) + t3;  // x2^2 xi + x3^2
  t4 = f2_mul_xi(t4) + t5;  // x5^2 xi + x1^2
  fp12 z;
  z.c0.c0 = f2_dbl(t0 - x.c0.c0) + t0;
  z.c0.c1 = f2_dbl(t2 - x.c0.c1) + t2;
  z.c0.c2 = f2_dbl(t4 - x.c0.c2) + t4;
  z.c1.c0 = f2_dbl(t8 + x.c1.c0) + t8;
  z.c1.c1 = f2_dbl(t6 + x.c1.c1) + t6;
  z.c1.c2 = f2_dbl(t7 + x.c1.c2) + t7;
  return z;
}

// BN parameter x in non-adjacent form (24 non-zero digits over 63 positions)
static constexpr uint64_t BN_X_NAF_POS = 0x450a14044a890a01ull;
static constexpr uint64_t BN_X_NAF_NEG = 0x0020815000200010ull;

// a^x, x = BN parameter, a in the cyclotomic subgroup (a^-1 = conj(a))
FTS_HDN fp12 f12_expt(const fp12& a) {
  fp12 r = a;
  fp12 ai = f12_conj(a);
#pragma nounroll
  for (int i = 61; i >= 0; i--) {
    r = f12_cyclo_sqr(r);
    if ((BN_X_NAF_POS >> i) & 1) r = r * a;
    if ((BN_X_NAF_NEG >> i) & 1) r = r * ai;
  }
  return r;
}

// final exponentiation: easy part (p^6-1)(p^2+1), hard part
//   FUENTES: 2x(6x^2+3x+1)(p^4-p^2+1)/r  via f^(l0 + l1 p + l2 p^2 + l3 p^3),
//   l0 = 1+6x+12x^2+12x^3, l1 = 4x+6x^2+12x^3, l2 = 6x+6x^2+12x^3,
//   l3 = -1+4x+6x^2+12x^3   (Fuentes-Castaneda et al.; later gnark releases).
FTS_HDN fp12 final_exp_fuentes(const fp12& f) {
  fp12 t = f12_conj(f) * f12_inv(f);
  t = f12_frob2(t) * t;
  fp12 a = f12_expt(t);                 // t^x
  fp12 a2 = f12_cyclo_sqr(a);           // t^2x
  fp12 a6 = f12_cyclo_sqr(a2) * a2;     // t^6x
  fp12 b = f12_expt(a6);                // t^6x^2
  fp12 c = f12_expt(f12_cyclo_sqr(b));  // t^12x^3
  fp12 A = a6 * b * c;                  // l2
  fp12 B = A * f12_conj(a2);            // l1
  fp12 res = f12_frob2(A);
  res = res * (A * b * t);              // l0
  res = res * f12_frob(B);
  res = res * f12_frob3(B * f12_conj(t));  // l3
  return res;
}

// EXACT: hard part (p^4-p^2+1)/r by the Scott et al. vectorial addition chain
// (ePrint 2008/490) that gnark-crypto v0.6.0's bn254 FinalExponentiation runs
// (the version IBM/mathlib 0a7378db6912 pins, go.mod:7,53): with m the easy-part
// output and m_k = m^(x^k),
//   y0 = m^p m^p^2 m^p^3, y1 = 1/m, y2 = (m_2)^p^2, y3 = 1/(m_1)^p,
//   y4 = 1/(m_1 (m_2)^p), y5 = 1/m_2, y6 = 1/(m_3 (m_3)^p),
//   result = y0 y1^2 y2^6 y3^12 y4^18 y5^30 y6^36.
FTS_HDN fp12 final_exp_exact(const fp12& f) {
  fp12 m = f12_conj(f) * f12_inv(f);
  m = f12_frob2(m) * m;
  fp12 mx = f12_expt(m), mx2 = f12_expt(mx), mx3 = f12_expt(mx2);
  fp12 y0 = f12_frob(m) * f12_frob2(m) * f12_frob3(m);
  fp12 y1 = f12_conj(m);
  fp12 y2 = f12_frob2(mx2);
  fp12 y3 = f12_conj(f12_frob(mx));
  fp12 y4 = f12_conj(mx * f12_frob(mx2));
  fp12 y5 = f12_conj(mx2);
  fp12 y6 = f12_conj(mx3 * f12_frob(mx3));
  fp12 t0 = f12_cyclo_sqr(y6) * y4 * y5;
  fp12 t1 = y3 * y5 * t0;
  t0 = t0 * y2;
  t1 = f12_cyclo_sqr(f12_cyclo_sqr(t1) * t0);
  t0 = t1 * y1;
  t1 = t1 * y0;
  return f12_cyclo_sqr(t0) * t1;
}

// variant: 0 = exact (FTZ_FEXP_EXACT), 1 = Fuentes (FTZ_FEXP_FUENTES)
FTS_HD fp12 final_exp(const fp12& f, int variant = 0) {
  return variant == 1 ? final_exp_fuentes(f) : final_exp_exact(f);
}

}  // namespace fts

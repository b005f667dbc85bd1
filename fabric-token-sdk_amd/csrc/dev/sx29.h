// Final exponentiation in the sextet layout with carry-free Fp2 accumulation.
//
// Same sextet layout, same formulas and so the same Fp12 values as the sx_*
// routines of dev/sextet.h (lane k owns coefficient k of f = sum f_k w^k); what
// changes is the arithmetic under each lane's Fp2 sum  sum_t a_t b_t:
//   - field elements are 9 signed 29-bit limbs (dev/fp29.h, Montgomery radix
//     R = 2^261) kept BALANCED: every limb in [-2^28, 2^28], |value| <= p/2 + e;
//   - a lane sums its Fp2 products schoolbook into two rows of 17 signed 64-bit
//     columns (4 x 81 v_mad_i64_i32 per Fp2 product, no carries); one limb
//     product is <= 2^56, so the 6 terms of an Fp12 product (12 field products
//     per column, 9 limb products each: 108 x 2^56) plus the reduction's
//     multiples of p (9 x 2^56) stay below 2^63;
//   - one Montgomery reduction per sum with balanced digits m_k (|m_k| <= 2^28)
//     against the balanced limbs of p, which returns a balanced value
//     |v| < 12 (p/2)^2 / 2^261 + p/2 < 0.52 p directly -- no final subtraction;
//   - xi a, 3 r -/+ 2 a and the other small linear maps are evaluated in 64-bit
//     limb sweeps together with one quotient-estimate reduction (f29_lin2).
// The one Fp12 inversion (sx_inv, once per job) runs in the 8 x 32-bit code and
// the result is converted; the GT value leaves through f29_to_fp.  Per Fp2
// product this is ~330 VALU instructions against ~480 for the 32-bit wide
// accumulation (one v_addc per MAD plus the 16-limb add/sub chains).
#pragma once
#include "fp29.h"
#include "sextet.h"

namespace fts {

// ----------------------------------------------------------- accumulation
// FTS_SX_KARA (default 1): the lane's Fp2 sum is kept as three Karatsuba rows
//   U = sum a0 b0,  V = sum a1 b1,  W = sum (a0 + a1)(b0 + b1)
// (3 x 81 MADs per Fp2 product instead of the schoolbook 4 x 81), and the two
// rows the reduction needs are formed once per sum: re = U - V, im = W - U - V.
// The rows are computed modulo 2^64 (unsigned: they may wrap, W in particular,
// whose operands are unbalanced limb sums); re and im are the schoolbook
// column sums exactly, whose bound (108 limb products of <= 2^56 per column)
// is unchanged, so every reduced value -- and every GT byte -- is bit-identical
// to the schoolbook accumulation.  A complex square s^2 adds s0^2, s1^2 and
// (s0 + s1)^2 to the rows as three 45-MAD squarings (doubled cross products).
#ifndef FTS_SX_KARA
#define FTS_SX_KARA 1
#endif
// a limb product as an unsigned 64-bit term (rows that may wrap modulo 2^64)
FTS_HD uint64_t w29_p(int32_t a, int32_t b) { return (uint64_t)((int64_t)a * (int64_t)b); }
#if FTS_SX_KARA
struct W29 {
  uint64_t u[17], v[17], w[17];
};
FTS_HD void w29_init(W29& w) {
#pragma unroll
  for (int i = 0; i < 17; i++) w.u[i] = w.v[i] = w.w[i] = 0;
}
// w += a b (a, b balanced, or limbs within 2^29)
FTS_HD void w29_mac(W29& w, const q2& a, const q2& b) {
  FTS_COUNT_MAD(192);  // the 32-bit equivalent (3 wide products), for opcounts
  FTS_SCHED_FENCE();
  const f29 sa = f29_add(a.c0, a.c1), sb = f29_add(b.c0, b.c1);
#pragma unroll
  for (int i = 0; i < 9; i++)
#pragma unroll
    for (int j = 0; j < 9; j++) {
      w.u[i + j] += w29_p(a.c0.l[i], b.c0.l[j]);
      w.v[i + j] += w29_p(a.c1.l[i], b.c1.l[j]);
      w.w[i + j] += w29_p(sa.l[i], sb.l[j]);
    }
}
// row += x^2: cross products once with the doubled operand (|2 x_i| < 2^31)
FTS_HD void w29_row_sqr(uint64_t r[17], const f29& x) {
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int32_t d = x.l[i] + x.l[i];
    r[2 * i] += w29_p(x.l[i], x.l[i]);
#pragma unroll
    for (int j = i + 1; j < 9; j++) r[i + j] += w29_p(d, x.l[j]);
  }
}
// w += s^2 (s balanced): 3 x 45 MADs
FTS_HD void w29_sqr_acc(W29& w, const q2& s) {
  FTS_COUNT_MAD(128);
  FTS_SCHED_FENCE();
  w29_row_sqr(w.u, s.c0);
  w29_row_sqr(w.v, s.c1);
  w29_row_sqr(w.w, f29_add(s.c0, s.c1));
}
#else
struct W29 {
  int64_t re[17], im[17];
};
FTS_HD void w29_init(W29& w) {
#pragma unroll
  for (int i = 0; i < 17; i++) w.re[i] = w.im[i] = 0;
}
// w += a b (a, b balanced)
FTS_HD void w29_mac(W29& w, const q2& a, const q2& b) {
  FTS_COUNT_MAD(192);  // the 32-bit equivalent (3 wide products), for opcounts
  FTS_SCHED_FENCE();
  f29 nb1 = f29_neg(b.c1);
#pragma unroll
  for (int i = 0; i < 9; i++)
#pragma unroll
    for (int j = 0; j < 9; j++) {
      w.re[i + j] += (int64_t)a.c0.l[i] * b.c0.l[j];
      w.re[i + j] += (int64_t)a.c1.l[i] * nb1.l[j];
      w.im[i + j] += (int64_t)a.c0.l[i] * b.c1.l[j];
      w.im[i + j] += (int64_t)a.c1.l[i] * b.c0.l[j];
    }
}
#endif
// Montgomery reduction of one row, balanced digits and result
FTS_HD f29 w29_redc(int64_t c[17]) {
  FTS_COUNT_MAD(72);
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const uint32_t m = ((uint32_t)c[k] * P29_INV) & (uint32_t)F29_MASK;
    const int32_t mb = (int32_t)((m + (uint32_t)F29_HALF) & (uint32_t)F29_MASK) - F29_HALF;
#pragma unroll
    for (int j = 0; j < 9; j++) c[k + j] += (int64_t)mb * P29B[j];
    c[k + 1] += c[k] >> 29;  // c[k] is now a multiple of 2^29
  }
  f29 r;
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc += c[9 + i];
    const int32_t lo = f29_bdigit(acc);
    r.l[i] = lo;
    acc = (acc + F29_HALF) >> 29;  // = (acc - lo) / 2^29: lo is acc's balanced low digit
  }
  r.l[8] = (int32_t)acc;
  return r;
}
#if FTS_SX_KARA
FTS_HD q2 w29_reduce(W29& w) {
  int64_t re[17], im[17];
#pragma unroll
  for (int i = 0; i < 17; i++) {
    re[i] = (int64_t)(w.u[i] - w.v[i]);
    im[i] = (int64_t)(w.w[i] - (w.u[i] + w.v[i]));
  }
  return {w29_redc(re), w29_redc(im)};
}
#else
FTS_HD q2 w29_reduce(W29& w) { return {w29_redc(w.re), w29_redc(w.im)}; }
// w += s^2 (s balanced) as (s0 + s1)(s0 - s1) + 2 s0 s1 u: two limb-product rows
// instead of the four of w29_mac(w, s, s)
FTS_HD void w29_sqr_acc(W29& w, const q2& s) {
  FTS_COUNT_MAD(128);
  FTS_SCHED_FENCE();
  const f29 p = f29_add(s.c0, s.c1), d = f29_sub(s.c0, s.c1), t = f29_add(s.c0, s.c0);
#pragma unroll
  for (int i = 0; i < 9; i++)
#pragma unroll
    for (int j = 0; j < 9; j++) {
      w.re[i + j] += (int64_t)p.l[i] * d.l[j];
      w.im[i + j] += (int64_t)t.l[i] * s.c1.l[j];
    }
}
#endif

// one Fp2 product a b (a, b limbs within 2^29), Karatsuba by columns: each
// column's three sums U_c, V_c, W_c are formed and folded into re_c = U_c - V_c,
// im_c = W_c - U_c - V_c at once, so only the two result rows stay live (68
// VGPRs instead of the three accumulation rows' 102) -- for a lone product
FTS_HD q2 w29_prod1(const q2& a, const q2& b) {
  FTS_COUNT_MAD(192);  // as w29_mac (the reductions count themselves)
  FTS_SCHED_FENCE();
  const f29 sa = f29_add(a.c0, a.c1), sb = f29_add(b.c0, b.c1);
  int64_t re[17], im[17];
#pragma unroll
  for (int c = 0; c < 17; c++) {
    uint64_t u = 0, v = 0, w = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = c - i;
      if (j < 0 || j > 8) continue;
      u += w29_p(a.c0.l[i], b.c0.l[j]);
      v += w29_p(a.c1.l[i], b.c1.l[j]);
      w += w29_p(sa.l[i], sb.l[j]);
    }
    re[c] = (int64_t)(u - v);
    im[c] = (int64_t)(w - (u + v));
  }
  return {w29_redc(re), w29_redc(im)};
}

FTS_HD q2 q2_mul(const q2& a, const q2& b) {
  W29 w;
  w29_init(w);
  w29_mac(w, a, b);
  return w29_reduce(w);
}

// ----------------------------------------------------------- sextet context
struct alignas(8) Q2Slot {
  int32_t w[18];
};
typedef FTS_LDS Q2Slot QSlotT;

// BOFS: slot of the second operand's group (b_0..b_5, then xi b_0..xi b_5);
// SX_B in the 30-slot layout, 12 in the 24-slot one of k_fexp_expt (which
// leaves SX_P unused and so fits two waves per SIMD in LDS).
template <class Sync, int BOFS = SX_B>
struct Sq {
  static constexpr int B = BOFS, BX = BOFS + 6;
  int k;
  QSlotT* s;
  bool wr;
  Sync sync;
  FTS_HD void put(int slot, const q2& a) const {
    if (wr) {
#pragma unroll
      for (int i = 0; i < 9; i++) {
        s[slot].w[i] = a.c0.l[i];
        s[slot].w[9 + i] = a.c1.l[i];
      }
    }
  }
  FTS_HD q2 get(int slot) const {
    q2 a;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      a.c0.l[i] = s[slot].w[i];
      a.c1.l[i] = s[slot].w[9 + i];
    }
    return a;
  }
};

template <class X>
FTS_HD void sq_pub(const X& x, int base, const q2& v) {
  x.put(base + x.k, v);
  x.put(base + 6 + x.k, q2_mul_xi_lazy(v));  // xi v is only ever a multiplicand
}

// c = a * b, b published in SX_B / SX_BX (as sx_mul)
template <class X>
FTS_HD q2 sq_mul(X x, q2 a) {
  x.put(SX_A + x.k, a);
  x.sync();
  W29 w;
  w29_init(w);
#pragma nounroll
  for (int i = 0; i < 6; i++) {
    int j = x.k - i;
    int sb = j < 0 ? X::BX + j + 6 : X::B + j;
    w29_mac(w, x.get(SX_A + i), x.get(sb));
  }
  x.sync();
  return w29_reduce(w);
}
template <class X>
FTS_HD q2 sq_mulv(const X& x, const q2& a, const q2& b) {
  sq_pub(x, X::B, b);
  return sq_mul(x, a);
}

#ifndef FTS_SX_CYC2
#define FTS_SX_CYC2 1
#endif
#if FTS_SX_CYC2
// Granger-Scott cyclotomic squaring (as sx_cyc_sqr) with ONE Fp2 product per
// lane.  The Fp4 pairs are (a_p, a_(p+3)); pair p's even lane (k = 2p) needs
// a_p^2 + xi a_(p+3)^2, its odd lane (k = 3, 5, 1 for p = 0, 1, 2) the cross
// product a_p a_(p+3).  The odd lane computes q = a_p a_(p+3) and hands it over
// through LDS; the even lane computes P = (a_p + a_(p+3)) (a_p + xi a_(p+3)) =
// a_p^2 + xi a_(p+3)^2 + (1 + xi) q, so
//   even:   3 (P - (1 + xi) q) - 2 a_k
//   k = 3, 5: 6 q + 2 a_k,   k = 1: 6 xi q + 2 a_k
// (each a four-term linear map, f29_lin4).  The even lane's operands are
// unreduced sums (limbs within 2^29: one product, 18 limb products of <= 2^58
// per column).  Versus one general product plus one complex square per lane:
// 3 x 81 limb products instead of 3 x 81 + 3 x 45.
template <class X>
FTS_HD q2 sq_cyc_sqr(X x, q2 a) {
  const int k = x.k, odd = k & 1;
  const int p = odd ? (k == 3 ? 0 : (k == 5 ? 1 : 2)) : (k >> 1);
  sq_pub(x, SX_A, a);
  x.sync();
  q2 u = x.get(SX_A + p), v = x.get(SX_A + p + 3), xv = x.get(SX_AX + p + 3);
  q2 s = q2_sel(odd, u, q2_add(u, v)), t = q2_sel(odd, v, q2_add(u, xv));
  q2 r = w29_prod1(s, t);
  x.sync();                       // every lane has read the AX slots
  if (odd) x.put(SX_AX + p, r);   // q of pair p
  x.sync();
  q2 q = x.get(SX_AX + p);
  x.sync();  // q read before the next publish rewrites AX
  // lane coefficients: out.c0 = cr r.c0 + b0 q.c0 + g0 q.c1 + ca a.c0,
  //                    out.c1 = cr r.c1 + b1 q.c0 + g1 q.c1 + ca a.c1
  int32_t cr = odd ? 0 : 3, ca = odd ? 2 : -2;
  int32_t b0 = odd ? (k == 1 ? 54 : 6) : -30, g0 = odd ? (k == 1 ? -6 : 0) : 3;
  int32_t b1 = odd ? (k == 1 ? 6 : 0) : -3, g1 = odd ? (k == 1 ? 54 : 6) : -30;
  return {f29_lin4(r.c0, cr, q.c0, b0, q.c1, g0, a.c0, ca), f29_lin4(r.c1, cr, q.c0, b1, q.c1, g1, a.c1, ca)};
}
#else
// Granger-Scott cyclotomic squaring (as sx_cyc_sqr): even lanes 3 r - 2 a,
// odd lanes 6 r + 2 a, r the lane's one or two products.  Every lane runs one
// general product (even lanes a_{m+3} (xi a_{m+3}), odd lanes their cross
// product) and one complex squaring (even lanes a_m^2, odd lanes of zero): six
// limb-product rows per lane instead of two general products' eight.
template <class X>
FTS_HD q2 sq_cyc_sqr(X x, q2 a) {
  const int k = x.k, m = k >> 1;
  sq_pub(x, SX_A, a);
  x.sync();
  bool odd = (k & 1) != 0;
  int i1 = odd ? (k == 1 ? 5 : (k == 3 ? 3 : 4)) : m + 3;
  int j1 = odd ? (k == 1 ? SX_AX + 2 : (k == 3 ? SX_A + 0 : SX_A + 1)) : SX_AX + m + 3;
  W29 w;
  w29_init(w);
  w29_mac(w, x.get(SX_A + i1), x.get(j1));
  w29_sqr_acc(w, q2_sel(odd, q2_zero(), x.get(SX_A + m)));
  x.sync();
  q2 r = w29_reduce(w);
  const int32_t cr = odd ? 6 : 3, ca = odd ? 2 : -2;
  return {f29_lin2(r.c0, cr, a.c0, ca), f29_lin2(r.c1, cr, a.c1, ca)};
}

#endif

FTS_HD q2 sq_conj(int k, const q2& a) { return (k & 1) ? q2_neg(a) : a; }
FTS_HD q2 sq_frob1(int k, const q2& a) { return q2_mul(q2_conj(a), q2_from_fp2(f2_const(FROB1[k]))); }
FTS_HD q2 sq_frob2(int k, const q2& a) { return q2_mul(a, q2_from_fp2(f2_of_fp(fe_const<ModP>(FROB2[k][0])))); }
FTS_HD q2 sq_frob3(int k, const q2& a) { return q2_mul(q2_conj(a), q2_from_fp2(f2_const(FROB3[k]))); }

// a^x, as sx_expt (width-4 NAF), for a = park slot src.  a^3, a^5 and a^7 are
// parked in pk slots ps .. ps+2 (dev: global dword planes) and, like a from
// src, republished from there when the digit's magnitude changes, so the loop
// holds only r and the product's operands and accumulator, and no LDS beyond
// the operand slots (in registers the odd powers spill at the 256 VGPRs of two
// waves per SIMD; in LDS they would halve the waves).
template <class X, class P>
FTS_HD q2 sq_expt(X x, const P& pk, int src, int ps) {
  q2 a = pk.get(src);
  q2 a2 = sq_cyc_sqr(x, a);
  q2 a3 = sq_mulv(x, a2, a);
  pk.put(ps, a3);
  q2 a5 = sq_mulv(x, a3, a2);
  pk.put(ps + 1, a5);
  pk.put(ps + 2, sq_mul(x, a5));
  int cur = 0;
  q2 r = a;
#pragma nounroll
  for (int i = 61; i >= 0; i--) {
    r = sq_cyc_sqr(x, r);
    // in the 18-slot layout the multiplier's slots alias SX_AX, which the
    // squaring overwrites: republish before every multiplication
    if (X::B == SX_AX) cur = 0;
    if ((BN_X_W4_NZ >> i) & 1) {
      int m = ((BN_X_W4_M3 >> i) & 1) ? 3 : (((BN_X_W4_M5 >> i) & 1) ? 5 : (((BN_X_W4_M7 >> i) & 1) ? 7 : 1));
      if (m != cur) {
        sq_pub(x, X::B, pk.get(m == 1 ? src : ps + (m - 3) / 2));
        cur = m;
      }
      bool neg = (BN_X_W4_NEG >> i) & 1;
      q2 t = neg ? sq_conj(x.k, r) : r;
      t = sq_mul(x, t);
      r = neg ? sq_conj(x.k, t) : t;
    }
  }
  return r;
}

// f^-1 (as sx_inv): den = f conj(f) in Fp6 (even lanes), the Fp6 inverse by
// the f6_inv formula with one Fp2 inversion per lane (32-bit code, converted)
template <class X>
FTS_HD q2 sq_inv(X x, q2 f) {
  const int k = x.k;
  q2 fc = sq_conj(k, f);
  q2 d = sq_mulv(x, fc, f);  // lanes 0, 2, 4: d0, d1, d2; odd lanes 0
  sq_pub(x, SX_A, d);
  x.sync();
  W29 w;
  w29_init(w);
#pragma nounroll
  for (int t = 0; t < 2; t++) {
    uint32_t e = term_at(SX_INV_TAB[t], k);
    q2 u = x.get(e & 63), v = x.get((e >> 6) & 63);
    v = q2_sel((e & TM_NEG) != 0, q2_neg(v), v);
    w29_mac(w, q2_sel((e & TM_ZERO) != 0, q2_zero(), u), v);
  }
  q2 t = w29_reduce(w);
  x.put(SX_P + k, t);
  x.sync();
  W29 v;
  w29_init(v);
#pragma nounroll
  for (int s = 0; s < 3; s++) w29_mac(v, x.get(s == 0 ? SX_A + 0 : (s == 1 ? SX_AX + 4 : SX_AX + 2)), x.get(SX_P + s));
  q2 tk = x.get(SX_P + (k >> 1));
  x.sync();
  fp2 di = f2_inv_inl(q2_to_fp2(w29_reduce(v)));  // inline: the easy-part kernel has the registers
  q2 inv6 = q2_sel((k & 1) == 0, q2_mul(tk, q2_from_fp2(di)), q2_zero());
  return sq_mulv(x, fc, inv6);
}

// Values handed between the final-exponentiation phases (and parked inside a
// phase) in global memory.  Plane (s * 18 + d) holds dword d of slot s for
// every lane of the launch (lane = global thread index), so a wave's put / get
// is 18 coalesced 256-byte stores / loads.  Ghost lanes neither store nor load
// (their results are never written).  FEXP_PARK_SLOTS slots per lane.
static constexpr int FEXP_PARK_SLOTS = 10;  // the Fuentes variant's 0..6 + 7..9
struct Park {
  int32_t* base;
  uint32_t lane, stride;
  bool on;
  // plane rows are uniform pointers (scalar registers) and the lane a 32-bit
  // offset, so the 18 accesses share one address register
  FTS_HD void put(int slot, const q2& a) const {
    if (!on) return;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      (base + (size_t)(slot * 18 + i) * stride)[lane] = a.c0.l[i];
      (base + (size_t)(slot * 18 + 9 + i) * stride)[lane] = a.c1.l[i];
    }
  }
  // an Fp value (8 words of the 32-bit form) in the first 8 planes of a slot,
  // at lane `at` (the batched inversion's per-job values, see sq_fexp_easy_a)
  FTS_HD void put_fp(int slot, uint32_t at, const fp& v) const {
    if (!on) return;
#pragma unroll
    for (int i = 0; i < 8; i++) (base + (size_t)(slot * 18 + i) * stride)[at] = (int32_t)v.v[i];
  }
  FTS_HD fp get_fp(int slot, uint32_t at) const {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" ::: "memory");
#endif
    fp v;
#pragma unroll
    for (int i = 0; i < 8; i++) v.v[i] = on ? (uint32_t)(base + (size_t)(slot * 18 + i) * stride)[at] : 0u;
    return v;
  }
  FTS_HD q2 get(int slot) const {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" ::: "memory");  // reload here: the value must not stay in registers since put()
#endif
    q2 a = q2_zero();
    if (!on) return a;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      a.c0.l[i] = (base + (size_t)(slot * 18 + i) * stride)[lane];
      a.c1.l[i] = (base + (size_t)(slot * 18 + 9 + i) * stride)[lane];
    }
    return a;
  }
};

// Exact final exponentiation f^((p^12-1)/r) (Scott et al. chain, as
// final_exp_exact in pairing.h) in three phases that the device runs as
// separate kernels (k_fexp_easy, k_fexp_expt x 3, k_fexp_hard): composed in
// one kernel the phases' register needs (171, 236 and ~200 VGPRs alone) did not
// fit together under the 256 of two waves per SIMD -- the compiler spilled
// 340 VGPRs (1 KB per lane) and the kernel moved ~26x its algorithmic bytes.
// Handing m, m^x, m^(x^2), m^(x^3) over in the park planes costs 72 bytes per
// lane per value.  Park slots: 0 m, 1 m^x, 2 m^(x^2), 3 m^(x^3); 4..6 the
// odd powers a^3, a^5, a^7 inside sq_expt.
//
// easy part: m = f^((p^6-1)(p^2+1))
template <class X>
FTS_HD q2 sq_fexp_easy(const X& x, const fp2& f) {
  const int k = x.k;
  q2 F = q2_from_fp2(f);
  q2 m = sq_mulv(x, sq_conj(k, F), sq_inv(x, F));
  return sq_mulv(x, sq_frob2(k, m), m);
}
// The easy part with its one Fp inversion batched over the whole launch (the
// device path; sq_fexp_easy above is the same value in one piece).  The
// inversion f^-1 = conj(f) / N(f) needs the inverse of an Fp norm n per job:
// inverted lane by lane (binary extended Euclid, data-dependent loops) it was
// 80 % of the easy part's instructions (measured by a build without it).
//   sq_fexp_easy_a: the Fp6 norm's terms tk (per lane, slot 4), the Fp2 value D
//     (slot 5) and n = N(D) (lane 0 of the job's sextet, slot 9 planes 0..7);
//   k_fexp_binv: every n of the launch inverted together (product tree per
//     256 jobs, one Euclid per tree), written back in place (n = 0 -> 0, as
//     fp_inv_var);
//   sq_fexp_easy_b: f^-1 from tk, D and n^-1, then m as sq_fexp_easy.
// Slots 4, 5 and 9 are free until the x-powers run.
static constexpr int FEXP_EASY_TK = 4, FEXP_EASY_D = 5, FEXP_EASY_N = 9;
template <class X, class P>
FTS_HD void sq_fexp_easy_a(const X& x, const fp2& f, const P& pk, uint32_t lane0) {
  const int k = x.k;
  q2 F = q2_from_fp2(f);
  q2 fc = sq_conj(k, F);
  q2 d = sq_mulv(x, fc, F);  // lanes 0, 2, 4: d0, d1, d2; odd lanes 0
  sq_pub(x, SX_A, d);
  x.sync();
  W29 w;
  w29_init(w);
#pragma nounroll
  for (int t = 0; t < 2; t++) {
    uint32_t e = term_at(SX_INV_TAB[t], k);
    q2 u = x.get(e & 63), v = x.get((e >> 6) & 63);
    v = q2_sel((e & TM_NEG) != 0, q2_neg(v), v);
    w29_mac(w, q2_sel((e & TM_ZERO) != 0, q2_zero(), u), v);
  }
  q2 t = w29_reduce(w);
  x.put(SX_P + k, t);
  x.sync();
  W29 v;
  w29_init(v);
#pragma nounroll
  for (int s = 0; s < 3; s++) w29_mac(v, x.get(s == 0 ? SX_A + 0 : (s == 1 ? SX_AX + 4 : SX_AX + 2)), x.get(SX_P + s));
  q2 tk = x.get(SX_P + (k >> 1));
  x.sync();
  const q2 D = w29_reduce(v);
  pk.put(FEXP_EASY_TK, tk);
  pk.put(FEXP_EASY_D, D);
  if (k == 0) {
    const fp2 Df = q2_to_fp2(D);
    pk.put_fp(FEXP_EASY_N, lane0, fe_sqr(Df.c0) + fe_sqr(Df.c1));
  }
}
template <class X, class P>
FTS_HD q2 sq_fexp_easy_b(const X& x, const fp2& f, const P& pk, uint32_t lane0) {
  const int k = x.k;
  q2 F = q2_from_fp2(f);
  q2 fc = sq_conj(k, F);
  const q2 tk = pk.get(FEXP_EASY_TK);
  const fp2 Df = q2_to_fp2(pk.get(FEXP_EASY_D));
  const fp ni = pk.get_fp(FEXP_EASY_N, lane0);
  const fp2 di = {Df.c0 * ni, fe_neg(Df.c1 * ni)};  // D^-1, as f2_inv_inl
  q2 inv6 = q2_sel((k & 1) == 0, q2_mul(tk, q2_from_fp2(di)), q2_zero());
  q2 m = sq_mulv(x, sq_conj(k, F), sq_mulv(x, fc, inv6));
  return sq_mulv(x, sq_frob2(k, m), m);
}

// hard part from the four parked powers: y0 y1^2 y2^6 y3^12 y4^18 y5^30 y6^36 as
//   t0 = y6^2 y4 y5,  t1 = y3 y5 t0,  t0 <- t0 y2,  t1 <- (t1^2 t0)^2,
//   result = (t1 y1)^2 (t1 y0)
// (the products of sx_final_exp_exact, ordered so that at most three Fp12
// values are live next to a product; inputs reloaded from the park slots)
template <class X, class P>
FTS_HD fp2 sq_fexp_hard_exact(const X& x, const P& pk) {
  const int k = x.k;
  q2 t0 = pk.get(3);                                                         // m^(x^3)
  t0 = sq_cyc_sqr(x, sq_conj(k, sq_mulv(x, t0, sq_frob1(k, t0))));         // y6^2
  q2 u = pk.get(1);                                                          // m^x
  t0 = sq_mulv(x, t0, sq_conj(k, sq_mulv(x, u, sq_frob1(k, pk.get(2)))));  // y6^2 y4
  q2 y5 = sq_conj(k, pk.get(2));
  t0 = sq_mulv(x, t0, y5);                                                   // t0 = y6^2 y4 y5
  u = sq_mulv(x, sq_conj(k, sq_frob1(k, u)), y5);                            // y3 y5
  q2 t1 = sq_mulv(x, u, t0);                                                 // t1 = y3 y5 t0
  t0 = sq_mulv(x, t0, sq_frob2(k, pk.get(2)));                               // t0 y2
  t1 = sq_cyc_sqr(x, sq_mulv(x, sq_cyc_sqr(x, t1), t0));
  q2 m = pk.get(0);
  u = sq_mulv(x, sq_frob1(k, m), sq_frob2(k, m));
  u = sq_mulv(x, u, sq_frob3(k, m));                                         // y0
  t0 = sq_mulv(x, t1, sq_conj(k, m));
  t1 = sq_mulv(x, t1, u);
  return q2_to_fp2(sq_mulv(x, sq_cyc_sqr(x, t0), t1));
}
// the three phases composed (host emulation; the device launches them apart)
template <class X, class P>
FTS_HD fp2 sq_final_exp_exact(const X& x, const fp2& f, const P& pk) {
  pk.put(0, sq_fexp_easy(x, f));
  for (int e = 0; e < 3; e++) pk.put(e + 1, sq_expt(x, pk, e, 4));
  return sq_fexp_hard_exact(x, pk);
}

// Fuentes-Castaneda multiple (the selectable FTZ_FEXP_FUENTES variant), phased
// like the exact one (k_fexp_easy, k_fexp_expt, k_fexp_fc_mid1, k_fexp_expt,
// k_fexp_fc_mid2, k_fexp_expt, k_fexp_fc_hard).  Slots: 0 t (easy part), 1 a =
// t^x, 2 a2, 3 a6, 4 b = a6^x, 5 b^2, 6 c = (b^2)^x; the x-powers' odd powers
// in FC_EXPT_SLOT ..+2.
static constexpr int FC_EXPT_SLOT = 7;
template <class X, class P>
FTS_HD void sq_fc_mid1(const X& x, const P& pk) {  // a2 = a^2, a6 = a2^3
  q2 a2 = sq_cyc_sqr(x, pk.get(1));
  pk.put(2, a2);
  pk.put(3, sq_mulv(x, sq_cyc_sqr(x, a2), a2));
}
template <class X, class P>
FTS_HD void sq_fc_mid2(const X& x, const P& pk) {  // b^2
  pk.put(5, sq_cyc_sqr(x, pk.get(4)));
}
template <class X, class P>
FTS_HD fp2 sq_fc_hard(const X& x, const P& pk) {
  const int k = x.k;
  q2 b = pk.get(4);
  q2 A = sq_mulv(x, sq_mulv(x, pk.get(3), b), pk.get(6));
  q2 B = sq_mulv(x, A, sq_conj(k, pk.get(2)));
  q2 res = sq_mulv(x, sq_frob2(k, A), sq_mulv(x, sq_mulv(x, A, b), pk.get(0)));
  res = sq_mulv(x, res, sq_frob1(k, B));
  res = sq_mulv(x, res, sq_frob3(k, sq_mulv(x, B, sq_conj(k, pk.get(0)))));
  return q2_to_fp2(res);
}
template <class X, class P>
FTS_HD fp2 sq_final_exp(const X& x, const fp2& f, const P& pk) {
  pk.put(0, sq_fexp_easy(x, f));
  pk.put(1, sq_expt(x, pk, 0, FC_EXPT_SLOT));
  sq_fc_mid1(x, pk);
  pk.put(4, sq_expt(x, pk, 3, FC_EXPT_SLOT));
  sq_fc_mid2(x, pk);
  pk.put(6, sq_expt(x, pk, 5, FC_EXPT_SLOT));
  return sq_fc_hard(x, pk);
}

// ----------------------------------------------------------- Miller f-chain
// Lines of the fixed Q (precompute_lines order) in the balanced form, built
// once per context (k_qlines).
struct LineCoef29 {
  q2 r0, r1, r2;
};
FTS_HD LineCoef29 linecoef29(const LineCoef& l) { return {q2_from_fp2(l.r0), q2_from_fp2(l.r1), q2_from_fp2(l.r2)}; }

// a b / 2^261 balanced (one row of the accumulation)
FTS_HD f29 f29_mulb(const f29& a, const f29& b) {
  int64_t c[17];
#pragma unroll
  for (int i = 0; i < 17; i++) c[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++)
#pragma unroll
    for (int j = 0; j < 9; j++) c[i + j] += (int64_t)a.l[i] * b.l[j];
  return w29_redc(c);
}

#if FTS_SX_KARA
// the Karatsuba rows take the same three squarings as w29_sqr_acc
FTS_HD void w29_sqr3_acc(W29& w, const q2& s) {
  FTS_COUNT_MAD(32);  // the schoolbook variant's count (160), for opcounts
  w29_sqr_acc(w, s);
}
#else
// w += s^2 (s balanced) as s0 s0 - s1 s1 + (2 s0) s1 u: three limb-product rows
// (the column bound stays that of w29_mac(w, s, s): 18 units of 2^56 per row)
FTS_HD void w29_sqr3_acc(W29& w, const q2& s) {
  FTS_COUNT_MAD(160);
  FTS_SCHED_FENCE();
  const f29 t = f29_add(s.c0, s.c0), n1 = f29_neg(s.c1);
#pragma unroll
  for (int i = 0; i < 9; i++)
#pragma unroll
    for (int j = 0; j < 9; j++) {
      w.re[i + j] += (int64_t)s.c0.l[i] * s.c0.l[j];
      w.re[i + j] += (int64_t)s.c1.l[i] * n1.l[j];
      w.im[i + j] += (int64_t)t.l[i] * s.c1.l[j];
    }
}
#endif

// c = a^2 (as sx_sqr): a, xi a and 2 a published (2 a unreduced: its limbs
// are within 2^29 and SX_SQR4_TAB gives every lane at most 6 operand units).
// Every lane runs three general products (even lanes SX_SQR4_TAB rows 1..3,
// odd lanes rows 0..2) and one three-row square (even lanes the diagonal
// a_{k/2}^2 of row 0, odd lanes of zero, their row 3 being empty): 15 limb-
// product rows per lane instead of 16.
template <class X>
FTS_HD q2 sq_sqr(X x, q2 a) {
  const int k = x.k;
  const bool odd = (k & 1) != 0;
  sq_pub(x, SX_A, a);
  x.put(SX_A2 + k, {f29_add(a.c0, a.c0), f29_add(a.c1, a.c1)});
  x.sync();
  W29 w;
  w29_init(w);
#pragma nounroll
  for (int t = 0; t < 3; t++) {
    uint32_t e = term_at(SX_SQR4_TAB[odd ? t : t + 1], k);
    w29_mac(w, x.get(e & 63), x.get((e >> 6) & 63));
  }
  w29_sqr3_acc(w, q2_sel(odd, q2_zero(), x.get(SX_A + (k >> 1))));
  x.sync();
  return w29_reduce(w);
}

// f * (l0 + l1 w + l3 w^3), the line in registers of every lane (as sx_mul_line_r)
template <class X>
FTS_HD q2 sq_mul_line_r(const X& x, const q2& f, const q2& l0, const q2& l1, const q2& l3) {
  sq_pub(x, SX_A, f);
  x.sync();
  W29 w;
  w29_init(w);
#pragma nounroll
  for (int t = 0; t < 3; t++) {
    int j = x.k - (t == 0 ? 0 : (t == 1 ? 1 : 3));
    int sb = j < 0 ? SX_AX + j + 6 : SX_A + j;
    w29_mac(w, t == 0 ? l0 : (t == 1 ? l1 : l3), x.get(sb));
  }
  x.sync();
  return w29_reduce(w);
}

// f * (pair-2 line s), the three evaluated coefficients read from the line
// buffer inside the term loop, one at a time (FTS_MILLER_EVLINE_IN_LOOP; the
// default loads all three before the product, sq_mul_line_r, which hides the
// load latency and fits the registers since the multiplicands are pinned)
#ifndef FTS_MILLER_EVLINE_IN_LOOP
#define FTS_MILLER_EVLINE_IN_LOOP 0
#endif
template <class X>
FTS_HD q2 sq_mul_evline(const X& x, const q2& f, const EvLineDev* l2, uint32_t s, uint32_t idx, uint32_t njobs) {
  sq_pub(x, SX_A, f);
  x.sync();
  W29 w;
  w29_init(w);
#pragma nounroll
  for (int t = 0; t < 3; t++) {
    int j = x.k - (t == 0 ? 0 : (t == 1 ? 1 : 3));
    int sb = j < 0 ? SX_AX + j + 6 : SX_A + j;
    w29_mac(w, evline_ld29(l2, s, t, idx, njobs), x.get(sb));
  }
  x.sync();
  return w29_reduce(w);
}

// f * (fixed-Q line at P1) (as sx_fixed_line): lanes 0..3 form r0.c0 yP,
// r0.c1 yP, r1.c0 xP, r1.c1 xP and exchange them through SX_P
template <class X>
FTS_HD q2 sq_fixed_line(const X& x, const q2& f, const LineCoef29& q, const f29& yP, const f29& xP, bool inf) {
  const int k = x.k;
  f29 a = (k == 0) ? q.r0.c0 : (k == 1) ? q.r0.c1 : (k == 2) ? q.r1.c0 : q.r1.c1;
  f29 m = k < 2 ? yP : xP;
  pin29(m);
  f29 prod = f29_mulb(a, m);
  x.put(SX_P + k, {prod, prod});
  x.sync();
  q2 l0 = {x.get(SX_P + 0).c0, x.get(SX_P + 1).c0};
  q2 l1 = {x.get(SX_P + 2).c0, x.get(SX_P + 3).c0};
  q2 one = {f29_breduce(f29_from_fp(fe_one<ModP>())), q2_zero().c1};
  l0 = q2_sel(inf, one, l0);
  l1 = q2_sel(inf, q2_zero(), l1);
  q2 l3 = q2_sel(inf, q2_zero(), q.r2);
  return sq_mul_line_r(x, f, l0, l1, l3);
}

// Fixed-Q line divided by r0 yP (an Fp2 factor, which the final exponentiation
// sends to 1): 1 + (r1/r0)(xP/yP) w + (r2/r0)(1/yP) w^3.  q holds r1/r0 and
// r2/r0 in its r1, r2 slots (k_qlines, once per context), xq = xP/yP and
// yi = 1/yP come from the G1 combine (g1_pnorm).  Lanes 0..3 form the four
// Fp products; f + f (l1 w + l3 w^3) then costs two limb-product pairs per
// lane instead of sq_fixed_line's three.
template <class X>
FTS_HD q2 sq_fixed_line_n(const X& x, const q2& f, const LineCoef29& q, const f29& xq, const f29& yi, bool inf) {
  const int k = x.k;
  f29 a = (k == 0) ? q.r1.c0 : (k == 1) ? q.r1.c1 : (k == 2) ? q.r2.c0 : q.r2.c1;
  f29 m = k < 2 ? xq : yi;
  pin29(m);
  f29 prod = f29_mulb(a, m);
  x.put(SX_P + k, {prod, prod});
  x.sync();
  q2 l1 = {x.get(SX_P + 0).c0, x.get(SX_P + 1).c0};
  q2 l3 = {x.get(SX_P + 2).c0, x.get(SX_P + 3).c0};
  sq_pub(x, SX_A, f);
  x.sync();
  W29 w;
  w29_init(w);
#pragma nounroll
  for (int t = 0; t < 2; t++) {
    int j = k - (t == 0 ? 1 : 3);
    int sb = j < 0 ? SX_AX + j + 6 : SX_A + j;
    w29_mac(w, t == 0 ? l1 : l3, x.get(sb));
  }
  x.sync();
  q2 r = w29_reduce(w);
  q2 g = {f29_lin2(f.c0, 1, r.c0, 1), f29_lin2(f.c1, 1, r.c1, 1)};
  return q2_sel(inf, f, g);
}

// sq_fixed_line_n with the lane's multiplicand v already selected (lanes 0, 1:
// xP/yP, lanes 2, 3: 1/yP; lanes 4, 5: anything)
template <class X>
FTS_HD q2 sq_fixed_line_nv(const X& x, const q2& f, const LineCoef29& q, const f29& v, bool inf) {
  const int k = x.k;
  f29 a = (k == 0) ? q.r1.c0 : (k == 1) ? q.r1.c1 : (k == 2) ? q.r2.c0 : q.r2.c1;
  f29 m = v;
  pin29(m);
  f29 prod = f29_mulb(a, m);
  x.put(SX_P + k, {prod, prod});
  x.sync();
  q2 l1 = {x.get(SX_P + 0).c0, x.get(SX_P + 1).c0};
  q2 l3 = {x.get(SX_P + 2).c0, x.get(SX_P + 3).c0};
  sq_pub(x, SX_A, f);
  x.sync();
  W29 w;
  w29_init(w);
#pragma nounroll
  for (int t = 0; t < 2; t++) {
    int j = k - (t == 0 ? 1 : 3);
    int sb = j < 0 ? SX_AX + j + 6 : SX_A + j;
    w29_mac(w, t == 0 ? l1 : l3, x.get(sb));
  }
  x.sync();
  q2 r = w29_reduce(w);
  q2 g = {f29_lin2(f.c0, 1, r.c0, 1), f29_lin2(f.c1, 1, r.c1, 1)};
  return q2_sel(inf, f, g);
}

// the lane's multiplicand of a normalised fixed line at P (pn = (xP/yP, 1/yP))
FTS_HD f29 sq_line_mult(int k, const G1Dev& pn) {
  fp v;
#pragma unroll
  for (int i = 0; i < 8; i++) v.v[i] = k < 2 ? pn.x[i] : pn.y[i];
  return f29_breduce(f29_from_fp(v));
}

// The prover's fixed-pair Miller product f(C, Q) f(A, PK1) f(B, PK2): all three
// G2 arguments fixed, their lines precomputed and normalised by r0 (each pair's
// Fp2 factor is sent to 1 by the final exponentiation); the squarings are shared
template <class X>
FTS_HD q2 sq_miller_f3n(const X& x, const LineCoef29* l0, const LineCoef29* l1, const LineCoef29* l2,
                        const G1Dev& pn0, const G1Dev& pn1, const G1Dev& pn2, bool inf0, bool inf1, bool inf2) {
  const f29 v0 = sq_line_mult(x.k, pn0), v1 = sq_line_mult(x.k, pn1), v2 = sq_line_mult(x.k, pn2);
  q2 one = {f29_breduce(f29_from_fp(fe_one<ModP>())), q2_zero().c1};
  q2 f = q2_sel(x.k == 0, one, q2_zero());
#pragma nounroll
  for (int s = 0; s < MILLER_LINES; s++) {
    bool sq = s < 64 ? ((MILLER_SQR.lo >> s) & 1) : ((MILLER_SQR.hi >> (s - 64)) & 1);
    if (sq) f = sq_sqr(x, f);
    // one copy of the line step in the loop (three inlined copies spilled)
#pragma nounroll
    for (int t = 0; t < 3; t++) {
      const LineCoef29* L = t == 0 ? l0 : (t == 1 ? l1 : l2);
      f29 v;
#pragma unroll
      for (int i = 0; i < 9; i++) v.l[i] = t == 0 ? v0.l[i] : (t == 1 ? v1.l[i] : v2.l[i]);
      f = sq_fixed_line_nv(x, f, L[s], v, t == 0 ? inf0 : (t == 1 ? inf1 : inf2));
    }
  }
  return f;
}

// 2-pair Miller loop with the normalised fixed-Q lines (same GT value after
// the final exponentiation as sq_miller_f; the Miller value differs by a
// factor in Fp2*)
template <class X>
FTS_HD q2 sq_miller_fn(const X& x, const LineCoef29* qlines_n, const g1a& P1, const G1Dev& pn, const EvLineDev* l2,
                       uint32_t idx, uint32_t njobs) {
  fp xqf, yif;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    xqf.v[i] = pn.x[i];
    yif.v[i] = pn.y[i];
  }
  const f29 xq = f29_breduce(f29_from_fp(xqf)), yi = f29_breduce(f29_from_fp(yif));
  q2 one = {f29_breduce(f29_from_fp(fe_one<ModP>())), q2_zero().c1};
  q2 f = q2_sel(x.k == 0, one, q2_zero());
#pragma nounroll
  for (int s = 0; s < MILLER_LINES; s++) {
    bool sq = s < 64 ? ((MILLER_SQR.lo >> s) & 1) : ((MILLER_SQR.hi >> (s - 64)) & 1);
    if (sq) f = sq_sqr(x, f);
    f = sq_fixed_line_n(x, f, qlines_n[s], xq, yi, P1.inf);
#if FTS_MILLER_EVLINE_IN_LOOP
    f = sq_mul_evline(x, f, l2, s, idx, njobs);
#else
    f = sq_mul_line_r(x, f, evline_ld29(l2, s, 0, idx, njobs), evline_ld29(l2, s, 1, idx, njobs),
                      evline_ld29(l2, s, 2, idx, njobs));
#endif
  }
  return f;
}

// 2-pair Miller loop, pair-2 lines precomputed (as sx_miller_f)
template <class X>
FTS_HD q2 sq_miller_f(const X& x, const LineCoef29* qlines, const g1a& P1, const EvLineDev* l2, uint32_t idx,
                      uint32_t njobs) {
  const f29 yP = f29_breduce(f29_from_fp(P1.y)), xP = f29_breduce(f29_from_fp(P1.x));
  q2 one = {f29_breduce(f29_from_fp(fe_one<ModP>())), q2_zero().c1};
  q2 f = q2_sel(x.k == 0, one, q2_zero());
#pragma nounroll
  for (int s = 0; s < MILLER_LINES; s++) {
    bool sq = s < 64 ? ((MILLER_SQR.lo >> s) & 1) : ((MILLER_SQR.hi >> (s - 64)) & 1);
    if (sq) f = sq_sqr(x, f);
    f = sq_fixed_line(x, f, qlines[s], yP, xP, P1.inf);
#if FTS_MILLER_EVLINE_IN_LOOP
    f = sq_mul_evline(x, f, l2, s, idx, njobs);
#else
    f = sq_mul_line_r(x, f, evline_ld29(l2, s, 0, idx, njobs), evline_ld29(l2, s, 1, idx, njobs),
                      evline_ld29(l2, s, 2, idx, njobs));
#endif
  }
  return f;
}

// LDS dwords per sextet region: NS slots of 18 dwords, padded.  The operand
// exchange is compiled to ds_read2_b64 / ds_read2_b32 / ds_write2_b64 /
// ds_write2_b32, all of which bank on (a/4) mod 32 (MI355X_MICROARCH.md, LDS
// table).  FTS_SQ_PAD (default 12): the region stride is = 12 mod 32 dwords.
// A model of the exchange's access patterns (broadcast gets, per-lane slot
// gets, per-lane puts; 16-lane groups for b64, 32-lane for b32; lane = 6
// sextet + k; the x-power's cyclotomic squarings and products, the Miller
// step's squaring, normalised fixed line and pair-2 line) puts the x-power at
// 2.6x and the Miller step at 1.4x fewer conflict cycles than the previous
// rule, the best of every stride mod 32 and of slot strides 18..30 (measured,
// 20 mod 32: k_fexp_expt 9.97 -> 3.34 conflict cycles per LDS instruction,
// 746 -> 728 us; profiles/r06/lds_pad.txt).  FTS_SQ_PAD = 0: the previous
// rule, distinct even banks mod 64 (stride = 2 x odd mod 64), which only the
// b64 reads' banking (mod 64) would favour.
#ifndef FTS_SQ_PAD
#define FTS_SQ_PAD 12
#endif
constexpr uint32_t sq_region_dwords(uint32_t ns) {
  uint32_t s = ns * 18;
  if (FTS_SQ_PAD)
    while (s % 32 != FTS_SQ_PAD) s += 2;
  else
    while ((s % 64) % 4 != 2) s += 2;
  return s;
}

}  // namespace fts

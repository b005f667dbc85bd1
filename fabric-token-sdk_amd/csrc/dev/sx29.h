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

struct q2 {
  f29 c0, c1;
};

static constexpr int32_t F29_HALF = 1 << 28;

// balanced low digit of a 64-bit accumulator: lo = acc mod 2^29 in [-2^28, 2^28)
FTS_HD int32_t f29_bdigit(int64_t acc) {
  return (int32_t)(((uint32_t)acc + (uint32_t)F29_HALF) & (uint32_t)F29_MASK) - F29_HALF;
}

// ca a + cb b - q p, balanced (|result| <= p/2 + e).  |ca|, |cb| <= 16 and
// inputs with |limb| <= 2^29: every term fits the 64-bit sweep.
FTS_HD f29 f29_lin2(const f29& a, int32_t ca, const f29& b, int32_t cb) {
  double t = (double)ca * ((double)a.l[8] * 536870912.0 + (double)a.l[7]) +
             (double)cb * ((double)b.l[8] * 536870912.0 + (double)b.l[7]);
  const int32_t q = (int32_t)__builtin_rint(t * P29_TOP_INV);
  f29 r;
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    acc += (int64_t)ca * a.l[i] + (int64_t)cb * b.l[i] - (int64_t)q * P29B[i];
    if (i < 8) {
      const int32_t lo = f29_bdigit(acc);
      r.l[i] = lo;
      acc = (acc - lo) >> 29;
    } else {
      r.l[8] = (int32_t)acc;
    }
  }
  return r;
}

FTS_HD q2 q2_neg(const q2& a) { return {f29_neg(a.c0), f29_neg(a.c1)}; }
FTS_HD q2 q2_conj(const q2& a) { return {a.c0, f29_neg(a.c1)}; }
FTS_HD q2 q2_zero() {
  q2 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.c0.l[i] = r.c1.l[i] = 0;
  return r;
}
FTS_HD q2 q2_sel(bool c, const q2& a, const q2& b) {
  q2 r;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    r.c0.l[i] = c ? a.c0.l[i] : b.c0.l[i];
    r.c1.l[i] = c ? a.c1.l[i] : b.c1.l[i];
  }
  return r;
}
// xi a = (9 a0 - a1) + (a0 + 9 a1) u, reduced
FTS_HD q2 q2_mul_xi(const q2& a) { return {f29_lin2(a.c0, 9, a.c1, -1), f29_lin2(a.c0, 1, a.c1, 9)}; }

FTS_HD f29 f29_breduce(const f29& a) { return f29_lin2(a, 1, a, 0); }

// canonical 32-bit Montgomery Fp2 <-> balanced form
FTS_HD q2 q2_from_fp2(const fp2& a) { return {f29_breduce(f29_from_fp(a.c0)), f29_breduce(f29_from_fp(a.c1))}; }
FTS_HD fp2 q2_to_fp2(const q2& a) { return {f29_to_fp(a.c0), f29_to_fp(a.c1)}; }

// ----------------------------------------------------------- accumulation
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
    acc = (acc - lo) >> 29;
  }
  r.l[8] = (int32_t)acc;
  return r;
}
FTS_HD q2 w29_reduce(W29& w) { return {w29_redc(w.re), w29_redc(w.im)}; }

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

template <class Sync>
struct Sq {
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
  x.put(base + 6 + x.k, q2_mul_xi(v));
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
    int sb = j < 0 ? SX_BX + j + 6 : SX_B + j;
    w29_mac(w, x.get(SX_A + i), x.get(sb));
  }
  x.sync();
  return w29_reduce(w);
}
template <class X>
FTS_HD q2 sq_mulv(const X& x, const q2& a, const q2& b) {
  sq_pub(x, SX_B, b);
  return sq_mul(x, a);
}

// Granger-Scott cyclotomic squaring (as sx_cyc_sqr): even lanes 3 r - 2 a,
// odd lanes 6 r + 2 a, r the lane's one or two products
template <class X>
FTS_HD q2 sq_cyc_sqr(X x, q2 a) {
  const int k = x.k, m = k >> 1;
  sq_pub(x, SX_A, a);
  x.sync();
  bool odd = (k & 1) != 0;
  int i1 = odd ? (k == 1 ? 5 : (k == 3 ? 3 : 4)) : m;
  int j1 = odd ? (k == 1 ? SX_AX + 2 : (k == 3 ? SX_A + 0 : SX_A + 1)) : SX_A + m;
  W29 w;
  w29_init(w);
#pragma nounroll
  for (int t = 0; t < 2; t++) {
    q2 u = x.get(t == 0 ? SX_A + i1 : SX_A + m + 3);
    q2 v = x.get(t == 0 ? j1 : SX_AX + m + 3);
    w29_mac(w, q2_sel(odd && t == 1, q2_zero(), u), v);
  }
  x.sync();
  q2 r = w29_reduce(w);
  const int32_t cr = odd ? 6 : 3, ca = odd ? 2 : -2;
  return {f29_lin2(r.c0, cr, a.c0, ca), f29_lin2(r.c1, cr, a.c1, ca)};
}

FTS_HD q2 sq_conj(int k, const q2& a) { return (k & 1) ? q2_neg(a) : a; }
FTS_HD q2 sq_frob1(int k, const q2& a) { return q2_mul(q2_conj(a), q2_from_fp2(f2_const(FROB1[k]))); }
FTS_HD q2 sq_frob2(int k, const q2& a) { return q2_mul(a, q2_from_fp2(f2_of_fp(fe_const<ModP>(FROB2[k][0])))); }
FTS_HD q2 sq_frob3(int k, const q2& a) { return q2_mul(q2_conj(a), q2_from_fp2(f2_const(FROB3[k]))); }

// a^x, as sx_expt (width-4 NAF, a^7 parked in the lane's SX_P slot)
template <class X>
FTS_HD q2 sq_expt(X x, q2 a) {
  q2 a2 = sq_cyc_sqr(x, a);
  q2 a3 = sq_mulv(x, a2, a);
  q2 a5 = sq_mulv(x, a3, a2);
  x.put(SX_P + x.k, sq_mul(x, a5));
  int cur = 0;
  q2 r = a;
#pragma nounroll
  for (int i = 61; i >= 0; i--) {
    r = sq_cyc_sqr(x, r);
    if ((BN_X_W4_NZ >> i) & 1) {
      int m = ((BN_X_W4_M3 >> i) & 1) ? 3 : (((BN_X_W4_M5 >> i) & 1) ? 5 : (((BN_X_W4_M7 >> i) & 1) ? 7 : 1));
      if (m != cur) {
        sq_pub(x, SX_B, m == 7 ? x.get(SX_P + x.k) : (m == 1 ? a : (m == 3 ? a3 : a5)));
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

// The two final exponentiations (same sequences as sx_final_exp_exact /
// sx_final_exp).  xo is the 32-bit context on the same LDS region, used for the
// inversion only; every slot it writes is dead once sx_inv returns.
template <class X, class XO>
FTS_HD fp2 sq_final_exp_exact(const X& x, const XO& xo, const fp2& f) {
  const int k = x.k;
  fp2 fi = sx_inv(xo, f);
  xo.sync();
  q2 F = q2_from_fp2(f);
  q2 m = sq_mulv(x, sq_conj(k, F), q2_from_fp2(fi));
  m = sq_mulv(x, sq_frob2(k, m), m);
  q2 in = m, mx, mx2, mx3;
#pragma nounroll
  for (int e = 0; e < 3; e++) {
    q2 r = sq_expt(x, in);
    if (e == 0) {
      mx = r;
    } else if (e == 1) {
      mx2 = r;
    } else {
      mx3 = r;
    }
    in = r;
  }
  q2 y3 = sq_conj(k, sq_frob1(k, mx));
  q2 y4 = sq_conj(k, sq_mulv(x, mx, sq_frob1(k, mx2)));
  q2 y5 = sq_conj(k, mx2);
  q2 y2 = sq_frob2(k, mx2);
  q2 y6 = sq_conj(k, sq_mulv(x, mx3, sq_frob1(k, mx3)));
  q2 t0 = sq_mulv(x, sq_mulv(x, sq_cyc_sqr(x, y6), y4), y5);
  q2 t1 = sq_mulv(x, sq_mulv(x, y3, y5), t0);
  t0 = sq_mulv(x, t0, y2);
  t1 = sq_cyc_sqr(x, sq_mulv(x, sq_cyc_sqr(x, t1), t0));
  q2 y0 = sq_mulv(x, sq_mulv(x, sq_frob1(k, m), sq_frob2(k, m)), sq_frob3(k, m));
  t0 = sq_mulv(x, t1, sq_conj(k, m));
  t1 = sq_mulv(x, t1, y0);
  return q2_to_fp2(sq_mulv(x, sq_cyc_sqr(x, t0), t1));
}

template <class X, class XO>
FTS_HD fp2 sq_final_exp(const X& x, const XO& xo, const fp2& f) {
  const int k = x.k;
  fp2 fi = sx_inv(xo, f);
  xo.sync();
  q2 t = sq_mulv(x, sq_conj(k, q2_from_fp2(f)), q2_from_fp2(fi));
  t = sq_mulv(x, sq_frob2(k, t), t);
  q2 in = t, a2, a6, b, c;
#pragma nounroll
  for (int e = 0; e < 3; e++) {
    q2 r = sq_expt(x, in);
    if (e == 0) {
      a2 = sq_cyc_sqr(x, r);
      a6 = sq_mulv(x, sq_cyc_sqr(x, a2), a2);
      in = a6;
    } else if (e == 1) {
      b = r;
      in = sq_cyc_sqr(x, b);
    } else {
      c = r;
    }
  }
  q2 A = sq_mulv(x, sq_mulv(x, a6, b), c);
  q2 B = sq_mulv(x, A, sq_conj(k, a2));
  q2 res = sq_frob2(k, A);
  res = sq_mulv(x, res, sq_mulv(x, sq_mulv(x, A, b), t));
  res = sq_mulv(x, res, sq_frob1(k, B));
  res = sq_mulv(x, res, sq_frob3(k, sq_mulv(x, B, sq_conj(k, t))));
  return q2_to_fp2(res);
}

// LDS bytes per sextet for the final exponentiation: the q2 slots, which also
// hold the 32-bit slots of the inversion (aliased, used one after the other)
static constexpr uint32_t SQ_FEXP_BYTES =
    SX_SLOTS_FEXP * sizeof(Q2Slot) > SX_SLOTS_FEXP * sizeof(F2Slot) ? SX_SLOTS_FEXP * sizeof(Q2Slot)
                                                                   : SX_SLOTS_FEXP * sizeof(F2Slot);

}  // namespace fts

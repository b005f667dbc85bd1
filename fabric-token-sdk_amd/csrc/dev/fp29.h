// Carry-free BN254 base-field arithmetic for the one-lane G1 loops (variable-
// and fixed-base scalar multiplication, MSM buckets): signed 9 x 29-bit limbs
// with 64-bit column accumulators.
//
// The 8 x 32-bit Montgomery product of fp.h issues one carry add per MAD
// (v_mad_u64_u32 + v_addc, ~300 instructions with the column moves); here a
// limb product is < 2^60 and a column of nine of them plus the reduction terms
// stays below 2^63, so every MAD accumulates straight into a signed 64-bit
// column (v_mad_i64_i32, no carries): 162 MADs + ~45 column instructions per
// product, 126 MADs per squaring.  Additions and subtractions are nine limb
// adds with no carry chain and no reduction; the cost moves to explicit
// normalisations (a carry sweep, f29_norm) and value reductions (one quotient
// estimate + a multiple of p, f29_reduce) placed where the bounds require them.
//
// Representation: value = sum l[i] 2^(29 i) with signed limbs, Montgomery radix
// R = 2^261 (> 169 p).  Bounds the formulas below keep (L = max |limb| in units
// of 2^29 - 1, B = |value| in units of p):
//   f29_mul / f29_sqr inputs: L_a L_b <= 2.5 (column |sum| < 9 (L_a L_b + 1) 2^58
//     < 2^63; f29_sqr needs L <= 1) and B_a B_b < 169 (then |out| < 2p);
//     output normalised: limbs 0..7 in [0, 2^29), limb 8 small and signed;
//   f29_add / f29_sub: L and B add (L <= 4 keeps every limb inside int32);
//   f29_norm: L -> 1, value unchanged;  f29_reduce: L -> 1, |value| <= p/2 + p.
// Values enter from the 32-bit Montgomery form (R = 2^256) by a shifted limb
// split (value x 32, B <= 32) and leave through one product by 2^256 mod p, a
// reduction and a final canonical subtraction (f29_to_fp), so the G1 code around
// the loops keeps its fp types.  tests/native/emu_exec.cpp checks every
// formula against the fp.h ones.
#pragma once
#include "curve.h"
#include "fp.h"
#include "fp29_const.h"

namespace fts {

struct f29 {
  int32_t l[9];
};

// A 32-bit value the compiler must treat as produced here: a lane-dependent
// multiplicand whose sign extension LLVM would otherwise hoist out of a loop
// (or keep from another block) is then multiplied as a full int64 x int64
// (v_mad_u64_u32 + 2 v_mul_lo_u32 + v_add3, 4 instructions) instead of one
// v_mad_i64_i32.
FTS_HD int32_t pin32(int32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(x));
#endif
  return x;
}
static constexpr int32_t F29_MASK = (1 << 29) - 1;

FTS_HD void pin29(f29& a) {
#pragma unroll
  for (int i = 0; i < 9; i++) a.l[i] = pin32(a.l[i]);
}

FTS_HD f29 f29_add(const f29& a, const f29& b) {
  f29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = a.l[i] + b.l[i];
  return r;
}
FTS_HD f29 f29_sub(const f29& a, const f29& b) {
  f29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = a.l[i] - b.l[i];
  return r;
}
FTS_HD f29 f29_neg(const f29& a) {
  f29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = -a.l[i];
  return r;
}

// carry sweep: limbs 0..7 into [0, 2^29), limb 8 takes the (signed) rest
FTS_HD f29 f29_norm(const f29& a) {
  f29 r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    int32_t t = a.l[i] + c;
    r.l[i] = t & F29_MASK;
    c = t >> 29;
  }
  r.l[8] = a.l[8] + c;
  return r;
}

// Montgomery product a b / 2^261 (product scanning; column k accumulates the
// a_i b_j and m_i p_j with i + j = k, m_k makes its low 29 bits vanish)
FTS_HD f29 f29_mul(const f29& a, const f29& b) {
  FTS_COUNT_MUL();
  int64_t acc = 0;
  uint32_t m[9];
  f29 r;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j >= 0 && j < 9) acc += (int64_t)a.l[i] * b.l[j];
    }
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (i < k && j >= 0 && j < 9) acc += (int64_t)(int32_t)m[i] * P29[j];
    }
    if (k < 9) {
      m[k] = ((uint32_t)acc * P29_INV) & (uint32_t)F29_MASK;
      acc += (int64_t)(int32_t)m[k] * P29[0];
    } else {
      r.l[k - 9] = (int32_t)(acc & F29_MASK);
    }
    acc >>= 29;
  }
  r.l[8] = (int32_t)acc;
  return r;
}

// f29_mul's value and limbs (the same Montgomery digits m_k) with the 81 limb
// products in 17 independent column sums and the reduction in 9 steps of nine
// independent MADs: a dependent chain of ~30 operations instead of ~160, for
// latency-bound single-wave code (the MSM's Horner chain)
FTS_HD f29 f29_mul_c(const f29& a, const f29& b) {
  FTS_COUNT_MUL();
  int64_t c[17];
#pragma unroll
  for (int k = 0; k < 17; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++)
#pragma unroll
    for (int j = 0; j < 9; j++) c[i + j] += (int64_t)a.l[i] * b.l[j];
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const uint32_t m = ((uint32_t)c[k] * P29_INV) & (uint32_t)F29_MASK;
    const int64_t t = c[k] + (int64_t)(int32_t)m * P29[0];  // low 29 bits now zero
#pragma unroll
    for (int j = 1; j < 9; j++) c[k + j] += (int64_t)(int32_t)m * P29[j];
    c[k + 1] += t >> 29;
  }
  f29 r;
#pragma unroll
  for (int k = 9; k < 16; k++) {
    r.l[k - 9] = (int32_t)(c[k] & F29_MASK);
    c[k + 1] += c[k] >> 29;
  }
  r.l[7] = (int32_t)(c[16] & F29_MASK);
  r.l[8] = (int32_t)(c[16] >> 29);
  return r;
}

// f29_sqr's value by f29_mul_c's scheme: column sums with the cross products
// once (doubled operand, L <= 1), then the same 9 reduction steps
FTS_HD f29 f29_sqr_c(const f29& a) {
  FTS_COUNT_MUL();
  int32_t d[9];
#pragma unroll
  for (int i = 0; i < 9; i++) d[i] = a.l[i] + a.l[i];
  int64_t c[17];
#pragma unroll
  for (int k = 0; k < 17; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    c[2 * i] += (int64_t)a.l[i] * a.l[i];
#pragma unroll
    for (int j = i + 1; j < 9; j++) c[i + j] += (int64_t)d[i] * a.l[j];
  }
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const uint32_t m = ((uint32_t)c[k] * P29_INV) & (uint32_t)F29_MASK;
    const int64_t t = c[k] + (int64_t)(int32_t)m * P29[0];
#pragma unroll
    for (int j = 1; j < 9; j++) c[k + j] += (int64_t)(int32_t)m * P29[j];
    c[k + 1] += t >> 29;
  }
  f29 r;
#pragma unroll
  for (int k = 9; k < 16; k++) {
    r.l[k - 9] = (int32_t)(c[k] & F29_MASK);
    c[k + 1] += c[k] >> 29;
  }
  r.l[7] = (int32_t)(c[16] & F29_MASK);
  r.l[8] = (int32_t)(c[16] >> 29);
  return r;
}

// a^2 / 2^261: the cross products once with a doubled operand (requires L <= 1)
FTS_HD f29 f29_sqr(const f29& a) {
  FTS_COUNT_MUL();
  int32_t d[9];
#pragma unroll
  for (int i = 0; i < 9; i++) d[i] = a.l[i] + a.l[i];
  int64_t acc = 0;
  uint32_t m[9];
  f29 r;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j > i && j < 9) acc += (int64_t)d[i] * a.l[j];
    }
    if ((k & 1) == 0 && k / 2 < 9) acc += (int64_t)a.l[k / 2] * a.l[k / 2];
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (i < k && j >= 0 && j < 9) acc += (int64_t)(int32_t)m[i] * P29[j];
    }
    if (k < 9) {
      m[k] = ((uint32_t)acc * P29_INV) & (uint32_t)F29_MASK;
      acc += (int64_t)(int32_t)m[k] * P29[0];
    } else {
      r.l[k - 9] = (int32_t)(acc & F29_MASK);
    }
    acc >>= 29;
  }
  r.l[8] = (int32_t)acc;
  return r;
}

// value - q p with q = round(value / p) from the top two limbs (a double
// estimate: exact when value is a multiple of p), normalised in the same carry
// sweep; |result| <= p/2 + 2^-40 p
FTS_HD f29 f29_reduce(const f29& a) {
  // the estimate needs no normalised input: the limbs below 7 move the value by
  // at most L 2^203, i.e. q by L / 2^50.6
  const f29& n = a;
  double t = (double)n.l[8] * 536870912.0 + (double)n.l[7];
  int32_t q = (int32_t)__builtin_rint(t * P29_TOP_INV);  // |error| < 2^-45: exact for multiples of p
  f29 r;
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    acc += (int64_t)n.l[i] - (int64_t)q * P29[i];
    if (i < 8) {
      r.l[i] = (int32_t)(acc & F29_MASK);
      acc >>= 29;
    } else {
      r.l[8] = (int32_t)acc;
    }
  }
  return r;
}

FTS_HD f29 fe29_p() {
  f29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = P29[i];
  return r;
}

// a == 0 mod p (any bounded input)
FTS_HD bool f29_is_zero(const f29& a) {
  f29 r = f29_reduce(a);
  int32_t o = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) o |= r.l[i];
  return o == 0;
}
// a reduced value (f29_reduce output) that is zero
FTS_HD bool f29_reduced_zero(const f29& r) {
  int32_t o = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) o |= r.l[i];
  return o == 0;
}

// 32-bit Montgomery (R = 2^256, any representative < 2^256) -> this form:
// the limbs of 32 x, i.e. the R = 2^261 Montgomery form of the same element
// (B <= 32 for x < p, L = 1)
FTS_HD f29 f29_from_fp(const fp& x) {
  f29 r;
  r.l[0] = (int32_t)((x.v[0] << 5) & (uint32_t)F29_MASK);
#pragma unroll
  for (int i = 1; i < 9; i++) {
    const int off = 29 * i - 5, w = off >> 5, s = off & 31;
    uint64_t lo = x.v[w], hi = w + 1 < 8 ? x.v[w + 1] : 0u;
    r.l[i] = (int32_t)((uint32_t)(((hi << 32) | lo) >> s) & (uint32_t)F29_MASK);
  }
  return r;
}

// back to the canonical 32-bit Montgomery form (value < p)
FTS_HD fp f29_to_fp(const f29& a) {
  f29 p29;
#pragma unroll
  for (int i = 0; i < 9; i++) p29.l[i] = P29_R256[i];
  f29 r = f29_reduce(f29_mul(a, p29));  // a 2^256 / 2^261: the R = 2^256 form, |r| <= 3p/2
  // into [0, p): add p while negative, subtract p while >= p (normalised limbs
  // compare lexicographically from the top)
#pragma unroll
  for (int it = 0; it < 2; it++) {
    f29 s = f29_norm(f29_add(r, fe29_p()));
    const bool take = r.l[8] < 0;
#pragma unroll
    for (int i = 0; i < 9; i++) r.l[i] = take ? s.l[i] : r.l[i];
  }
#pragma unroll
  for (int it = 0; it < 2; it++) {
    f29 s = f29_norm(f29_sub(r, fe29_p()));
    const bool take = s.l[8] >= 0;
#pragma unroll
    for (int i = 0; i < 9; i++) r.l[i] = take ? s.l[i] : r.l[i];
  }
  fp o;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int b = 32 * j, i = b / 29, s = b % 29;
    uint64_t v = (uint64_t)(uint32_t)r.l[i] | ((uint64_t)(uint32_t)(i + 1 < 9 ? r.l[i + 1] : 0) << 29);
    if (i + 2 < 9) v |= (uint64_t)(uint32_t)r.l[i + 2] << 58;
    o.v[j] = (uint32_t)(v >> s);
  }
  return o;
}

// ------------------------------------------------- balanced form, Fp2 (q2)
// The pairing side (dev/sx29.h) keeps values BALANCED: limbs 0..7 in
// [-2^28, 2^28), |value| <= p/2 + e, so that a 64-bit column can absorb 117
// limb products of at most 2^56 each.
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
FTS_HD f29 f29_lin2(const f29& a_, int32_t ca, const f29& b_, int32_t cb) {
  if (!__builtin_constant_p(ca)) ca = pin32(ca);
  if (!__builtin_constant_p(cb)) cb = pin32(cb);
  f29 a = a_, b = b_;  // limbs as 32-bit values here (not sign-extended copies from elsewhere)
  pin29(a);
  pin29(b);
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
      acc = (acc + F29_HALF) >> 29;  // = (acc - lo) / 2^29: lo is acc's balanced low digit
    } else {
      r.l[8] = (int32_t)acc;
    }
  }
  return r;
}

// ca a + cb b without the quotient: one balanced carry sweep (limbs 0..7 in
// [-2^28, 2^28), limb 8 the signed rest), the value unchanged -- for operands
// that are only ever multiplied (|value| <= (|ca| + |cb|)(p/2 + e) stays far
// inside the product's value budget, and the limbs inside its column budget)
FTS_HD f29 f29_lin2_ns(const f29& a_, int32_t ca, const f29& b_, int32_t cb) {
  f29 a = a_, b = b_;
  pin29(a);
  pin29(b);
  f29 r;
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    acc += (int64_t)ca * a.l[i] + (int64_t)cb * b.l[i];
    if (i < 8) {
      r.l[i] = f29_bdigit(acc);
      acc = (acc + F29_HALF) >> 29;
    } else {
      r.l[8] = (int32_t)acc;
    }
  }
  return r;
}

// c0 x0 + c1 x1 + c2 x2 + c3 x3 - q p, balanced (|result| <= p/2 + e); |c_i|
// <= 64 and balanced inputs (|limb| <= 2^29)
FTS_HD f29 f29_lin4(const f29& x0_, int32_t c0, const f29& x1_, int32_t c1, const f29& x2_, int32_t c2,
                    const f29& x3_, int32_t c3) {
  f29 x0 = x0_, x1 = x1_, x2 = x2_, x3 = x3_;
  pin29(x0);
  pin29(x1);
  pin29(x2);
  pin29(x3);
  c0 = pin32(c0);
  c1 = pin32(c1);
  c2 = pin32(c2);
  c3 = pin32(c3);
  double t = (double)c0 * ((double)x0.l[8] * 536870912.0 + (double)x0.l[7]) +
             (double)c1 * ((double)x1.l[8] * 536870912.0 + (double)x1.l[7]) +
             (double)c2 * ((double)x2.l[8] * 536870912.0 + (double)x2.l[7]) +
             (double)c3 * ((double)x3.l[8] * 536870912.0 + (double)x3.l[7]);
  const int32_t q = (int32_t)__builtin_rint(t * P29_TOP_INV);
  f29 r;
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    acc += (int64_t)c0 * x0.l[i] + (int64_t)c1 * x1.l[i] + (int64_t)c2 * x2.l[i] + (int64_t)c3 * x3.l[i] -
           (int64_t)q * P29B[i];
    if (i < 8) {
      r.l[i] = f29_bdigit(acc);
      acc = (acc + F29_HALF) >> 29;
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
// the same value carry-swept only (|value| <= 5 p + e): a multiplicand
FTS_HD q2 q2_mul_xi_lazy(const q2& a) { return {f29_lin2_ns(a.c0, 9, a.c1, -1), f29_lin2_ns(a.c0, 1, a.c1, 9)}; }
FTS_HD q2 q2_add(const q2& a, const q2& b) { return {f29_add(a.c0, b.c0), f29_add(a.c1, b.c1)}; }

FTS_HD f29 f29_breduce(const f29& a) { return f29_lin2(a, 1, a, 0); }

// canonical 32-bit Montgomery Fp2 <-> balanced form
FTS_HD q2 q2_from_fp2(const fp2& a) { return {f29_breduce(f29_from_fp(a.c0)), f29_breduce(f29_from_fp(a.c1))}; }
FTS_HD fp2 q2_to_fp2(const q2& a) { return {f29_to_fp(a.c0), f29_to_fp(a.c1)}; }

// ---------------------------------------------------------------- G1 (a = 0)
// Jacobian point in this form with an explicit infinity flag.  Coordinates
// between operations: normalised, |value| <= 3p/2 (f29_reduce outputs or
// products).  Same formulas (and so the same projective point up to the
// representation of each coordinate) as curve.h jac_dbl / jac_add_aff.
struct j29 {
  f29 x, y, z;
  bool inf;
};

// dbl-2009-l: 2M + 5S.  Bounds in comments as (B, L).
FTS_HD j29 j29_dbl(const j29& p) {
  f29 A = f29_sqr(p.x);                            // (2, 1)
  f29 Bq = f29_sqr(p.y);                           // (2, 1)
  f29 C = f29_sqr(Bq);                             // (2, 1)
  f29 T2 = f29_sqr(f29_norm(f29_add(p.x, Bq)));    // (1.5 + 2)^2 < 169
  f29 D1 = f29_norm(f29_sub(f29_sub(T2, A), C));   // (6, 1)
  f29 D = f29_add(D1, D1);                         // (12, 2)
  f29 E = f29_norm(f29_add(f29_add(A, A), A));     // (6, 1)
  f29 F = f29_sqr(E);                              // 36: (2, 1)
  f29 X3 = f29_reduce(f29_sub(f29_norm(f29_sub(F, D)), D));        // (26, 3) -> (1.5, 1)
  f29 Y3a = f29_mul(E, f29_norm(f29_sub(D, X3)));  // 6 x 13.5 < 169: (2, 1)
  f29 C2 = f29_add(C, C);
  f29 C4 = f29_norm(f29_add(C2, C2));              // (8, 1)
  f29 Y3 = f29_reduce(f29_sub(Y3a, f29_add(C4, C4)));              // (18, 3) -> (1.5, 1)
  f29 Z3 = f29_mul(f29_add(p.y, p.y), p.z);        // 3 x 2, L 2 x 1: (2, 1); infinity keeps z = 0
  return {X3, Y3, Z3, p.inf};
}

// add-2007-bl mixed addition p + (x2, y2), (x2, y2) affine and not infinity,
// B <= 32, L <= 1 (f29_from_fp outputs): 7M + 4S.  The exceptional cases are
// caught after the fact: Z3 = 2 Z1 H vanishes iff H does, and then the sum is
// infinity (rr != 0) or a doubling (rr == 0, p == (x2, y2)).
FTS_HD j29 j29_madd(const j29& p, const f29& x2, const f29& y2) {
  if (p.inf) return {f29_reduce(x2), f29_reduce(y2), f29_reduce(f29_from_fp(fe_one<ModP>())), false};
  f29 Z1Z1 = f29_sqr(p.z);                         // (2, 1)
  f29 U2 = f29_mul(x2, Z1Z1);                      // 32 x 2: (2, 1)
  f29 S2 = f29_mul(y2, f29_mul(p.z, Z1Z1));        // (2, 1)
  f29 H = f29_norm(f29_sub(U2, p.x));              // (3.5, 1)
  f29 rr = f29_sub(S2, p.y);                       // (3.5, 2)
  f29 HH = f29_sqr(H);                             // (2, 1)
  f29 HH2 = f29_add(HH, HH);
  f29 I = f29_norm(f29_add(HH2, HH2));             // (8, 1)
  f29 J = f29_mul(H, I);                           // 28: (2, 1)
  f29 r2 = f29_norm(f29_add(rr, rr));              // (7, 1)
  f29 V = f29_mul(p.x, I);                         // 12: (2, 1)
  f29 X3 = f29_reduce(f29_sub(f29_sub(f29_sub(f29_sqr(r2), J), V), V));  // (8, 4) -> (1.5, 1)
  f29 Y3a = f29_mul(r2, f29_norm(f29_sub(V, X3))); // 7 x 3.5: (2, 1)
  f29 YJ = f29_mul(p.y, J);                        // (2, 1)
  f29 Y3 = f29_reduce(f29_sub(f29_sub(Y3a, YJ), YJ));              // (6, 3) -> (1.5, 1)
  f29 ZH = f29_norm(f29_add(p.z, H));              // (5, 1)
  f29 Z3 = f29_reduce(f29_sub(f29_sub(f29_sqr(ZH), Z1Z1), HH));    // 25: (6, 3) -> (1.5, 1)
  if (f29_reduced_zero(Z3)) {
    if (f29_is_zero(rr)) return j29_dbl(p);  // p == (x2, y2)
    j29 o = p;
    o.inf = true;
    return o;
  }
  return {X3, Y3, Z3, false};
}

// add-2007-bl full Jacobian addition p + q: 11M + 5S, inputs normalised with
// B <= 2 (products or f29_reduce outputs).  Same exceptional handling as
// j29_madd: Z3 = ((Z1 + Z2)^2 - Z1Z1 - Z2Z2) H = 2 Z1 Z2 H vanishes iff H does.
FTS_HD j29 j29_add(const j29& p, const j29& q) {
  if (p.inf) return q;
  if (q.inf) return p;
  f29 Z1Z1 = f29_sqr(p.z);                         // (2, 1)
  f29 Z2Z2 = f29_sqr(q.z);                         // (2, 1)
  f29 U1 = f29_mul(p.x, Z2Z2);                     // 2 x 2: (2, 1)
  f29 U2 = f29_mul(q.x, Z1Z1);                     // (2, 1)
  f29 S1 = f29_mul(p.y, f29_mul(q.z, Z2Z2));       // (2, 1)
  f29 S2 = f29_mul(q.y, f29_mul(p.z, Z1Z1));       // (2, 1)
  f29 H = f29_norm(f29_sub(U2, U1));               // (4, 1)
  f29 H2 = f29_norm(f29_add(H, H));                // (8, 1)
  f29 I = f29_sqr(H2);                             // 64: (2, 1)
  f29 J = f29_mul(H, I);                           // 8: (2, 1)
  f29 rr = f29_sub(S2, S1);                        // (4, 2)
  f29 r2 = f29_norm(f29_add(rr, rr));              // (8, 1)
  f29 V = f29_mul(U1, I);                          // 4: (2, 1)
  f29 X3 = f29_reduce(f29_sub(f29_sub(f29_sub(f29_sqr(r2), J), V), V));  // 64 -> (8, 4) -> (1.5, 1)
  f29 Y3a = f29_mul(r2, f29_norm(f29_sub(V, X3))); // 8 x 3.5: (2, 1)
  f29 SJ = f29_mul(S1, J);                         // (2, 1)
  f29 Y3 = f29_reduce(f29_sub(f29_sub(Y3a, SJ), SJ));              // (6, 3) -> (1.5, 1)
  f29 ZZ = f29_sqr(f29_norm(f29_add(p.z, q.z)));   // 16: (2, 1)
  f29 Z3 = f29_reduce(f29_mul(f29_norm(f29_sub(f29_sub(ZZ, Z1Z1), Z2Z2)), H));  // 6 x 4: (2, 1) -> (1.5, 1)
  if (f29_reduced_zero(Z3)) {
    if (f29_is_zero(rr)) return j29_dbl(p);  // p == q
    j29 o = p;
    o.inf = true;
    return o;
  }
  return {X3, Y3, Z3, false};
}

// ---------------------------------------------------- XYZZ bucket accumulator
// (products in the column-sum form f29_mul_c / f29_sqr_c: the same limbs as
// f29_mul / f29_sqr with 17 independent accumulators instead of one running
// sum, so the dependent chains of these long runs of additions are short)
// x = X / ZZ, y = Y / ZZZ with ZZ^3 = ZZZ^2: the mixed addition needs 8M + 2S
// (madd-2008-s) against 7M + 4S and the doublings of the Jacobian one -- the
// MSM bucket sums are long runs of mixed additions.  Coordinates between
// operations as j29's: normalised, |value| <= 2p.
struct x29 {
  f29 x, y, zz, zzz;
  bool inf;
};

// 2 (x, y) for an affine point, xyzz mdbl-2008-s-1 (the acc == P case)
FTS_HD x29 x29_dbl_aff(const f29& x0, const f29& y0) {
  f29 x = f29_reduce(x0), y = f29_reduce(y0);      // (1.5, 1)
  f29 U = f29_norm(f29_add(y, y));                 // (3, 1)
  f29 V = f29_sqr_c(U);                              // (2, 1)
  f29 W = f29_mul_c(U, V);                           // (2, 1)
  f29 S = f29_mul_c(x, V);                           // (2, 1)
  f29 xx = f29_sqr_c(x);
  f29 M = f29_norm(f29_add(f29_add(xx, xx), xx));  // (6, 1)
  f29 X3 = f29_reduce(f29_sub(f29_sub(f29_sqr_c(M), S), S));         // (40, 3) -> (1.5, 1)
  f29 Y3 = f29_reduce(f29_sub(f29_mul_c(M, f29_norm(f29_sub(S, X3))), f29_mul_c(W, y)));  // (4, 2)
  return {X3, Y3, V, W, false};
}

// p + (x2, y2), (x2, y2) affine and not infinity, B <= 32, L <= 1 (f29_from_fp
// outputs, possibly negated): madd-2008-s.  P = U2 - X1 vanishes iff the x
// coordinates agree: then the sum is a doubling (R = 0) or infinity.
FTS_HD x29 x29_madd(const x29& p, const f29& x2, const f29& y2) {
  if (p.inf) {
    f29 one = f29_reduce(f29_from_fp(fe_one<ModP>()));
    return {f29_reduce(x2), f29_reduce(y2), one, one, false};
  }
  f29 U2 = f29_mul_c(x2, p.zz);                      // 32 x 2: (2, 1)
  f29 S2 = f29_mul_c(y2, p.zzz);                     // (2, 1)
  f29 P = f29_norm(f29_sub(U2, p.x));              // (4, 1)
  f29 R = f29_norm(f29_sub(S2, p.y));              // (4, 1)
  if (f29_is_zero(P)) {
    if (f29_is_zero(R)) return x29_dbl_aff(x2, y2);
    x29 o = p;
    o.inf = true;
    return o;
  }
  f29 PP = f29_sqr_c(P);                             // 16: (2, 1)
  f29 PPP = f29_mul_c(P, PP);                        // 8: (2, 1)
  f29 Q = f29_mul_c(p.x, PP);                        // 4: (2, 1)
  f29 X3 = f29_reduce(f29_sub(f29_sub(f29_sub(f29_sqr_c(R), PPP), Q), Q));  // (8, 4) -> (1.5, 1)
  f29 Y3a = f29_mul_c(R, f29_norm(f29_sub(Q, X3)));  // 4 x 3.5: (2, 1)
  f29 Y3 = f29_reduce(f29_sub(Y3a, f29_mul_c(p.y, PPP)));            // (4, 2) -> (1.5, 1)
  return {X3, Y3, f29_mul_c(p.zz, PP), f29_mul_c(p.zzz, PPP), false};
}

// to Jacobian without an inversion: Z' = ZZ ZZZ, X' = X ZZ ZZZ^2, Y' = Y ZZZ^4
// (X'/Z'^2 = X/ZZ, and Y'/Z'^3 = Y/ZZZ because ZZ^3 = ZZZ^2)
FTS_HD j29 x29_to_j29(const x29& p) {
  if (p.inf) {
    j29 o{};
    o.inf = true;
    return o;
  }
  f29 t = f29_sqr(p.zzz);                          // ZZZ^2
  return {f29_mul(f29_mul(p.x, p.zz), t), f29_mul(p.y, f29_sqr(t)), f29_mul(p.zz, p.zzz), false};
}

FTS_HD j29 j29_from(const g1j& p) {
  return {f29_reduce(f29_from_fp(p.x)), f29_reduce(f29_from_fp(p.y)), f29_reduce(f29_from_fp(p.z)), is_zero(p.z)};
}
FTS_HD g1j j29_to(const j29& p) {
  if (p.inf) return jac_inf<fp>();
  return {f29_to_fp(p.x), f29_to_fp(p.y), f29_to_fp(p.z)};
}

}  // namespace fts

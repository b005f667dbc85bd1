// Lazily reduced ("wide") Fp2 arithmetic for the sextet pairing kernels.
//
// A sum of Fp2 products  sum_t a_t * b_t  is accumulated as two unreduced
// 512-bit integers (real, imaginary) and Montgomery-reduced once at the end:
// each Fp2 product costs 3 x 64 MADs (Karatsuba on full-width products)
// instead of 3 x 136 for three reduced Montgomery products, and the final
// reductions (2 x 72 MADs) are shared by the whole sum.
//
// Bounds (p < 2^253.6, operands reduced < p):
//   t0 = a0 b0 < p^2, t1 = a1 b1 < p^2, t2 = (a0+a1)(b0+b1) < 4p^2
//   real += t0 - t1   on an accumulator initialised to 6p^2: never negative
//                     for up to 6 terms, final value < 12 p^2 < 2^511
//   imag += t2 - t0 - t1 = a0 b1 + a1 b0 < 2p^2 per term, on an accumulator
//                     initialised to 2p^2: final value < 14 p^2
//   REDC(T < 14 p^2) < 14 p^2 / 2^256 + p < 3.7 p: two conditional subtractions
#pragma once
#include "tower.h"

namespace fts {

#include "fp_wide_gen.h"

// r[16] = a[8] * b[8]
FTS_HD void mul_wide(uint32_t r[16], const uint32_t a[8], const uint32_t b[8]) {
#if defined(__HIP_DEVICE_COMPILE__) && FTS_ONEASM
  mul_wide_oneasm(r, a, b);
#elif defined(__HIP_DEVICE_COMPILE__)
  mul_wide_asm(r, a, b);
#else
  uint64_t acc = 0;
  uint32_t hi = 0;
  for (int k = 0; k < 15; k++) {
    for (int i = 0; i < 8; i++) {
      int j = k - i;
      if (j < 0 || j > 7) continue;
      uint64_t p = (uint64_t)a[i] * b[j];
      uint64_t s = acc + p;
      hi += (uint32_t)(s < acc);
      acc = s;
    }
    r[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  r[15] = (uint32_t)acc;
#endif
}

// Montgomery reduction of t < 14 p^2:  t / 2^256 mod p, fully reduced.
FTS_HD fp redc_wide(const uint32_t t[16]) {
  FTS_COUNT_MAD(72);
  fp r;
#if defined(__HIP_DEVICE_COMPILE__) && FTS_ONEASM
  redc_wide_oneasm<ModP>(r.v, t);
#elif defined(__HIP_DEVICE_COMPILE__)
  redc_wide_asm(r.v, t);
#else
  uint64_t acc = 0;
  uint32_t hi = 0;
  uint32_t m[8];
  for (int k = 0; k < 16; k++) {
    uint64_t s = acc + t[k];
    hi += (uint32_t)(s < acc);
    acc = s;
    for (int i = 0; i < 8 && i < k; i++) {
      int j = k - i;
      if (j > 7) continue;
      uint64_t p = (uint64_t)m[i] * P_MOD[j];
      uint64_t q = acc + p;
      hi += (uint32_t)(q < acc);
      acc = q;
    }
    if (k < 8) {
      m[k] = (uint32_t)acc * P_INV;
      uint64_t p = (uint64_t)m[k] * P_MOD[0];
      uint64_t q = acc + p;
      hi += (uint32_t)(q < acc);
      acc = q;
    } else {
      r.v[k - 8] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
#endif
#if defined(__HIP_DEVICE_COMPILE__) && FTS_ASM_CHAINS
  condsub2_p_asm(r.v);
  return r;
#else
  uint32_t t2[8], pm[8], p2[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    pm[i] = P_MOD[i];
    p2[i] = P_X2[i];
  }
  if (!sub8(t2, r.v, p2)) r = fe_const<ModP>(t2);
  if (!sub8(t2, r.v, pm)) r = fe_const<ModP>(t2);
  return r;
#endif
}

FTS_HD void add16(uint32_t r[16], const uint32_t a[16]) {
#if defined(__HIP_DEVICE_COMPILE__) && FTS_ASM_CHAINS
  add16_asm(r, a);
  return;
#endif
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) r[i] = addc32(r[i], a[i], c, &c);
}

FTS_HD void sub16(uint32_t r[16], const uint32_t a[16]) {
#if defined(__HIP_DEVICE_COMPILE__) && FTS_ASM_CHAINS
  sub16_asm(r, a);
  return;
#endif
  uint32_t b = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) r[i] = subb32(r[i], a[i], b, &b);
}

// Scheduling fence (device): keeps the compiler from hoisting the next term's
// operand loads above the current term's multiply chains, which otherwise
// doubles the live registers and spills.
#if defined(__HIP_DEVICE_COMPILE__)
#define FTS_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define FTS_SCHED_FENCE() ((void)0)
#endif

// Lazily reduced Fp2 accumulator (up to 6 products of reduced operands).
struct Wide2 {
  uint32_t re[16], im[16];
};

FTS_HD void w2_init(Wide2& w) {
#pragma unroll
  for (int i = 0; i < 16; i++) {
    w.re[i] = P2X6[i];
    w.im[i] = P2X2[i];
  }
}

// w += a * b   (a, b reduced Fp2).  Ordered so that one 16-limb product is
// live at a time; the imaginary accumulator starts at 2p^2 so that it stays
// non-negative between "- t0 - t1" and "+ t2" (multiples of p vanish in REDC).
FTS_HD void w2_mac(Wide2& w, const fp2& a, const fp2& b) {
  FTS_COUNT_MAD(192);  // 3 full-width 8x8 products
  FTS_SCHED_FENCE();
  uint32_t t[16], sa[8], sb[8];
  mul_wide(t, a.c0.v, b.c0.v);
  add16(w.re, t);
  sub16(w.im, t);
  mul_wide(t, a.c1.v, b.c1.v);
  sub16(w.re, t);
  sub16(w.im, t);
  add8(sa, a.c0.v, a.c1.v);  // < 2p < 2^255: no carry out
  add8(sb, b.c0.v, b.c1.v);
  mul_wide(t, sa, sb);
  add16(w.im, t);
}

FTS_HD fp2 w2_reduce(const Wide2& w) { return {redc_wide(w.re), redc_wide(w.im)}; }

}  // namespace fts

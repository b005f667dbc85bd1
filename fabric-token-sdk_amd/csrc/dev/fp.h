// BN254 prime-field arithmetic for CDNA4 (gfx950): 8 x 32-bit limbs, Montgomery
// form (R = 2^256), CIOS multiplication written as u32 x u32 -> u64 MAD chains
// (lowered to v_mad_u64_u32 + carry adds).  One field element per lane.
//
// The same header compiles for the host (FTS_HD expands to `inline`) so the
// test-only emulation library can check every formula against the Python
// oracle on CPU; the product library only ever runs it on the GPU.
//
// Replaces the Fp/Fr arithmetic mathlib obtains from gnark-crypto v0.6.0
// (ecc/bn254/fp, fr) -- SURVEY.md Appendix C.
#pragma once
#include <stdint.h>
#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define FTS_HD __host__ __device__ __forceinline__
#define FTS_HDN __host__ __device__ __noinline__ inline
#else
#define FTS_HD inline
#define FTS_HDN inline
#endif
#include "constants.h"

// Test-only instrumentation (host emulation build): counts u32 x u32 -> u64
// MADs (a Montgomery product = 136; M = MADs / 136 in profiles/opcounts.json).
#ifdef FTS_COUNT_OPS
extern thread_local unsigned long long fts_mont_count;
#define FTS_COUNT_MAD(n) (fts_mont_count += (n))
#else
#define FTS_COUNT_MAD(n) ((void)0)
#endif
#define FTS_COUNT_MUL() FTS_COUNT_MAD(136)

namespace fts {

struct ModP {
  static constexpr const uint32_t* m = P_MOD;
  static constexpr uint32_t inv = P_INV;
  static constexpr const uint32_t* r2 = P_R2;
  static constexpr const uint32_t* one = P_ONE;
};
struct ModR {
  static constexpr const uint32_t* m = R_MOD;
  static constexpr uint32_t inv = R_INV;
  static constexpr const uint32_t* r2 = R_R2;
  static constexpr const uint32_t* one = R_ONE;
};

template <class M>
struct Fe {
  uint32_t v[8];
};
typedef Fe<ModP> fp;
typedef Fe<ModR> fr;

template <class M>
FTS_HD Fe<M> fe_zero() {
  Fe<M> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = 0;
  return r;
}

template <class M>
FTS_HD Fe<M> fe_one() {
  Fe<M> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = M::one[i];
  return r;
}

template <class M>
FTS_HD Fe<M> fe_const(const uint32_t* c) {
  Fe<M> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = c[i];
  return r;
}

// a >= m ?  (plain integer compare with the modulus)
template <class M>
FTS_HD bool fe_geq_mod(const uint32_t a[8]) {
  bool gt = false, eq = true;
#pragma unroll
  for (int i = 7; i >= 0; i--) {
    bool lt_i = a[i] < M::m[i];
    bool gt_i = a[i] > M::m[i];
    gt = gt || (eq && gt_i);
    eq = eq && !lt_i && !gt_i;
    (void)lt_i;
  }
  return gt || eq;
}

// 32-bit add/subtract with carry.  On the device these are clang's
// __builtin_addc/__builtin_subc, which lower to v_add_co_u32 / v_addc_co_u32
// (v_sub_co_u32 / v_subb_co_u32) chains: one instruction per limb.  (Plain C
// on uint64_t becomes 64-bit v_lshl_add_u64 sequences with twice the registers.)
FTS_HD uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_addc(a, b, cin, cout);
#else
  uint64_t s = (uint64_t)a + b + cin;
  *cout = (uint32_t)(s >> 32);
  return (uint32_t)s;
#endif
}
FTS_HD uint32_t subb32(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_subc(a, b, bin, bout);
#else
  uint64_t d = (uint64_t)a - b - bin;
  *bout = (uint32_t)(d >> 63);
  return (uint32_t)d;
#endif
}

// r = a - b (borrow discarded); returns borrow
FTS_HD uint32_t sub8(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = subb32(a[i], b[i], borrow, &borrow);
  return borrow;
}

FTS_HD uint32_t add8(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = addc32(a[i], b[i], c, &c);
  return c;
}

#ifndef FTS_ASM_CHAINS
#define FTS_ASM_CHAINS 1  // device: modular add/sub and final subtractions as asm carry chains
#endif
#include "fp_asm.h"
#if defined(__HIP_DEVICE_COMPILE__) && FTS_ASM_CHAINS
template <class M>
__device__ __forceinline__ void addmod_asm(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]);
template <>
__device__ __forceinline__ void addmod_asm<ModP>(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  addmod_p_asm(r, a, b);
}
template <>
__device__ __forceinline__ void addmod_asm<ModR>(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  addmod_r_asm(r, a, b);
}
template <class M>
__device__ __forceinline__ void submod_asm(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]);
template <>
__device__ __forceinline__ void submod_asm<ModP>(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  submod_p_asm(r, a, b);
}
template <>
__device__ __forceinline__ void submod_asm<ModR>(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  submod_r_asm(r, a, b);
}
template <class M>
__device__ __forceinline__ void condsub_asm(uint32_t x[8]);
template <>
__device__ __forceinline__ void condsub_asm<ModP>(uint32_t x[8]) {
  condsub_p_asm(x);
}
template <>
__device__ __forceinline__ void condsub_asm<ModR>(uint32_t x[8]) {
  condsub_r_asm(x);
}
#endif

template <class M>
FTS_HD Fe<M> operator+(const Fe<M>& a, const Fe<M>& b) {
#if defined(__HIP_DEVICE_COMPILE__) && FTS_ASM_CHAINS
  Fe<M> o;
  addmod_asm<M>(o.v, a.v, b.v);
  return o;
#endif
  Fe<M> r, t;
  add8(r.v, a.v, b.v);  // < 2m < 2^256: no carry out
  uint32_t mm[8];
#pragma unroll
  for (int i = 0; i < 8; i++) mm[i] = M::m[i];
  uint32_t br = sub8(t.v, r.v, mm);
  return br ? r : t;
}

template <class M>
FTS_HD Fe<M> operator-(const Fe<M>& a, const Fe<M>& b) {
#if defined(__HIP_DEVICE_COMPILE__) && FTS_ASM_CHAINS
  Fe<M> o;
  submod_asm<M>(o.v, a.v, b.v);
  return o;
#endif
  Fe<M> r, t;
  uint32_t br = sub8(r.v, a.v, b.v);
  uint32_t mm[8];
#pragma unroll
  for (int i = 0; i < 8; i++) mm[i] = M::m[i];
  add8(t.v, r.v, mm);
  return br ? t : r;
}

template <class M>
FTS_HD Fe<M> fe_neg(const Fe<M>& a) {
  return fe_zero<M>() - a;
}

template <class M>
FTS_HD Fe<M> fe_dbl(const Fe<M>& a) {
  return a + a;
}

#include "fp_fips.h"
#ifndef FTS_ONEASM
#define FTS_ONEASM 1  // device: whole limb products as one asm statement (gen_oneasm.py)
#endif
#include "fp_oneasm.h"

#if defined(__HIP_DEVICE_COMPILE__)
template <class M>
__device__ __forceinline__ Fe<M> mont_mul_fips(const Fe<M>& a, const Fe<M>& b) {
  Fe<M> x, y;
#if FTS_ONEASM
  mont_mul_oneasm<M>(x.v, a.v, b.v);
#else
  mont_mul_fips_limbs<M>(x.v, a.v, b.v);
#endif
#if FTS_ASM_CHAINS
  condsub_asm<M>(x.v);
  (void)y;
  return x;
#else
  uint32_t pm[8];
#pragma unroll
  for (int j = 0; j < 8; j++) pm[j] = M::m[j];
  uint32_t br = sub8(y.v, x.v, pm);
  return br ? x : y;
#endif
}
#endif

// Montgomery multiplication, CIOS, 32-bit limbs.  Inputs < m, output < m.
template <class M>
FTS_HD Fe<M> mont_mul_cios(const Fe<M>& a, const Fe<M>& b) {
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
    uint32_t m = t[0] * M::inv;
    c = (uint64_t)m * M::m[0] + t[0];
#pragma unroll
    for (int j = 1; j < 8; j++) {
      c = (uint64_t)m * M::m[j] + t[j] + (c >> 32);
      t[j - 1] = (uint32_t)c;
    }
    s = (uint64_t)t[8] + (c >> 32);
    t[7] = (uint32_t)s;
    t[8] = t[9] + (uint32_t)(s >> 32);
  }
  Fe<M> r, u;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  uint32_t mm[8];
#pragma unroll
  for (int i = 0; i < 8; i++) mm[i] = M::m[i];
  uint32_t br = sub8(u.v, r.v, mm);
  // t < 2m and m < 2^254, so t[8] == 0 here
  return br ? r : u;
}

#if !defined(__HIP_DEVICE_COMPILE__) && defined(FTS_HOST64)
// Host-only (CPU baseline build, oracle/cpu): the same Montgomery product
// with 4 x 64-bit limbs and 128-bit products.  R = 2^256 in both limb
// layouts and the 8 x u32 little-endian limbs ARE the 4 x u64 limbs in
// memory, so results are bit-identical to the 32-bit CIOS.
constexpr uint64_t fts_neg_inv64(uint64_t m0) {
  uint64_t y = 1;
  for (int i = 0; i < 7; i++) y *= 2 - m0 * y;  // Newton: y = m0^-1 mod 2^64
  return (uint64_t)0 - y;
}
template <class M>
inline Fe<M> mont_mul_host64(const Fe<M>& a, const Fe<M>& b) {
  typedef unsigned __int128 u128;
  constexpr uint64_t m0 = (uint64_t)M::m[0] | ((uint64_t)M::m[1] << 32), m1 = (uint64_t)M::m[2] | ((uint64_t)M::m[3] << 32),
                     m2 = (uint64_t)M::m[4] | ((uint64_t)M::m[5] << 32), m3 = (uint64_t)M::m[6] | ((uint64_t)M::m[7] << 32);
  constexpr uint64_t inv = fts_neg_inv64(m0);
  const uint64_t m[4] = {m0, m1, m2, m3};
  uint64_t x[4], y[4];
  for (int i = 0; i < 4; i++) {
    x[i] = (uint64_t)a.v[2 * i] | ((uint64_t)a.v[2 * i + 1] << 32);
    y[i] = (uint64_t)b.v[2 * i] | ((uint64_t)b.v[2 * i + 1] << 32);
  }
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c = (u128)x[j] * y[i] + t[j] + (uint64_t)(c >> 64);
      t[j] = (uint64_t)c;
    }
    u128 s = (u128)t[4] + (uint64_t)(c >> 64);
    t[4] = (uint64_t)s;
    t[5] = (uint64_t)(s >> 64);
    uint64_t q = t[0] * inv;
    c = (u128)q * m[0] + t[0];
    for (int j = 1; j < 4; j++) {
      c = (u128)q * m[j] + t[j] + (uint64_t)(c >> 64);
      t[j - 1] = (uint64_t)c;
    }
    s = (u128)t[4] + (uint64_t)(c >> 64);
    t[3] = (uint64_t)s;
    t[4] = t[5] + (uint64_t)(s >> 64);
  }
  // t < 2m: one conditional subtraction
  uint64_t u[4], br = 0;
  for (int j = 0; j < 4; j++) {
    u128 d = (u128)t[j] - m[j] - br;
    u[j] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  const uint64_t* r = br ? t : u;
  Fe<M> o;
  for (int i = 0; i < 4; i++) {
    o.v[2 * i] = (uint32_t)r[i];
    o.v[2 * i + 1] = (uint32_t)(r[i] >> 32);
  }
  return o;
}
#endif

#ifndef FTS_MUL_IMPL
#define FTS_MUL_IMPL 1  // 0: CIOS in C, 1: FIPS with inline v_mad_u64_u32 (device)
#endif

template <class M>
FTS_HD Fe<M> operator*(const Fe<M>& a, const Fe<M>& b) {
  FTS_COUNT_MUL();
#if defined(__HIP_DEVICE_COMPILE__) && FTS_MUL_IMPL == 1
  return mont_mul_fips(a, b);
#elif !defined(__HIP_DEVICE_COMPILE__) && defined(FTS_HOST64)
  return mont_mul_host64(a, b);
#else
  return mont_mul_cios(a, b);
#endif
}

template <class M>
FTS_HD Fe<M> fe_sqr(const Fe<M>& a) {
  return a * a;
}

template <class M>
FTS_HD bool fe_is_zero(const Fe<M>& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= a.v[i];
  return o == 0;
}

template <class M>
FTS_HD bool fe_eq(const Fe<M>& a, const Fe<M>& b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= a.v[i] ^ b.v[i];
  return o == 0;
}

// canonical integer (little-endian limbs, any value < 2^256) -> Montgomery
template <class M>
FTS_HD Fe<M> fe_from_int(const uint32_t a[8]) {
  // reduce a < 2^256 to < m by conditional subtractions (m > 2^253: at most 7)
  Fe<M> x;
#pragma unroll
  for (int i = 0; i < 8; i++) x.v[i] = a[i];
  uint32_t mm[8];
#pragma unroll
  for (int i = 0; i < 8; i++) mm[i] = M::m[i];
#pragma nounroll
  for (int k = 0; k < 7; k++) {
    uint32_t t[8];
    uint32_t br = sub8(t, x.v, mm);
    if (!br) {
#pragma unroll
      for (int i = 0; i < 8; i++) x.v[i] = t[i];
    }
  }
  return x * fe_const<M>(M::r2);
}

// Montgomery -> canonical integer limbs
template <class M>
FTS_HD void fe_to_int(uint32_t out[8], const Fe<M>& a) {
  Fe<M> one;
#pragma unroll
  for (int i = 0; i < 8; i++) one.v[i] = (i == 0);
  Fe<M> r = a * one;
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = r.v[i];
}

// big-endian 32 bytes <-> limbs
FTS_HD void be32_to_limbs(uint32_t out[8], const uint8_t* b) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint8_t* q = b + 28 - 4 * i;
    out[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}

// be32_to_limbs / limbs_to_be32 for GLOBAL memory: 16-byte vector accesses
// when the address is 16-byte aligned (the planners align wire and arena
// entries), byte accesses otherwise.  (Not for private arrays: taking a vector
// view of a local array would put it in scratch memory.)
FTS_HD void be32_to_limbs_g(uint32_t out[8], const uint8_t* b) {
#if defined(__HIP_DEVICE_COMPILE__)
  if ((((uintptr_t)b) & 15) == 0) {
    uint4 v0 = reinterpret_cast<const uint4*>(b)[0], v1 = reinterpret_cast<const uint4*>(b)[1];
    out[7] = __builtin_bswap32(v0.x);
    out[6] = __builtin_bswap32(v0.y);
    out[5] = __builtin_bswap32(v0.z);
    out[4] = __builtin_bswap32(v0.w);
    out[3] = __builtin_bswap32(v1.x);
    out[2] = __builtin_bswap32(v1.y);
    out[1] = __builtin_bswap32(v1.z);
    out[0] = __builtin_bswap32(v1.w);
    return;
  }
#endif
  be32_to_limbs(out, b);
}

FTS_HD void limbs_to_be32(uint8_t* b, const uint32_t in[8]);
FTS_HD void limbs_to_be32_g(uint8_t* b, const uint32_t in[8]) {
#if defined(__HIP_DEVICE_COMPILE__)
  if ((((uintptr_t)b) & 15) == 0) {
    uint4 v0, v1;
    v0.x = __builtin_bswap32(in[7]);
    v0.y = __builtin_bswap32(in[6]);
    v0.z = __builtin_bswap32(in[5]);
    v0.w = __builtin_bswap32(in[4]);
    v1.x = __builtin_bswap32(in[3]);
    v1.y = __builtin_bswap32(in[2]);
    v1.z = __builtin_bswap32(in[1]);
    v1.w = __builtin_bswap32(in[0]);
    reinterpret_cast<uint4*>(b)[0] = v0;
    reinterpret_cast<uint4*>(b)[1] = v1;
    return;
  }
#endif
  limbs_to_be32(b, in);
}

FTS_HD void limbs_to_be32(uint8_t* b, const uint32_t in[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint8_t* q = b + 28 - 4 * i;
    q[0] = (uint8_t)(in[i] >> 24);
    q[1] = (uint8_t)(in[i] >> 16);
    q[2] = (uint8_t)(in[i] >> 8);
    q[3] = (uint8_t)in[i];
  }
}

// a^e for a fixed 256-bit exponent (left-to-right, 2-bit windows: 3 table
// entries keep the register footprint small; 256 squarings + <= 128 products)
template <class M>
FTS_HDN Fe<M> fe_pow(const Fe<M>& a, const uint32_t* e) {
  Fe<M> a2 = fe_sqr(a);
  Fe<M> a3 = a2 * a;
  Fe<M> r = fe_one<M>();
#pragma nounroll
  for (int w = 127; w >= 0; w--) {
    r = fe_sqr(r);
    r = fe_sqr(r);
    uint32_t d = (e[w >> 4] >> ((w & 15) * 2)) & 3;
    if (d) {
      Fe<M> s;
#pragma unroll
      for (int i = 0; i < 8; i++) s.v[i] = d == 1 ? a.v[i] : (d == 2 ? a2.v[i] : a3.v[i]);
      r = r * s;
    }
  }
  return r;
}

FTS_HD fp fp_inv(const fp& a) { return fe_pow<ModP>(a, P_MINUS_2); }

// Variable-time inverse by the binary extended Euclidean algorithm: ~2 log2 p
// halvings and ~log2 p subtractions of 8-limb integers, about 5x fewer
// instructions than the Fermat chain.  For latency-bound single-lane code on
// public values only (MSM Horner); the data-dependent loop diverges in a wave.
}  // namespace fts
#include "safegcd.h"
namespace fts {

FTS_HD fp fp_inv_eea(const fp& am) {
  if (fe_is_zero(am)) return am;
  uint32_t u[8], v[8], x1[8], x2[8], pm[8], t[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    u[i] = am.v[i];  // the Montgomery representative a R as a plain integer
    v[i] = P_MOD[i];
    pm[i] = P_MOD[i];
    x1[i] = i == 0 ? 1u : 0u;
    x2[i] = 0;
  }
  auto is_one = [](const uint32_t* a) {
    uint32_t o = a[0] ^ 1u;
    for (int i = 1; i < 8; i++) o |= a[i];
    return o == 0;
  };
  // a / 2 and x / 2 mod p (x + p < 2^255 when x is odd)
  auto halve = [&](uint32_t* a, uint32_t* x) {
    for (int i = 0; i < 7; i++) a[i] = (a[i] >> 1) | (a[i + 1] << 31);
    a[7] >>= 1;
    if (x[0] & 1) add8(x, x, pm);
    for (int i = 0; i < 7; i++) x[i] = (x[i] >> 1) | (x[i + 1] << 31);
    x[7] >>= 1;
  };
  while (!is_one(u) && !is_one(v)) {
    while (!(u[0] & 1)) halve(u, x1);
    while (!(v[0] & 1)) halve(v, x2);
    if (sub8(t, u, v) == 0) {  // u >= v
      for (int i = 0; i < 8; i++) u[i] = t[i];
      if (sub8(x1, x1, x2)) add8(x1, x1, pm);
    } else {
      sub8(v, v, u);
      if (sub8(x2, x2, x1)) add8(x2, x2, pm);
    }
  }
  // x = (a R)^-1 as a plain integer; the Montgomery form of a^-1 is x R^2
  const bool from_u = is_one(u);  // select values, not arrays: no private-memory copy
  fp x;
#pragma unroll
  for (int i = 0; i < 8; i++) x.v[i] = from_u ? x1[i] : x2[i];
  fp r2 = fe_const<ModP>(P_R2);
  return (x * r2) * r2;
}
// the same inverse by Bernstein-Yang divsteps (dev/safegcd.h; checked against
// fp_inv_eea on the device and the host); FTS_INV_EEA = 1 keeps the Euclid
#ifndef FTS_INV_EEA
#define FTS_INV_EEA 0
#endif
// divsteps on 30-bit limbs (default) or 62-bit limbs (FTS_INV_SG30 = 0)
#ifndef FTS_INV_SG30
#define FTS_INV_SG30 1
#endif
template <int LIMBS>
FTS_HD fp fp_inv_sg(const fp& am) {
  if (fe_is_zero(am)) return am;
  fp x;
  // (a R)^-1 as a plain integer; the Montgomery form of a^-1 is x R^2
  if (LIMBS == 30)
    sg30_inv_int(am.v, x.v);
  else
    sg_inv_int(am.v, x.v);
  fp r2 = fe_const<ModP>(P_R2);
  return (x * r2) * r2;
}
FTS_HD fp fp_inv_var(const fp& am) {
#if FTS_INV_EEA
  return fp_inv_eea(am);
#elif FTS_INV_SG30
  return fp_inv_sg<30>(am);
#else
  return fp_inv_sg<62>(am);
#endif
}
FTS_HD fr fr_inv(const fr& a) { return fe_pow<ModR>(a, R_MINUS_2); }

// square root for p = 3 mod 4; returns false if a is not a square
FTS_HD bool fp_sqrt(fp& out, const fp& a) {
  fp s = fe_pow<ModP>(a, P_SQRT_EXP);
  out = s;
  return fe_eq(fe_sqr(s), a);
}

}  // namespace fts

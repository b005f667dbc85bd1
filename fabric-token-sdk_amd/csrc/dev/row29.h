// Row-distributed carry-free Fp arithmetic for latency-bound single-wave
// chains (the MSM's Horner combination of the window sums): one field element
// per DPP row of 16 lanes, lane r holding limb r of the 9 x 29-bit signed
// representation of dev/fp29.h (lanes 9..15 hold 0), so a wave carries four
// independent elements, one per row.
//
// A one-lane product (f29_mul_c) issues 162 v_mad_i64_i32 for one result; here
// the 81 limb products are 9 row-wide MADs (lane c accumulates column c: a_i
// broadcast with row_newbcast:i times b_(c-i) shifted in with row_shr:i) and
// the Montgomery reduction 9 more (lane c adds m_k p_(c-k)), each step's digit
// m_k read from lane k by row_newbcast and its carry moved to lane k + 1.  The
// results are the SAME integers with the same normalised limbs as f29_mul_c /
// f29_norm / f29_reduce (normalisation is unique: limbs 0..7 in [0, 2^29), limb
// 8 the signed rest), so code built on them keeps f29's bounds and bytes.
// tools/fpcheck.hip checks every routine against its f29 counterpart on the
// device (ftz_rowcheck).
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "fp29.h"

namespace fts {

// this lane's limb of a row element
struct r29 {
  int32_t v;
};

__device__ __forceinline__ uint32_t row_lane() { return threadIdx.x & 15; }
__device__ __forceinline__ uint32_t row_index() { return (threadIdx.x >> 4) & 3; }

template <int N>
__device__ __forceinline__ int32_t dpp_bcast(int32_t x) {  // every lane of the row: lane N's x
  return __builtin_amdgcn_update_dpp(0, x, 0x150 + N, 0xF, 0xF, false);
}
template <int N>
__device__ __forceinline__ int32_t dpp_shr(int32_t x) {  // lane r: lane r - N's x (0 below the row)
  if constexpr (N == 0)
    return x;
  else
    return __builtin_amdgcn_update_dpp(0, x, 0x110 + N, 0xF, 0xF, true);
}
template <int N>
__device__ __forceinline__ int32_t dpp_shl(int32_t x) {  // lane r: lane r + N's x (0 past the row)
  if constexpr (N == 0)
    return x;
  else
    return __builtin_amdgcn_update_dpp(0, x, 0x100 + N, 0xF, 0xF, true);
}
template <int N>
__device__ __forceinline__ int64_t dpp_bcast64(int64_t x) {
  const uint32_t lo = (uint32_t)dpp_bcast<N>((int32_t)(uint32_t)x);
  const uint32_t hi = (uint32_t)dpp_bcast<N>((int32_t)(uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
template <int N>
__device__ __forceinline__ int64_t dpp_shr64(int64_t x) {
  const uint32_t lo = (uint32_t)dpp_shr<N>((int32_t)(uint32_t)x);
  const uint32_t hi = (uint32_t)dpp_shr<N>((int32_t)(uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
template <int N>
__device__ __forceinline__ int64_t dpp_shl64(int64_t x) {
  const uint32_t lo = (uint32_t)dpp_shl<N>((int32_t)(uint32_t)x);
  const uint32_t hi = (uint32_t)dpp_shl<N>((int32_t)(uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, class F>
__device__ __forceinline__ void row_for(const F& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    row_for<B + 1, E>(f);
  }
}

// lane r of the row's copy of an f29 (the conversions in and out)
__device__ __forceinline__ r29 row_from(const f29& a) {
  const uint32_t r = row_lane();
  int32_t v = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) v = r == (uint32_t)i ? a.l[i] : v;
  return {v};
}
__device__ __forceinline__ f29 row_to(const r29& a) {
  f29 o;
  row_for<0, 9>([&](auto I) { o.l[I] = dpp_bcast<I>(a.v); });
  return o;
}

__device__ __forceinline__ r29 row_add(const r29& a, const r29& b) { return {a.v + b.v}; }
__device__ __forceinline__ r29 row_sub(const r29& a, const r29& b) { return {a.v - b.v}; }

// exact normalisation of lanes 0..8 (limbs 0..7 into [0, 2^29), lane 8 the
// signed rest) by parallel carry rounds until no lane below 8 carries: the
// unique form f29_norm's sequential sweep produces.  x: the lane's 64-bit limb.
__device__ __forceinline__ int32_t row_norm64(int64_t x) {
  const uint32_t r = row_lane();
  for (;;) {
    const int64_t c = r < 8 ? (x >> 29) : 0;
    if (!__builtin_amdgcn_ballot_w64(c != 0)) break;  // wave-uniform exit: every row normalised
    x = (r < 8 ? (x & F29_MASK) : x) + dpp_shr64<1>(c);
  }
  return (int32_t)x;
}
__device__ __forceinline__ r29 row_norm(const r29& a) { return {row_norm64((int64_t)a.v)}; }

// f29_reduce: value - q p, q from the top two limbs (the same double estimate)
__device__ __forceinline__ r29 row_reduce(const r29& a) {
  const double t = (double)dpp_bcast<8>(a.v) * 536870912.0 + (double)dpp_bcast<7>(a.v);
  const int32_t q = (int32_t)__builtin_rint(t * P29_TOP_INV);
  const uint32_t r = row_lane();
  int32_t pr = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) pr = r == (uint32_t)i ? P29[i] : pr;
  return {row_norm64((int64_t)a.v - (int64_t)q * pr)};
}

// a == 0 (after row_reduce's normalisation: every limb of the row zero)
__device__ __forceinline__ bool row_zero_reduced(const r29& a) {
  const uint64_t nz = __builtin_amdgcn_ballot_w64(a.v != 0);
  return ((nz >> (16 * row_index())) & 0xFFFF) == 0;
}
__device__ __forceinline__ bool row_is_zero(const r29& a) { return row_zero_reduced(row_reduce(a)); }

// f29_mul_c: the Montgomery product a b / 2^261 with f29_mul_c's digits m_k
__device__ __forceinline__ r29 row_mul(const r29& a, const r29& b) {
  const uint32_t r = row_lane();
  int64_t col = 0;  // lane c: column c (c <= 15)
  row_for<0, 9>([&](auto I) { col += (int64_t)dpp_bcast<I>(a.v) * dpp_shr<I>(b.v); });
  int64_t col16 = (int64_t)dpp_bcast<8>(a.v) * dpp_bcast<8>(b.v);  // column 16, in every lane
  int32_t prow = 0;  // lane r: p_r
#pragma unroll
  for (int i = 0; i < 9; i++) prow = r == (uint32_t)i ? P29[i] : prow;
  row_for<0, 9>([&](auto K) {
    const uint32_t m = ((uint32_t)dpp_bcast<K>((int32_t)(uint32_t)col) * P29_INV) & (uint32_t)F29_MASK;
    col += (int64_t)(int32_t)m * dpp_shr<K>(prow);  // lane c += m p_(c-K)
    if constexpr (K == 8) col16 += (int64_t)(int32_t)m * P29[8];
    const int64_t t = dpp_bcast64<K>(col) >> 29;  // column K's low 29 bits are zero now
    col += r == (uint32_t)(K + 1) ? t : 0;
  });
  // columns 9..16 -> lanes 0..7, then the exact carry sweep
  int64_t x = dpp_shl64<9>(col);
  x = r == 7 ? col16 : (r < 7 ? x : 0);
  return {row_norm64(x)};
}

// up to four independent products, product q on row q, every row getting all
// of them back (ds_bpermute from lane 16 q + r)
template <int CNT>
__device__ __forceinline__ void row_level(const r29 (&a)[CNT], const r29 (&b)[CNT], r29 (&out)[CNT]) {
  if constexpr (CNT == 1) {
    out[0] = row_mul(a[0], b[0]);
  } else {
    const uint32_t q = row_index();
    r29 x = a[0], y = b[0];
#pragma unroll
    for (int i = 1; i < CNT; i++) {
      x.v = q == (uint32_t)i ? a[i].v : x.v;
      y.v = q == (uint32_t)i ? b[i].v : y.v;
    }
    const r29 p = row_mul(x, y);
#pragma unroll
    for (int i = 0; i < CNT; i++)
      out[i].v = __builtin_amdgcn_ds_bpermute((int)((16 * i + row_lane()) * 4), p.v);
  }
}

}  // namespace fts

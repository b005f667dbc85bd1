// Kernels of the standalone G1 MSM (dev/msm.h): one lane per item.
#include <hip/hip_runtime.h>

#include "dev/msm.h"
#include "launch.h"
#include "dev/row29.h"

using namespace fts;

#define LANE_PROLOGUE(n)                                  \
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;     \
  if (i >= (n)) return;

// 64-byte gnark RawBytes (uncompressed, big-endian) -> Montgomery affine;
// ok[i] = 0 for a point off the curve or not in canonical form.
__global__ void __launch_bounds__(256) k_msm_load_pts(uint32_t n, const uint8_t* raw_pts, G1Dev* pts, uint8_t* ok) {
  LANE_PROLOGUE(n);
  g1a a;
  ok[i] = g1_from_raw(raw_pts + 64 * (size_t)i, a) ? 1 : 0;
  G1Dev d;
  g1_store(d, a);
  pts[i] = d;
}

// gnark SetBytes check of n 64-byte element slots (dev/jobs.h g1_setbytes;
// token-request actions, request.cpp)
__global__ void __launch_bounds__(256) k_g1_check(uint32_t n, const uint8_t* slots, uint8_t* ok) {
  LANE_PROLOGUE(n);
  g1a a;
  ok[i] = g1_setbytes(slots + 64 * (size_t)i, 64, a) ? 1 : 0;
}

// final add of a point-split MSM (dev/msm.h g1_sum_raw): one lane; status[0] =
// n on success, else the index of the first bad point
__global__ void __launch_bounds__(64) k_g1_sum(uint32_t n, const uint8_t* raw, uint8_t* out, uint32_t* status) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  status[0] = g1_sum_raw(n, raw, out);
}

// 32-byte big-endian scalars -> 8 limbs reduced mod r
__global__ void __launch_bounds__(256) k_msm_load_scal(uint32_t n, const uint8_t* raw_scal, uint32_t (*scal)[8]) {
  LANE_PROLOGUE(n);
  uint32_t k[8];
  be32_to_limbs(k, raw_scal + 32 * (size_t)i);
  fe_to_int(scal[i], fe_from_int<ModR>(k));
}

// point i's entries (every window, both GLV halves) counted into their
// (window, bucket) group: the counting sort of small plans (msm_rt.hip)
__device__ __forceinline__ void msm_count_point(const MsmPlan& p, uint32_t i, const uint32_t* key, uint32_t* cnt) {
  const uint32_t halves = p.glv ? 2u : 1u;
  for (uint32_t w = 0; w < p.windows; w++)
    for (uint32_t h = 0; h < halves; h++) atomicAdd(&cnt[w * p.buckets + key[(size_t)w * p.nv + i + h * p.n]], 1u);
}

// one lane per point: sort keys + values of every window (dev/msm.h
// msm_job_keys); cnt != nullptr: also the group counts
__global__ void __launch_bounds__(256) k_msm_keys(MsmPlan p, const uint32_t (*scal)[8], uint32_t* key,
                                                  uint32_t* val, uint32_t* cnt) {
  LANE_PROLOGUE(p.n);
  msm_job_keys(p, i, scal, key, val);
  if (cnt) msm_count_point(p, i, key, cnt);
}

// counting sort, second half: entry t of group g lands at start[g] + its rank
// among the group's entries (an atomic decrement of the count: any order in a
// bucket gives the same sum); one lane per point, every window
__global__ void __launch_bounds__(256) k_msm_scatter(MsmPlan p, const uint32_t* key, const uint32_t* val,
                                                     const uint32_t* start, uint32_t* cnt, uint32_t* perm) {
  LANE_PROLOGUE(p.n);
  const uint32_t halves = p.glv ? 2u : 1u;
  for (uint32_t w = 0; w < p.windows; w++)
    for (uint32_t h = 0; h < halves; h++) {
      const size_t t = (size_t)w * p.nv + i + h * p.n;
      const uint32_t g = w * p.buckets + key[t];
      perm[start[g] + atomicSub(&cnt[g], 1u) - 1u] = val[t];
    }
}

// the same from 32-byte big-endian scalars in HBM for points [i0, i1) (the
// chunk a host copy has delivered): reduce mod r, keep the limbs for later runs,
// and write the sort keys -- k_msm_load_scal and k_msm_keys in one pass
__global__ void __launch_bounds__(256) k_msm_keys_raw(MsmPlan p, uint32_t i0, uint32_t i1, const uint8_t* raw,
                                                      uint32_t (*scal)[8], uint32_t* key, uint32_t* val,
                                                      uint32_t* cnt) {
  uint32_t i = i0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= i1) return;
  uint32_t k[8];
  be32_to_limbs_g(k, raw + 32 * (size_t)i);
  fe_to_int(scal[i], fe_from_int<ModR>(k));
  msm_job_keys(p, i, scal, key, val);
  if (cnt) msm_count_point(p, i, key, cnt);
}

// one lane per sorted entry: bucket ranges
__global__ void __launch_bounds__(256) k_msm_bounds(MsmPlan p, uint64_t total, const uint32_t* skey,
                                                    const uint32_t* sval, uint32_t* start, uint32_t* end) {
  uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  msm_job_bounds(p, t, total, skey, sval, start, end);
}

// exclusive scan, 1024 elements per workgroup; block totals to `tot`
__global__ void __launch_bounds__(1024) k_scan_block(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* tot) {
  __shared__ uint32_t s[1024];
  uint32_t t = threadIdx.x, i = blockIdx.x * 1024 + t;
  uint32_t v = i < n ? in[i] : 0;
  s[t] = v;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {
    uint32_t a = t >= o ? s[t - o] : 0;
    __syncthreads();
    s[t] += a;
    __syncthreads();
  }
  if (i < n) out[i] = s[t] - v;
  if (t == 1023) tot[blockIdx.x] = s[1023];
}

// k_msm_counts fused with the first level of the slot-count scan: count[g] and
// the bucket's slot count m_g, then the block-exclusive scan of m into soff and
// the block totals into tot (the higher levels as in scan(), msm_rt.hip)
__global__ void __launch_bounds__(1024) k_msm_counts_scan(MsmPlan p, const uint32_t* start, const uint32_t* end,
                                                          uint32_t* count, uint32_t* soff, uint32_t* tot) {
  __shared__ uint32_t sh[1024];
  const uint32_t n = p.rw * p.buckets, t = threadIdx.x, i = blockIdx.x * 1024 + t;
  uint32_t v = 0;
  if (i < n) {
    const uint32_t c = start ? end[i] - start[i] : end[i];
    count[i] = c;
    v = msm_bucket_slots(p, c);
  }
  sh[t] = v;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {
    uint32_t a = t >= o ? sh[t - o] : 0;
    __syncthreads();
    sh[t] += a;
    __syncthreads();
  }
  if (i < n) soff[i] = sh[t] - v;
  if (t == 1023) tot[blockIdx.x] = sh[1023];
}

__global__ void __launch_bounds__(1024) k_scan_add(uint32_t* out, uint32_t n, const uint32_t* add) {
  uint32_t i = blockIdx.x * 1024 + threadIdx.x;
  if (i < n) out[i] += add[blockIdx.x];
}

__global__ void __launch_bounds__(256) k_msm_owner(MsmPlan p, const uint32_t* count, const uint32_t* soff,
                                                   uint32_t* owner, uint32_t* wlo, uint32_t* whi) {
  LANE_PROLOGUE(p.rw * p.buckets);
  msm_job_owner(p, i, count, soff, owner, wlo, whi);
}

__global__ void __launch_bounds__(256) k_msm_phi(MsmPlan p, G1Dev* pts) {
  LANE_PROLOGUE(p.n);
  msm_job_phi(p, i, pts);
}

// resident-point mode: 2^(c w) P_v for every window (dev/msm.h msm_job_precompute)
__global__ void __launch_bounds__(256) k_msm_precompute(MsmPlan p, G1Dev* pts) {
  LANE_PROLOGUE(p.nv);
  msm_job_precompute(p, i, pts);
}

// ---- bucket slots ordered by length, so that the lanes of a wave add about
// the same number of points (bucket loads are Poisson-distributed).  Counting
// sort over the T + 1 lengths with per-block LDS histograms: one global atomic
// per (block, length) instead of one per slot on a handful of counters.
static constexpr uint32_t MSM_LEN_BINS = 1024;  // > slot_cap (checked by the planner)

__global__ void __launch_bounds__(256) k_msm_len_hist(MsmPlan p, const uint32_t* whi, const uint32_t* owner,
                                                      const uint32_t* soff, const uint32_t* count, uint32_t* hist) {
  __shared__ uint32_t h[MSM_LEN_BINS];
  uint32_t nb = p.slot_cap + 1, j = blockIdx.x * blockDim.x + threadIdx.x, L = whi[p.rw - 1];
  for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) h[b] = 0;
  __syncthreads();
  if (j < L) atomicAdd(&h[p.slot_cap - msm_slot_len(p, j, owner, soff, count)], 1u);  // longest first
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x)
    if (h[b]) atomicAdd(&hist[b], h[b]);
}

// exclusive scan of the (<= 1024) length bins, one block
__global__ void __launch_bounds__(1024) k_msm_len_scan(MsmPlan p, uint32_t* hist) {
  __shared__ uint32_t s[MSM_LEN_BINS];
  uint32_t t = threadIdx.x, nb = p.slot_cap + 1;
  uint32_t v = t < nb ? hist[t] : 0;
  s[t] = v;
  __syncthreads();
  for (uint32_t o = 1; o < MSM_LEN_BINS; o <<= 1) {
    uint32_t a = t >= o ? s[t - o] : 0;
    __syncthreads();
    s[t] += a;
    __syncthreads();
  }
  if (t < nb) hist[t] = s[t] - v;
}

__global__ void __launch_bounds__(256) k_msm_len_scatter(MsmPlan p, const uint32_t* whi, const uint32_t* owner,
                                                         const uint32_t* soff, const uint32_t* count,
                                                         uint32_t* cursor, uint32_t* order) {
  __shared__ uint32_t h[MSM_LEN_BINS];
  uint32_t nb = p.slot_cap + 1, j = blockIdx.x * blockDim.x + threadIdx.x, L = whi[p.rw - 1];
  for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) h[b] = 0;
  __syncthreads();
  uint32_t bin = 0, rank = 0;
  if (j < L) {
    bin = p.slot_cap - msm_slot_len(p, j, owner, soff, count);
    rank = atomicAdd(&h[bin], 1u);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x)
    if (h[b]) h[b] = atomicAdd(&cursor[b], h[b]);
  __syncthreads();
  if (j < L) order[h[bin] + rank] = j;
}

// one lane per bucket slot, slots taken in length order (all windows)
__global__ void __launch_bounds__(128) k_msm_bucket(MsmPlan p, const uint32_t* whi, const uint32_t* order,
                                                    const uint32_t* owner, const uint32_t* soff,
                                                    const uint32_t* start, const uint32_t* count,
                                                    const uint32_t* perm, const G1Dev* pts, G1JDev* slot_sum) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= whi[p.rw - 1]) return;
  uint32_t j = order[i];
  g1j_store(slot_sum[j], msm_job_slot(p, j, owner, soff, start, count, perm, pts));
}


// ---- 4-lane cooperative point arithmetic (the tree's additions; the serial
// Horner chain of FTS_MSM_HOST_HORNER=0 and the quad segments).  A
// wave issues a one-lane product at the cost of a 64-lane one, so the chain's
// latency is the number of dependent products times one product's latency:
// every lane holds the same point, lane k (mod 4) computes the k-th independent
// product of each dependency level (f29_mul_c: carry-free, column sums, short
// dependent chains; every quad of lanes does the same) and the lanes read the
// products of their quad through DPP quad_perm broadcasts (values stay in vector
// registers: read as uniform values, v_readlane, the compiler moved the point
// formulas to the scalar unit and spilled).  Same operations as j29_dbl / j29_add (dev/fp29.h) grouped
// into levels, so the same limbs.
// out[I..CNT) = the products of lanes I.. of this lane's quad (DPP quad_perm broadcast)
template <int I, int CNT>
__device__ __forceinline__ void quad_get(const f29& r, f29 (&out)[CNT]) {
  if constexpr (I < CNT) {
#pragma unroll
    for (int q = 0; q < 9; q++) out[I].l[q] = __builtin_amdgcn_mov_dpp(r.l[q], 0x55 * I, 0xF, 0xF, false);
    quad_get<I + 1, CNT>(r, out);
  }
}

// the operand of lane k (mod 4): a per-limb select chain on values pinned in
// vector registers (an empty asm per limb: otherwise the compiler turned the
// selects into loads from a dynamically indexed stack copy of the operands)
__device__ __forceinline__ f29 lane_sel(int k, const f29& v0, const f29& v1, const f29& v2, const f29& v3) {
  f29 r;
#pragma unroll
  for (int q = 0; q < 9; q++) {
    int32_t x0 = v0.l[q], x1 = v1.l[q], x2 = v2.l[q], x3 = v3.l[q];
    asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
    int32_t t = k == 1 ? x1 : x0;
    t = k == 2 ? x2 : t;
    r.l[q] = k == 3 ? x3 : t;
  }
  return r;
}

// a level of squarings only (f29_sqr_c: 45 limb products instead of 81)
template <int CNT>
__device__ __forceinline__ void coop29_sqr_level(const f29 (&a)[CNT], f29 (&out)[CNT]) {
  const int k = (int)(threadIdx.x & 3);
  quad_get<0, CNT>(f29_sqr_c(lane_sel(k, a[0], a[CNT > 1 ? 1 : 0], a[CNT > 2 ? 2 : 0], a[CNT > 3 ? 3 : 0])), out);
}

template <int CNT>
__device__ __forceinline__ void coop29_level(const f29 (&a)[CNT], const f29 (&b)[CNT], f29 (&out)[CNT]) {
  if constexpr (CNT == 1) {  // every lane computes the one product: no select, no broadcast
    out[0] = f29_mul_c(a[0], b[0]);
    return;
  }
  const int k = (int)(threadIdx.x & 3);  // every quad of lanes computes the level
  const f29& a1 = a[CNT > 1 ? 1 : 0];
  const f29& a2 = a[CNT > 2 ? 2 : 0];
  const f29& a3 = a[CNT > 3 ? 3 : 0];
  const f29& b1 = b[CNT > 1 ? 1 : 0];
  const f29& b2 = b[CNT > 2 ? 2 : 0];
  const f29& b3 = b[CNT > 3 ? 3 : 0];
  quad_get<0, CNT>(f29_mul_c(lane_sel(k, a[0], a1, a2, a3), lane_sel(k, b[0], b1, b2, b3)), out);
}

// dbl-2009-l (j29_dbl's formulas) in place: 3 product levels instead of 7
// products, the first two squarings only (Z3 = 2 Y Z as (Y + Z)^2 - Y^2 - Z^2:
// the same value, another representative).  The point lives in plain variables
// (a j29 carried through the loop with its flag was kept in scratch memory)
__device__ __forceinline__ void coop29_dbl(f29& X, f29& Y, f29& Z) {
  f29 A, Bq, Z3, C, T2, F, Y3a;
  {
    f29 a[4] = {X, Y, f29_norm(f29_add(Y, Z)), Z}, o[4];  // (Y + Z): B <= 3.5, L 1
    coop29_sqr_level<4>(a, o);
    A = o[0];
    Bq = o[1];
    Z3 = f29_reduce(f29_sub(f29_sub(o[2], o[1]), o[3]));  // (6, 3) -> (1.5, 1)
  }
  f29 E = f29_norm(f29_add(f29_add(A, A), A));
  {
    f29 t = f29_norm(f29_add(X, Bq));
    f29 a[3] = {Bq, t, E}, o[3];
    coop29_sqr_level<3>(a, o);
    C = o[0];
    T2 = o[1];
    F = o[2];
  }
  f29 D1 = f29_norm(f29_sub(f29_sub(T2, A), C));
  f29 D = f29_add(D1, D1);
  f29 X3 = f29_reduce(f29_sub(f29_norm(f29_sub(F, D)), D));
  {
    f29 a[1] = {E}, b[1] = {f29_norm(f29_sub(D, X3))}, o[1];
    coop29_level<1>(a, b, o);
    Y3a = o[0];
  }
  f29 C2 = f29_add(C, C);
  f29 C4 = f29_norm(f29_add(C2, C2));
  X = X3;
  Y = f29_reduce(f29_sub(Y3a, f29_add(C4, C4)));
  Z = Z3;
}

// add-2007-bl (j29_add) in place, (X, Y, Z, inf) += q: 5 product levels
// instead of 16 products
__device__ __forceinline__ void coop29_add(f29& X, f29& Y, f29& Z, bool& inf, const j29& q) {
  if (q.inf) return;
  if (inf) {
    X = q.x;
    Y = q.y;
    Z = q.z;
    inf = false;
    return;
  }
  f29 Z1Z1, Z2Z2, ZZ, U1, U2, t1, t2, S1, S2, I, J, V, R2, Z3p, Y3a, SJ;
  {
    f29 zs = f29_norm(f29_add(Z, q.z));
    f29 a[3] = {Z, q.z, zs}, b[3] = {Z, q.z, zs}, o[3];
    coop29_level<3>(a, b, o);
    Z1Z1 = o[0];
    Z2Z2 = o[1];
    ZZ = o[2];
  }
  {
    f29 a[4] = {X, q.x, q.z, Z}, b[4] = {Z2Z2, Z1Z1, Z2Z2, Z1Z1}, o[4];
    coop29_level<4>(a, b, o);
    U1 = o[0];
    U2 = o[1];
    t1 = o[2];
    t2 = o[3];
  }
  f29 H = f29_norm(f29_sub(U2, U1));
  f29 H2 = f29_norm(f29_add(H, H));
  {
    f29 a[3] = {Y, q.y, H2}, b[3] = {t1, t2, H2}, o[3];
    coop29_level<3>(a, b, o);
    S1 = o[0];
    S2 = o[1];
    I = o[2];
  }
  f29 rr = f29_sub(S2, S1);
  f29 r2 = f29_norm(f29_add(rr, rr));
  {
    f29 zd = f29_norm(f29_sub(f29_sub(ZZ, Z1Z1), Z2Z2));
    f29 a[4] = {H, U1, r2, zd}, b[4] = {I, I, r2, H}, o[4];
    coop29_level<4>(a, b, o);
    J = o[0];
    V = o[1];
    R2 = o[2];
    Z3p = o[3];
  }
  f29 X3 = f29_reduce(f29_sub(f29_sub(f29_sub(R2, J), V), V));
  {
    f29 a[2] = {r2, S1}, b[2] = {f29_norm(f29_sub(V, X3)), J}, o[2];
    coop29_level<2>(a, b, o);
    Y3a = o[0];
    SJ = o[1];
  }
  f29 Y3 = f29_reduce(f29_sub(f29_sub(Y3a, SJ), SJ));
  f29 Z3 = f29_reduce(Z3p);
  if (f29_reduced_zero(Z3)) {  // H == 0: p == q (a doubling) or p == -q (infinity)
    if (f29_is_zero(rr))
      coop29_dbl(X, Y, Z);
    else
      inf = true;
    return;
  }
  X = X3;
  Y = Y3;
  Z = Z3;
}

// ---- the same formulas on dev/row29.h: each element one DPP row, a level's
// (up to four) products one per row (row_level), so a product is 18 row-wide
// MADs instead of 162 one-lane ones; every limb identical to coop29_*.
// FTS_MSM_ROW_HORNER=1 selects these for the Horner chain.  Measured (round 6,
// profiles/r06/msm_row.txt): the rows' products are 2.36x faster than one-lane
// f29_mul_c in a dependent chain, but the whole MSM is 3-4% SLOWER than with
// the quad-cooperative coop29_* chain below (the normalisation rounds and the
// bpermute exchange eat the MAD saving), so the default stays 0.
#ifndef FTS_MSM_ROW_HORNER
#define FTS_MSM_ROW_HORNER 0
#endif
__device__ __forceinline__ r29 rnorm(const r29& a) { return row_norm(a); }
__device__ __forceinline__ r29 rred(const r29& a) { return row_reduce(a); }

__device__ __forceinline__ void row29_dbl(r29& X, r29& Y, r29& Z) {
  r29 A, Bq, Z3, C, T2, F, Y3a;
  {
    r29 a[4] = {X, Y, rnorm(row_add(Y, Z)), Z}, o[4];
    row_level<4>(a, a, o);
    A = o[0];
    Bq = o[1];
    Z3 = rred(row_sub(row_sub(o[2], o[1]), o[3]));
  }
  r29 E = rnorm(row_add(row_add(A, A), A));
  {
    r29 t = rnorm(row_add(X, Bq));
    r29 a[3] = {Bq, t, E}, o[3];
    row_level<3>(a, a, o);
    C = o[0];
    T2 = o[1];
    F = o[2];
  }
  r29 D1 = rnorm(row_sub(row_sub(T2, A), C));
  r29 D = row_add(D1, D1);
  r29 X3 = rred(row_sub(rnorm(row_sub(F, D)), D));
  {
    r29 a[1] = {E}, b[1] = {rnorm(row_sub(D, X3))}, o[1];
    row_level<1>(a, b, o);
    Y3a = o[0];
  }
  r29 C2 = row_add(C, C);
  r29 C4 = rnorm(row_add(C2, C2));
  X = X3;
  Y = rred(row_sub(Y3a, row_add(C4, C4)));
  Z = Z3;
}

__device__ __forceinline__ void row29_add(r29& X, r29& Y, r29& Z, bool& inf, const r29& qx, const r29& qy,
                                          const r29& qz, bool qinf) {
  if (qinf) return;
  if (inf) {
    X = qx;
    Y = qy;
    Z = qz;
    inf = false;
    return;
  }
  r29 Z1Z1, Z2Z2, ZZ, U1, U2, t1, t2, S1, S2, I, J, V, R2, Z3p, Y3a, SJ;
  {
    r29 zs = rnorm(row_add(Z, qz));
    r29 a[3] = {Z, qz, zs}, o[3];
    row_level<3>(a, a, o);
    Z1Z1 = o[0];
    Z2Z2 = o[1];
    ZZ = o[2];
  }
  {
    r29 a[4] = {X, qx, qz, Z}, b[4] = {Z2Z2, Z1Z1, Z2Z2, Z1Z1}, o[4];
    row_level<4>(a, b, o);
    U1 = o[0];
    U2 = o[1];
    t1 = o[2];
    t2 = o[3];
  }
  r29 H = rnorm(row_sub(U2, U1));
  r29 H2 = rnorm(row_add(H, H));
  {
    r29 a[3] = {Y, qy, H2}, b[3] = {t1, t2, H2}, o[3];
    row_level<3>(a, b, o);
    S1 = o[0];
    S2 = o[1];
    I = o[2];
  }
  r29 rr = row_sub(S2, S1);
  r29 r2 = rnorm(row_add(rr, rr));
  {
    r29 zd = rnorm(row_sub(row_sub(ZZ, Z1Z1), Z2Z2));
    r29 a[4] = {H, U1, r2, zd}, b[4] = {I, I, r2, H}, o[4];
    row_level<4>(a, b, o);
    J = o[0];
    V = o[1];
    R2 = o[2];
    Z3p = o[3];
  }
  r29 X3 = rred(row_sub(row_sub(row_sub(R2, J), V), V));
  {
    r29 a[2] = {r2, S1}, b[2] = {rnorm(row_sub(V, X3)), J}, o[2];
    row_level<2>(a, b, o);
    Y3a = o[0];
    SJ = o[1];
  }
  r29 Y3 = rred(row_sub(row_sub(Y3a, SJ), SJ));
  r29 Z3 = rred(Z3p);
  if (row_zero_reduced(Z3)) {  // H == 0: p == q (a doubling) or p == -q (infinity)
    if (row_is_zero(rr))
      row29_dbl(X, Y, Z);
    else
      inf = true;
    return;
  }
  X = X3;
  Y = Y3;
  Z = Z3;
}

// k P (k < 2^32) on the quad: j29_mul_small's 2-bit windows from the top one
// with coop29_dbl / coop29_add (k is quad-uniform; m P != O for 0 < m < 2^32)
__device__ __forceinline__ void coop29_mul_small(f29& X, f29& Y, f29& Z, bool& inf, uint32_t k) {
  if (inf) return;
  if (!k) {
    inf = true;
    return;
  }
  const j29 p1 = {X, Y, Z, false};
  f29 X2 = X, Y2 = Y, Z2 = Z;
  coop29_dbl(X2, Y2, Z2);
  const j29 p2 = {X2, Y2, Z2, false};
  bool i3 = false;
  f29 X3 = X2, Y3 = Y2, Z3 = Z2;
  coop29_add(X3, Y3, Z3, i3, p1);
  const j29 p3 = {X3, Y3, Z3, false};
  const int top = 31 - __builtin_clz(k), w = top >> 1;
  uint32_t d = (k >> (2 * w)) & 3u;
  const j29& a0 = d == 1 ? p1 : (d == 2 ? p2 : p3);
  X = a0.x;
  Y = a0.y;
  Z = a0.z;
  for (int i = w - 1; i >= 0; i--) {
    coop29_dbl(X, Y, Z);
    coop29_dbl(X, Y, Z);
    d = (k >> (2 * i)) & 3u;
    if (d) coop29_add(X, Y, Z, inf, d == 1 ? p1 : (d == 2 ? p2 : p3));
  }
}

// Segment sums (dev/msm.h msm_job_segment).  FTS_MSM_QUAD_SEG=1: one
// quad per segment, the running sums and the bl multiple (j29_mul_small: ~13
// doublings + 7 additions at 2^14) on coop29_*, 64 segments per 256-lane block;
// the stage is a latency-bound chain per segment (2^16 points: 55k segments, a
// single-lane chain of ~16 additions + 13 doublings).  0 (default, measured
// faster: the one-lane chains interleave their independent products and need
// a quarter of the waves): one lane per segment.
__global__ void __launch_bounds__(MSM_SEG_THREADS) k_msm_segment(MsmPlan p, uint32_t w0, uint32_t w1,
                                                                 const uint32_t* wlo, const uint32_t* whi,
                                                                 const uint32_t* owner, const G1JDev* slot_sum,
                                                                 G1JDev* part) {
#if FTS_MSM_QUAD_SEG
  const uint32_t i = w0 * p.segs + blockIdx.x * MSM_SEG_PER_BLOCK + (threadIdx.x >> 2);
  if (i >= w1 * p.segs) return;  // quad-uniform
  const uint32_t w = i / p.segs, sg = i - w * p.segs;
  const bool lead = (threadIdx.x & 3) == 0;
  const uint32_t lo = wlo[w] + sg * p.seg_len;
  uint32_t hi = lo + p.seg_len;
  if (hi > whi[w]) hi = whi[w];
  if (lo >= hi) {
    if (lead) g1j_store(part[i], jac_inf<fp>());
    return;
  }
  f29 RX{}, RY{}, RZ{}, AX{}, AY{}, AZ{};
  bool rinf = true, ainf = true;
  for (uint32_t j = hi; j > lo; j--) {
    coop29_add(RX, RY, RZ, rinf, j29_ld(slot_sum[j - 1]));
    if (j - 1 == lo || owner[j - 2] != owner[j - 1]) coop29_add(AX, AY, AZ, ainf, {RX, RY, RZ, rinf});
  }
  coop29_mul_small(RX, RY, RZ, rinf, owner[lo] - w * p.buckets);
  coop29_add(AX, AY, AZ, ainf, {RX, RY, RZ, rinf});
  if (lead) g1j_store(part[i], j29_to({AX, AY, AZ, ainf}));
#else
  uint32_t i = w0 * p.segs + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= w1 * p.segs) return;
  uint32_t w = i / p.segs, s = i - w * p.segs;
  g1j_store(part[i], msm_job_segment(p, w, s, wlo, whi, owner, slot_sum));
#endif
}

// tree sum of m consecutive parts per window in chunks of MSM_TREE_CHUNK:
// out[w][ceil(m / chunk)].  FTS_MSM_QUAD_TREE (default 1): a block of 256 lanes
// is 64 quads, each addition of a level runs on one quad (coop29_add: 5 product
// levels instead of one lane's 16 dependent products), a chunk of 128 parts is
// 7 levels.  0: one lane per addition, chunks of 256 (8 levels).  Only the
// levels the chunk's live parts need (a window's last level often holds a few
// dozen).  Carry-free form in LDS: one conversion in, one out.
__global__ void __launch_bounds__(256) k_msm_tree(const G1JDev* in, uint32_t m, G1JDev* out) {
  constexpr uint32_t CH = MSM_TREE_CHUNK;
  __shared__ j29 s[CH];
  const uint32_t chunks = (m + CH - 1) / CH;
  const uint32_t w = blockIdx.x / chunks, ch = blockIdx.x - w * chunks, t = threadIdx.x;
  const uint32_t i = ch * CH + t;
  if (t < CH) s[t] = i < m ? j29_ld(in[(size_t)w * m + i]) : j29_inf();
  __syncthreads();
  uint32_t live = min(CH, m - ch * CH), o = 1;
  while (2 * o < live) o *= 2;
#if FTS_MSM_QUAD_TREE
  const uint32_t q = t >> 2;  // quad-uniform branches: the 4 lanes hold the same point
  for (; live > 1; live = o, o >>= 1) {
    if (q < o && q + o < live) {
      const j29 a = s[q], b = s[q + o];
      f29 X = a.x, Y = a.y, Z = a.z;
      bool inf = a.inf;
      coop29_add(X, Y, Z, inf, b);
      if ((t & 3) == 0) s[q] = {X, Y, Z, inf};
    }
    __syncthreads();
  }
#else
  for (; live > 1; live = o, o >>= 1) {
    if (t < o && t + o < live) s[t] = j29_add(s[t], s[t + o]);
    __syncthreads();
  }
#endif
  if (t == 0) g1j_store(out[(size_t)w * chunks + ch], j29_to(s[0]));
}

// (FTS_MSM_HOST_HORNER=0 only: the default combines the windows on the host,
// msm_rt.hip msm_horner_host.)
// Horner steps for reduction windows w_hi-1 down to w_lo: acc = 2^c acc + W_w,
// on one wave with the 4-lane cooperative carry-free point ops, the Jacobian
// result in acc_buf.  W_w arrives as `per` partial sums (wparts[w per + k], the
// last tree level's chunks): the wave's 16 quads first add up the windows'
// partials in parallel (quad q takes windows q, q + 16, ...) and publish the
// window sums through LDS, which replaces a tree launch of one block per
// window.  The affine conversion (one binary-EEA inverse: ~40k instructions
// issued by a single lane) runs on the host after the 96-byte read-back
// (msm_rt.hip g1j_to_raw).  With pre (one reduction window) the chain is the
// window sum itself.
static constexpr uint32_t HORNER_MAX_WINDOWS = 32;
__global__ void __launch_bounds__(64) k_msm_horner(MsmPlan p, uint32_t w_hi, uint32_t w_lo, const G1JDev* wparts,
                                                   uint32_t per, G1JDev* acc_buf) {
  __shared__ j29 ws[HORNER_MAX_WINDOWS];
  if (blockIdx.x != 0) return;
  const uint32_t quad = threadIdx.x >> 2;
  for (uint32_t w = w_lo + quad; w < w_hi; w += 16) {
    f29 X{}, Y{}, Z{};
    bool inf = true;
    for (uint32_t k = 0; k < per; k++) coop29_add(X, Y, Z, inf, j29_ld(wparts[(size_t)w * per + k]));
    if ((threadIdx.x & 3) == 0) ws[w - w_lo] = {X, Y, Z, inf};
  }
  __syncthreads();
  j29 a0 = w_hi == p.rw ? j29_inf() : j29_ld(*acc_buf);
#if FTS_MSM_ROW_HORNER
  r29 X = row_from(a0.x), Y = row_from(a0.y), Z = row_from(a0.z);
  bool inf = a0.inf;
  for (int w = (int)w_hi - 1; w >= (int)w_lo; w--) {
    if (w != (int)p.rw - 1 && !inf)
      for (uint32_t q = 0; q < p.c; q++) row29_dbl(X, Y, Z);
    const j29& q = ws[w - (int)w_lo];
    row29_add(X, Y, Z, inf, row_from(q.x), row_from(q.y), row_from(q.z), q.inf);
  }
  const j29 res = {row_to(X), row_to(Y), row_to(Z), inf};
  if (threadIdx.x != 0) return;
  g1j_store(*acc_buf, j29_to(res));
#else
  f29 X = a0.x, Y = a0.y, Z = a0.z;
  bool inf = a0.inf;
  for (int w = (int)w_hi - 1; w >= (int)w_lo; w--) {
    if (w != (int)p.rw - 1 && !inf)
      for (uint32_t q = 0; q < p.c; q++) coop29_dbl(X, Y, Z);
    coop29_add(X, Y, Z, inf, ws[w - (int)w_lo]);
  }
  if (threadIdx.x != 0) return;
  g1j_store(*acc_buf, j29_to({X, Y, Z, inf}));
#endif
}

// test points with known logs: P_i = (i + off) G from the generator's fixed-base
// table, chunks of `chunk` consecutive points per lane made affine together
// (Montgomery batch inversion; zs is chunk * lanes Fp of scratch)
__global__ void __launch_bounds__(128) k_msm_genpoints(uint32_t n, uint32_t off, uint32_t chunk, const G1Dev* gtab,
                                                       G1JDev* jtmp, uint32_t (*zs)[8], G1Dev* pts) {
  uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t i0 = lane * chunk;
  if (i0 >= n) return;
  uint32_t cnt = n - i0 < chunk ? n - i0 : chunk;
  uint32_t k[8] = {i0 + off, 0, 0, 0, 0, 0, 0, 0};
  g1j acc = g1_fixed_acc(jac_inf<fp>(), gtab, G1B_GEN, k);
  g1a G = g1_load(gtab[(size_t)G1B_GEN * G1TAB_WINDOWS * G1TAB_DIGITS]);  // |d| = 1 of window 0
  fp prod = fe_one<ModP>();
  for (uint32_t e = 0; e < cnt; e++) {
    if (e) acc = jac_add_aff(acc, G);
    g1j_store(jtmp[i0 + e], acc);
    prod = prod * acc.z;
    for (int q = 0; q < 8; q++) zs[i0 + e][q] = prod.v[q];
  }
  fp inv = fp_inv(prod);
  for (int e = (int)cnt - 1; e >= 0; e--) {
    g1j pj = g1j_load(jtmp[i0 + e]);
    fp prev = e ? fe_const<ModP>(zs[i0 + e - 1]) : fe_one<ModP>();
    fp zi = inv * prev;
    inv = inv * pj.z;
    fp zi2 = zi * zi;
    g1a a;
    a.x = pj.x * zi2;
    a.y = pj.y * zi2 * zi;
    a.inf = false;
    G1Dev d;
    g1_store(d, a);
    pts[i0 + e] = d;
  }
}

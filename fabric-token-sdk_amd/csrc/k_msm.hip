// Kernels of the standalone G1 MSM (dev/msm.h): one lane per item.
#include <hip/hip_runtime.h>

#include "dev/msm.h"
#include "launch.h"

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

// one lane per point: sort keys + values of every window (dev/msm.h msm_job_keys)
__global__ void __launch_bounds__(256) k_msm_keys(MsmPlan p, const uint32_t (*scal)[8], uint32_t* key,
                                                  uint32_t* val) {
  LANE_PROLOGUE(p.n);
  msm_job_keys(p, i, scal, key, val);
}

// one lane per sorted entry: bucket ranges
__global__ void __launch_bounds__(256) k_msm_bounds(uint64_t total, const uint32_t* skey, uint32_t* start,
                                                    uint32_t* end) {
  uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  msm_job_bounds(t, total, skey, start, end);
}

// count[g] = end[g] - start[g] and the bucket's slot count
__global__ void __launch_bounds__(256) k_msm_counts(MsmPlan p, const uint32_t* start, const uint32_t* end,
                                                    uint32_t* count, uint32_t* m) {
  LANE_PROLOGUE(p.rw * p.buckets);
  uint32_t c = end[i] - start[i];
  count[i] = c;
  m[i] = msm_bucket_slots(p, c);
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

__global__ void __launch_bounds__(128) k_msm_segment(MsmPlan p, uint32_t w0, uint32_t w1, const uint32_t* wlo,
                                                     const uint32_t* whi, const uint32_t* owner,
                                                     const G1JDev* slot_sum, G1JDev* part) {
  uint32_t i = w0 * p.segs + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= w1 * p.segs) return;
  uint32_t w = i / p.segs, s = i - w * p.segs;
  g1j_store(part[i], msm_job_segment(p, w, s, wlo, whi, owner, slot_sum));
}

// tree sum of m consecutive parts per window in chunks of 256: out[w][ceil(m/256)]
// (carry-free form in LDS: one conversion in, one out)
__global__ void __launch_bounds__(256) k_msm_tree(const G1JDev* in, uint32_t m, G1JDev* out) {
  __shared__ j29 s[256];
  uint32_t chunks = (m + 255) / 256;
  uint32_t w = blockIdx.x / chunks, ch = blockIdx.x - w * chunks, t = threadIdx.x;
  uint32_t i = ch * 256 + t;
  s[t] = i < m ? j29_ld(in[(size_t)w * m + i]) : j29_inf();
  __syncthreads();
  for (uint32_t o = 128; o > 0; o >>= 1) {
    if (t < o) s[t] = j29_add(s[t], s[t + o]);
    __syncthreads();
  }
  if (t == 0) g1j_store(out[(size_t)w * chunks + ch], j29_to(s[0]));
}

// ---- 4-lane cooperative point arithmetic for the serial Horner chain.  A
// wave issues a one-lane Montgomery product at the cost of a 64-lane one, so
// the chain's latency is the number of dependent products: every lane holds
// the same point, lane k < 4 computes the k-th independent product of each
// dependency level, and the products are exchanged through LDS.
struct Coop {
  int k;
  uint32_t (*sh)[8];
  // one level: lane k computes a_k * b_k (k < cnt); returns all cnt products
  __device__ void level(int cnt, const fp* a, const fp* b, fp* out) const {
    fp x = a[0], y = b[0];
#pragma unroll
    for (int i = 1; i < 4; i++)
      if (i < cnt && k == i) {
        x = a[i];
        y = b[i];
      }
    fp r = x * y;
    if (k < cnt)
#pragma unroll
      for (int q = 0; q < 8; q++) sh[k][q] = r.v[q];
    __syncthreads();
    for (int i = 0; i < cnt; i++)
#pragma unroll
      for (int q = 0; q < 8; q++) out[i].v[q] = sh[i][q];
    __syncthreads();
  }
};

// dbl-2009-l (same values as jac_dbl): 3 product levels instead of 7 products
__device__ g1j coop_dbl(const Coop& c, const g1j& p) {
  fp o[4];
  {
    fp a[4] = {p.x, p.y, p.y, p.y}, b[4] = {p.x, p.y, p.z, p.z};
    c.level(3, a, b, o);
  }
  fp A = o[0], B = o[1], YZ = o[2];
  fp E = A + A + A, s = p.x + B;
  {
    fp a[4] = {B, s, E, E}, b[4] = {B, s, E, E};
    c.level(3, a, b, o);
  }
  fp C = o[0], D = o[1] - A - C;
  D = D + D;
  fp X3 = o[2] - D - D;
  {
    fp dx = D - X3;
    fp a[4] = {E, E, E, E}, b[4] = {dx, dx, dx, dx};
    c.level(1, a, b, o);
  }
  fp C8 = C + C;
  C8 = C8 + C8;
  C8 = C8 + C8;
  return {X3, o[0] - C8, YZ + YZ};
}

// add-2007-bl (same values as jac_add_inl): 6 product levels instead of 16 products
__device__ g1j coop_add(const Coop& c, const g1j& p, const g1j& q) {
  if (is_zero(p.z)) return q;
  if (is_zero(q.z)) return p;
  fp o[4];
  {
    fp a[4] = {p.z, q.z, p.z, p.z}, b[4] = {p.z, q.z, q.z, q.z};
    c.level(3, a, b, o);
  }
  fp Z1Z1 = o[0], Z2Z2 = o[1], Z1Z2 = o[2];
  {
    fp a[4] = {p.x, q.x, p.y, q.y}, b[4] = {Z2Z2, Z1Z1, q.z, p.z};
    c.level(4, a, b, o);
  }
  fp U1 = o[0], U2 = o[1];
  {
    fp a[4] = {o[2], o[3], o[2], o[2]}, b[4] = {Z2Z2, Z1Z1, Z2Z2, Z2Z2};
    c.level(2, a, b, o);
  }
  fp S1 = o[0];
  fp H = U2 - U1, rr = o[1] - S1;
  if (is_zero(H)) {
    if (is_zero(rr)) return coop_dbl(c, p);
    return jac_inf<fp>();
  }
  fp H2 = H + H;
  rr = rr + rr;
  {
    fp a[4] = {H2, rr, Z1Z2, Z1Z2}, b[4] = {H2, rr, H, H};
    c.level(3, a, b, o);
  }
  fp I = o[0], R2 = o[1], Zh = o[2];
  {
    fp a[4] = {H, U1, H, H}, b[4] = {I, I, I, I};
    c.level(2, a, b, o);
  }
  fp J = o[0], V = o[1];
  fp X3 = R2 - J - V - V;
  {
    fp vx = V - X3;
    fp a[4] = {rr, S1, rr, rr}, b[4] = {vx, J, vx, vx};
    c.level(2, a, b, o);
  }
  return {X3, o[0] - o[1] - o[1], Zh + Zh};
}

// Horner steps for reduction windows w_hi-1 down to w_lo: acc = 2^c acc + W_w,
// on one wave with the 4-lane cooperative point ops (measured: 0.55 ms at 2^20
// against 1.3 ms for one lane in the carry-free form -- four independent
// 32-bit products per level beat one carry-free chain); the last call (w_lo = 0)
// converts to affine (binary-EEA inverse) and gnark RawBytes.  With pre (one
// reduction window) this is the affine conversion alone.
__global__ void __launch_bounds__(64) k_msm_horner(MsmPlan p, uint32_t w_hi, uint32_t w_lo, const G1JDev* wsum,
                                                   G1JDev* acc_buf, G1Dev* res, uint8_t* bytes) {
  __shared__ uint32_t sh[4][8];
  if (blockIdx.x != 0) return;
  Coop c{(int)threadIdx.x, sh};
  g1j acc = w_hi == p.rw ? jac_inf<fp>() : g1j_load(*acc_buf);
  for (int w = (int)w_hi - 1; w >= (int)w_lo; w--) {
    if (w != (int)p.rw - 1)
      for (uint32_t q = 0; q < p.c; q++) acc = coop_dbl(c, acc);
    acc = coop_add(c, acc, g1j_load(wsum[w]));
  }
  if (threadIdx.x != 0) return;
  g1j_store(*acc_buf, acc);
  if (w_lo == 0) {
    g1a r;
    r.inf = is_zero(acc.z);
    fp zi = fp_inv_var(acc.z), zi2 = sqr(zi);
    r.x = r.inf ? fe_zero<ModP>() : acc.x * zi2;
    r.y = r.inf ? fe_zero<ModP>() : acc.y * zi2 * zi;
    G1Dev d;
    g1_store(d, r);
    *res = d;
    g1_to_bytes(bytes, r);
  }
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

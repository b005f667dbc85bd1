// Kernel translation unit (one per kernel family keeps hipcc builds parallel).
#include <hip/hip_runtime.h>

#include "dev/binv.h"
#include "dev/jobs.h"
#include "launch.h"

#ifndef FTS_G1PART_PRIO
#define FTS_G1PART_PRIO 0  // wave priority of k_g1_part (A/B)
#endif
#ifndef FTS_COMBINE_PRIO
#define FTS_COMBINE_PRIO FTS_BINV_PRIO  // wave priority of the block inversion's Euclid (dev/binv.h)
#endif

using namespace fts;

#define JOB_KERNEL_PROLOGUE(n)                          \
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; \
  if (i >= (n)) return;

// Uniform parts of the G1 jobs (fixed-base slots and GLV variable parts), one
// lane per part: lanes [f n, (f+1) n) all run the same code path.
__global__ void __launch_bounds__(128) k_g1_part(const G1Job* jobs, uint32_t n, const VTerm* vt, const G1Dev* pts,
                                                 const uint32_t (*scal)[8], const G1Dev* tab, G1JDev* part,
                                                 G1Dev* vtab) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 4 * n) return;
#if FTS_G1PART_PRIO
  __builtin_amdgcn_s_setprio(FTS_G1PART_PRIO);
#endif
  job_g1_part(jobs, n, i, vt, pts, scal, tab, part, vtab);
}

// Block-wide Montgomery batch inversion: thread t holds x_t (zero -> treated
// as 1); returns 1/x_t.  Prefix and suffix products by Hillis-Steele scans in
// LDS (2 log2(NT) products per thread), one field inversion per block done by
// wave 0 alone (a wave issues an inversion at the same cost for 1 lane as for
// 64, so inverting per lane costs every wave a full inversion).
template <int NT>
__device__ fp block_batch_inv(fp x, uint32_t (*pre)[NT], uint32_t (*suf)[NT], uint32_t* tot) {
  const int t = threadIdx.x;
  if (is_zero(x)) x = fe_one<ModP>();
  fp p = x, q = x;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    pre[k][t] = p.v[k];
    suf[k][t] = q.v[k];
  }
  __syncthreads();
#pragma nounroll
  for (int off = 1; off < NT; off <<= 1) {
    fp a = fe_one<ModP>(), b = fe_one<ModP>();
    if (t >= off)
#pragma unroll
      for (int k = 0; k < 8; k++) a.v[k] = pre[k][t - off];
    if (t + off < NT)
#pragma unroll
      for (int k = 0; k < 8; k++) b.v[k] = suf[k][t + off];
    __syncthreads();
    p = p * a;
    q = q * b;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      pre[k][t] = p.v[k];
      suf[k][t] = q.v[k];
    }
    __syncthreads();
  }
  if (t < 64) {  // wave 0 only
    fp all;
#pragma unroll
    for (int k = 0; k < 8; k++) all.v[k] = pre[k][NT - 1];
    __builtin_amdgcn_s_setprio(FTS_COMBINE_PRIO);  // the block waits on this wave
    fp ia = fp_inv_var(all);  // public values; one wave, one value: no divergence
    __builtin_amdgcn_s_setprio(0);
    if (t == 0)
#pragma unroll
      for (int k = 0; k < 8; k++) tot[k] = ia.v[k];
  }
  __syncthreads();
  fp r, a = fe_one<ModP>(), b = fe_one<ModP>();
#pragma unroll
  for (int k = 0; k < 8; k++) r.v[k] = tot[k];
  if (t > 0)
#pragma unroll
    for (int k = 0; k < 8; k++) a.v[k] = pre[k][t - 1];
  if (t + 1 < NT)
#pragma unroll
    for (int k = 0; k < 8; k++) b.v[k] = suf[k][t + 1];
  return r * a * b;
}

static constexpr int COMBINE_NT = 256;
// One batch inversion of Z Y per block gives both 1/Z (the affine result) and
// the normalised Miller evaluation point (x/y, 1/y) written to pnorm[out]
// (g1_pnorm; Y != 0 for every finite point of the prime-order G1).
__global__ void __launch_bounds__(COMBINE_NT) k_g1_combine(const G1Job* jobs, uint32_t n, const G1JDev* part,
                                                           G1Dev* g1out, uint8_t* arena, G1Dev* pnorm) {
  __shared__ uint32_t pre[8][COMBINE_NT], suf[8][COMBINE_NT], tot[8];
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  bool valid = i < n;  // every thread of the block takes part in the scans
  g1j acc = valid ? job_g1_sum_parts(jobs[i], i, n, part) : jac_inf<fp>();
  fp inv = block_batch_inv<COMBINE_NT>(acc.z * acc.y, pre, suf, tot);
  if (valid) {
    job_g1_finish(jobs[i], acc, acc.y * inv, g1out, arena);
    g1_pnorm(acc, inv, pnorm[jobs[i].out]);
  }
}

// ---- wide-window G1 tables (C = 16): per (base, window) the point
// B_w = 2^(C w) B, then every lane fills a chunk of consecutive digits by
// repeated mixed additions of B_w, made affine together (Montgomery batch
// inversion; jtmp / zs hold chunk * lanes Jacobian points / prefix products).
__global__ void __launch_bounds__(64) k_tab_g1_bw(const G1Dev* bases, uint32_t nb, G1Dev* bw) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb * (uint32_t)G1TAB_WINDOWS) return;
  uint32_t b = i / G1TAB_WINDOWS, w = i - b * G1TAB_WINDOWS;
  g1j acc = jac_from_aff(g1_load(bases[b]));
  for (uint32_t q = 0; q < (uint32_t)G1TAB_C * w; q++) acc = jac_dbl(acc);
  G1Dev d;
  g1_store(d, jac_to_aff(acc));
  bw[i] = d;
}

__global__ void __launch_bounds__(128) k_tab_g1_fill(const G1Dev* bw, uint32_t nb, uint32_t chunk, G1JDev* jtmp,
                                                     uint32_t (*zs)[8], G1Dev* tab) {
  uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x, per = G1TAB_DIGITS / chunk;
  if (lane >= nb * (uint32_t)G1TAB_WINDOWS * per) return;
  uint32_t t = lane / per, c = lane - t * per;
  size_t base = (size_t)t * G1TAB_DIGITS + (size_t)c * chunk;  // entry of |d| = c chunk + 1
  g1a B = g1_load(bw[t]);
  g1j acc = aff_mul_u64(B, (uint64_t)c * chunk + 1);
  fp prod = fe_one<ModP>();
  for (uint32_t e = 0; e < chunk; e++) {
    if (e) acc = jac_add_aff(acc, B);
    g1j_store(jtmp[base + e], acc);
    prod = prod * acc.z;
#pragma unroll
    for (int q = 0; q < 8; q++) zs[base + e][q] = prod.v[q];
  }
  fp inv = fp_inv_var(prod);
  for (int e = (int)chunk - 1; e >= 0; e--) {
    g1j pj = g1j_load(jtmp[base + e]);
    fp prev = e ? fe_const<ModP>(zs[base + e - 1]) : fe_one<ModP>();
    fp zi = inv * prev;
    inv = inv * pj.z;
    fp zi2 = sqr(zi);
    g1a a;
    a.x = pj.x * zi2;
    a.y = pj.y * zi2 * zi;
    a.inf = false;
    G1Dev d;
    g1_store(d, a);
    tab[base + e] = d;
  }
}

__global__ void __launch_bounds__(64) k_tab_g1(const G1Dev* bases, uint32_t n, G1Dev* tab) {
  JOB_KERNEL_PROLOGUE(n);
  job_tab_g1(i, bases, tab);
}

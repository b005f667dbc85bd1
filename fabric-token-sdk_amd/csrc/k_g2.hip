// Kernel translation unit (one per kernel family keeps hipcc builds parallel).
#include <hip/hip_runtime.h>

#include "dev/binv.h"
#include "dev/g2lines29.h"
#include "dev/g2x29.h"
#include "dev/jobs.h"
#include "launch.h"

using namespace fts;

#ifndef FTS_G2_PART_X29
#define FTS_G2_PART_X29 1
#endif
#ifndef FTS_G2_PART_WAVES
#define FTS_G2_PART_WAVES 1  // waves per SIMD k_g2_part is compiled for
#endif

#ifndef FTS_G2LINES_PRIO
#define FTS_G2LINES_PRIO 0  // wave priority of k_g2lines1 (A/B)
#endif

#define JOB_KERNEL_PROLOGUE(n)                          \
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; \
  if (i >= (n)) return;

__global__ void __launch_bounds__(128) k_g2(const G2Job* jobs, uint32_t n, const uint32_t (*scal)[8],
                                            const G2Dev* tab, G2Dev* g2out) {
  JOB_KERNEL_PROLOGUE(n);
  job_g2(jobs[i], scal, tab, g2out);
}

// t' of every membership job and its 88 Miller lines evaluated at R: sextet
// layout, 10 jobs per one-wave workgroup (sx_job_g2lines).
__global__ void __launch_bounds__(64, 2) k_g2lines(const G2Job* g2, const PairJob* pr, uint32_t n,
                                                   const uint32_t (*scal)[8], const G2Dev* tab, G2Dev* g2out,
                                                   const G1Dev* pts, EvLineDev* lines) {
  SX_SLOTS_DECL(SX_SLOTS_MILLER_F)
  SX_KERNEL_PROLOGUE(n);
  sx_job_g2lines(x, g2[jc], pr[jc], scal, tab, g2out, pts, lines, jc, n, valid);
}

// The same in the one-lane layout, split (job_g2_part / job_g2lines_parts):
// FTS_G2_PART_X29 (default 1) sums the parts in the carry-free XYZZ form
// (dev/g2x29.h), 0 in the 32-bit Jacobian one.
// four lanes per job sum the table points (part-major, so every wave runs one
// part), then one lane per job adds the partials and emits the lines.
__global__ void __launch_bounds__(64, FTS_G2_PART_WAVES) k_g2_part(const G2Job* g2, uint32_t n, const uint32_t (*scal)[8],
                                                const G2Dev* tab, G2PartDev* part) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 4 * n) return;
  uint32_t q = i / n, job = i - q * n;
#if FTS_G2_PART_X29
  job_g2_part_x29(g2[job], (int)q, scal, tab, part[i]);
#else
  job_g2_part(g2[job], (int)q, scal, tab, part[i]);
#endif
}
// FTS_G2_BINV (default 1): the partial sums added in k_g2_sum and the
// launch's inversions batched (k_g2_binv) before k_g2lines1, instead of one
// inversion per lane inside it (X29 line chain only)
__global__ void __launch_bounds__(64) k_g2_sum(uint32_t n, G2PartDev* part) {
  JOB_KERNEL_PROLOGUE(n);
  job_g2_sum(part, i, n);
}
__global__ void __launch_bounds__(256) k_g2_binv(uint32_t n, G2PartDev* part) {
  __shared__ uint32_t tree[512][8];
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  uint32_t* w = part[n + (j < n ? j : 0)].w;
  binv_tree256(
      tree, threadIdx.x, j < n,
      [&] {
        fp v;
#pragma unroll
        for (int q = 0; q < 8; q++) v.v[q] = w[q];
        return v;
      },
      [&](const fp& v) {
#pragma unroll
        for (int q = 0; q < 8; q++) w[q] = v.v[q];
      });
}
__global__ void __launch_bounds__(64) k_g2lines1(const G2Job* g2, const PairJob* pr, uint32_t n,
                                                 const G2PartDev* part, G2Dev* g2out, const G1Dev* pts,
                                                 EvLineDev* lines) {
  JOB_KERNEL_PROLOGUE(n);
#if FTS_G2LINES_PRIO
  __builtin_amdgcn_s_setprio(FTS_G2LINES_PRIO);
#endif
#if FTS_G2LINES_X29 && FTS_G2_BINV
  job_g2lines_summed_x29(g2[i], pr[i], part, g2out, pts, lines, i, n);
#elif FTS_G2LINES_X29
  job_g2lines_parts_x29(g2[i], pr[i], part, g2out, pts, lines, i, n);
#else
  job_g2lines_parts(g2[i], pr[i], part, g2out, pts, lines, i, n);
#endif
}

// ---- wide-window G2 tables (C > 8), as k_tab_g1_bw / k_tab_g1_fill
__global__ void __launch_bounds__(64) k_tab_g2_bw(const G2Dev* bases, G2Dev* bw) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint32_t)(G2B_COUNT * G2TAB_WINDOWS)) return;
  uint32_t b = i / G2TAB_WINDOWS, w = i - b * G2TAB_WINDOWS;
  g2j acc = jac_from_aff(g2_load(bases[b]));
  for (uint32_t q = 0; q < (uint32_t)G2TAB_C * w; q++) acc = jac_dbl(acc);
  G2Dev d;
  g2_store(d, jac_to_aff(acc));
  bw[i] = d;
}

struct G2JDev {
  uint32_t w[48];
};

__global__ void __launch_bounds__(128) k_tab_g2_fill(const G2Dev* bw, uint32_t chunk, uint32_t (*jt)[48],
                                                     uint32_t (*zs)[16], G2Dev* tab) {
  uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x, per = G2TAB_DIGITS / chunk;
  if (lane >= (uint32_t)(G2B_COUNT * G2TAB_WINDOWS) * per) return;
  uint32_t t = lane / per, c = lane - t * per;
  size_t base = (size_t)t * G2TAB_DIGITS + (size_t)c * chunk;
  g2a B = g2_load(bw[t]);
  g2j acc = aff_mul_u64(B, (uint64_t)c * chunk + 1);
  fp2 prod = f2_one();
  auto st = [](uint32_t* o, const fp2& a) {
#pragma unroll
    for (int q = 0; q < 8; q++) {
      o[q] = a.c0.v[q];
      o[8 + q] = a.c1.v[q];
    }
  };
  auto ld = [](const uint32_t* o) {
    fp2 a;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      a.c0.v[q] = o[q];
      a.c1.v[q] = o[8 + q];
    }
    return a;
  };
  for (uint32_t e = 0; e < chunk; e++) {
    if (e) acc = jac_add_aff(acc, B);
    st(jt[base + e], acc.x);
    st(jt[base + e] + 16, acc.y);
    st(jt[base + e] + 32, acc.z);
    prod = prod * acc.z;
    st(zs[base + e], prod);
  }
  fp2 inv = f2_inv(prod);
  for (int e = (int)chunk - 1; e >= 0; e--) {
    fp2 X = ld(jt[base + e]), Y = ld(jt[base + e] + 16), Z = ld(jt[base + e] + 32);
    fp2 prev = e ? ld(zs[base + e - 1]) : f2_one();
    fp2 zi = inv * prev;
    inv = inv * Z;
    fp2 zi2 = zi * zi;
    g2a a;
    a.x = X * zi2;
    a.y = Y * zi2 * zi;
    a.inf = false;
    G2Dev d;
    g2_store(d, a);
    tab[base + e] = d;
  }
}

__global__ void __launch_bounds__(64) k_tab_g2(const G2Dev* bases, uint32_t n, G2Dev* tab) {
  JOB_KERNEL_PROLOGUE(n);
  job_tab_g2(i, bases, tab);
}

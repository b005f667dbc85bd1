// Kernel translation unit (one per kernel family keeps hipcc builds parallel).
#include <hip/hip_runtime.h>

#include "dev/jobs.h"
#ifdef FTS_MILLER_KARA  // A/B builds: the Miller kernels' accumulation alone
#define FTS_SX_KARA FTS_MILLER_KARA
#endif
#include "dev/sx29.h"
#include "launch.h"

using namespace fts;

// 2-pair Miller loops (f-chain; pair 2's lines come evaluated from k_g2lines),
// sextet layout: 10 jobs per 64-lane wave (lanes 60..63 shadow the last sextet
// read-only), one wave per workgroup, carry-free accumulation (dev/sx29.h).
__global__ void __launch_bounds__(64, 2) k_miller(const PairJob* jobs, uint32_t n, const LineCoef29* qlines,
                                                  const EvLineDev* lines2, const G1Dev* g1out, F12Dev* fbuf) {
  SQ_KERNEL_PROLOGUE(n, SX_SLOTS_MILLER_F)
  const PairJob& j = jobs[jc];
  fp2 f = q2_to_fp2(sq_miller_f(x, qlines, g1_load(g1out[j.p1]), lines2, jc, n));
  if (valid) {
    uint32_t* o = &fbuf[jc].w[16 * sx_f12_index(x.k)];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      o[i] = f.c0.v[i];
      o[8 + i] = f.c1.v[i];
    }
  }
}

// The same with the fixed-Q lines normalised by r0 yP (sq_miller_fn): two
// limb-product pairs per lane instead of three for every fixed line.
__global__ void __launch_bounds__(64, 2) k_miller_n(const PairJob* jobs, uint32_t n, const LineCoef29* qlines_n,
                                                    const EvLineDev* lines2, const G1Dev* g1out, const G1Dev* pnorm,
                                                    F12Dev* fbuf) {
  SQ_KERNEL_PROLOGUE(n, SX_SLOTS_MILLER_F)
  const PairJob& j = jobs[jc];
  fp2 f = q2_to_fp2(sq_miller_fn(x, qlines_n, g1_load(g1out[j.p1]), pnorm[j.p1], lines2, jc, n));
  if (valid) {
    uint32_t* o = &fbuf[jc].w[16 * sx_f12_index(x.k)];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      o[i] = f.c0.v[i];
      o[8 + i] = f.c1.v[i];
    }
  }
}

// The prover's fixed-pair product f(C, Q) f(A, PK1) f(B, PK2) (sq_miller_f3n):
// p1 = C, p2 = A, p3 = B (g1out indices, normalised points in pnorm); pklines_n
// holds PK1's then PK2's normalised lines
__global__ void __launch_bounds__(64, 2) k_miller_f3(const PairJob* jobs, uint32_t n, const LineCoef29* qlines_n,
                                                     const LineCoef29* pklines_n, const G1Dev* g1out,
                                                     const G1Dev* pnorm, F12Dev* fbuf) {
  SQ_KERNEL_PROLOGUE(n, SX_SLOTS_MILLER_F)
  const PairJob& j = jobs[jc];
  fp2 f = q2_to_fp2(sq_miller_f3n(x, qlines_n, pklines_n, pklines_n + MILLER_LINES, pnorm[j.p1], pnorm[j.p2],
                                  pnorm[j.p3], g1_load(g1out[j.p1]).inf, g1_load(g1out[j.p2]).inf,
                                  g1_load(g1out[j.p3]).inf));
  if (valid) {
    uint32_t* o = &fbuf[jc].w[16 * sx_f12_index(x.k)];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      o[i] = f.c0.v[i];
      o[8 + i] = f.c1.v[i];
    }
  }
}

// the fixed Q's lines, in both forms (one lane), and normalised by r0 (r1/r0,
// r2/r0 in the r1, r2 slots; *norm = 0 if some r0 vanishes, then k_miller runs)
__global__ void k_qlines(const G2Dev* q, LineCoef* out, LineCoef29* out29, LineCoef29* out29n, int* n, int* norm) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    int m = precompute_lines(out, g2_load(*q));
    int ok = 1;
    for (int i = 0; i < m; i++) {
      out29[i] = linecoef29(out[i]);
      ok &= f2_is_zero(out[i].r0) ? 0 : 1;
      fp2 ri = f2_is_zero(out[i].r0) ? f2_one() : f2_inv(out[i].r0);
      LineCoef l = {f2_one(), out[i].r1 * ri, out[i].r2 * ri};
      out29n[i] = linecoef29(l);
    }
    *n = m;
    *norm = ok;
  }
}

// Kernel translation unit (one per kernel family keeps hipcc builds parallel).
#include <hip/hip_runtime.h>

#include "dev/jobs.h"
#include "dev/sx29.h"
#include "launch.h"

using namespace fts;

// Final exponentiations, sextet layout (see k_miller): k_fexp_exact computes
// f^((p^12-1)/r) (FTZ_FEXP_EXACT, the default), k_fexp the Fuentes-Castaneda
// multiple (FTZ_FEXP_FUENTES); the context's option picks the kernel.
//
// FTS_FEXP_F29 = 1 (default): the carry-free 29-bit accumulation of dev/sx29.h;
// 0: the 32-bit wide accumulation of dev/sextet.h.
#ifndef FTS_FEXP_F29
#define FTS_FEXP_F29 1
#endif

#if FTS_FEXP_F29
template <int EXACT, class X>
__device__ __forceinline__ void sq_job_fexp(const X& x, const PairJob& j, const F12Dev* fin, uint32_t idx,
                                            uint8_t* arena, bool valid) {
  const uint32_t* w = &fin[idx].w[16 * sx_f12_index(x.k)];
  fp2 f;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    f.c0.v[i] = w[i];
    f.c1.v[i] = w[8 + i];
  }
  fp2 g = EXACT ? sq_final_exp_exact(x, f) : sq_final_exp(x, f);
  if (valid) sx_gt_bytes(arena + j.bytes, x.k, g);
}
#endif

__global__ void __launch_bounds__(64, 2) k_fexp(const PairJob* jobs, uint32_t n, const F12Dev* fbuf,
                                             uint8_t* arena) {
#if FTS_FEXP_F29
  SQ_KERNEL_PROLOGUE(n, SX_SLOTS_FEXP)
  sq_job_fexp<0>(x, jobs[jc], fbuf, jc, arena, valid);
#else
  SX_SLOTS_DECL(SX_SLOTS_FEXP)
  SX_KERNEL_PROLOGUE(n);
  sx_job_fexp<0>(x, jobs[jc], fbuf, jc, arena, valid);
#endif
}

__global__ void __launch_bounds__(64, 2) k_fexp_exact(const PairJob* jobs, uint32_t n, const F12Dev* fbuf,
                                                   uint8_t* arena) {
#if FTS_FEXP_F29
  SQ_KERNEL_PROLOGUE(n, SX_SLOTS_FEXP)
  sq_job_fexp<1>(x, jobs[jc], fbuf, jc, arena, valid);
#else
  SX_SLOTS_DECL(SX_SLOTS_FEXP)
  SX_KERNEL_PROLOGUE(n);
  sx_job_fexp<1>(x, jobs[jc], fbuf, jc, arena, valid);
#endif
}

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
// FTS_FEXP_F29 = 1 (default): the carry-free 29-bit accumulation of dev/sx29.h,
// its Q2 slots aliasing the 32-bit slots of the one inversion; 0: dev/sextet.h.
#ifndef FTS_FEXP_F29
#define FTS_FEXP_F29 1
#endif

#if FTS_FEXP_F29
template <int EXACT, class X, class XO>
__device__ __forceinline__ void sq_job_fexp(const X& x, const XO& xo, const PairJob& j, const F12Dev* fin, uint32_t idx,
                            uint8_t* arena, bool valid) {
  const uint32_t* w = &fin[idx].w[16 * sx_f12_index(x.k)];
  fp2 f;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    f.c0.v[i] = w[i];
    f.c1.v[i] = w[8 + i];
  }
  fp2 g = EXACT ? sq_final_exp_exact(x, xo, f) : sq_final_exp(x, xo, f);
  if (valid) sx_gt_bytes(arena + j.bytes, x.k, g);
}
// q2 slots of a sextet, +16 bytes of padding (see SX_SLOTS_DECL)
#define SQ_FEXP_PROLOGUE(n)                                                   \
  static constexpr uint32_t sx_stride_ = SQ_FEXP_BYTES / 16 + 1;              \
  __shared__ uint4 sx_raw_[SX_JOBS_PER_WAVE * sx_stride_];                    \
  SX_KERNEL_PROLOGUE(n);                                                      \
  Sq<SyncWave> q{k_, (QSlotT*)(sx_raw_ + sx_ * sx_stride_), !ghost_, {}};
#endif

__global__ void __launch_bounds__(64, 2) k_fexp(const PairJob* jobs, uint32_t n, const F12Dev* fbuf,
                                             uint8_t* arena) {
#if FTS_FEXP_F29
  SQ_FEXP_PROLOGUE(n)
  sq_job_fexp<0>(q, x, jobs[jc], fbuf, jc, arena, valid);
#else
  SX_SLOTS_DECL(SX_SLOTS_FEXP)
  SX_KERNEL_PROLOGUE(n);
  sx_job_fexp<0>(x, jobs[jc], fbuf, jc, arena, valid);
#endif
}

__global__ void __launch_bounds__(64, 2) k_fexp_exact(const PairJob* jobs, uint32_t n, const F12Dev* fbuf,
                                                   uint8_t* arena) {
#if FTS_FEXP_F29
  SQ_FEXP_PROLOGUE(n)
  sq_job_fexp<1>(q, x, jobs[jc], fbuf, jc, arena, valid);
#else
  SX_SLOTS_DECL(SX_SLOTS_FEXP)
  SX_KERNEL_PROLOGUE(n);
  sx_job_fexp<1>(x, jobs[jc], fbuf, jc, arena, valid);
#endif
}

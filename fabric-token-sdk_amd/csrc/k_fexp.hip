// Kernel translation unit (one per kernel family keeps hipcc builds parallel).
#include <hip/hip_runtime.h>

#include "dev/binv.h"
#include "dev/jobs.h"
#include "dev/sx29.h"
#include "launch.h"

using namespace fts;

// Final exponentiations, sextet layout (see k_miller), carry-free 29-bit
// accumulation (dev/sx29.h).  FTZ_FEXP_EXACT (the default) computes
// f^((p^12-1)/r) in five launches -- k_fexp_easy, k_fexp_expt x 3, k_fexp_hard
// -- that hand m, m^x, m^(x^2), m^(x^3) over in the park planes (Park,
// fexp_park_bytes); FTZ_FEXP_FUENTES (the Fuentes-Castaneda multiple) in
// seven (the same easy and x-power kernels plus k_fexp_fc_*).  All launches of
// one pass use the same grid, so a lane's park index is the same in every
// phase.

#define FEXP_PARK Park pk{park, blockIdx.x * 64 + threadIdx.x, gridDim.x * 64, !ghost_};

__device__ __forceinline__ fp2 fexp_load(const F12Dev* fin, uint32_t idx, int k) {
  const uint32_t* w = &fin[idx].w[16 * sx_f12_index(k)];
  fp2 f;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    f.c0.v[i] = w[i];
    f.c1.v[i] = w[8 + i];
  }
  return f;
}

// phase 1: easy part, m -> park slot 0
__global__ void __launch_bounds__(64, 2) k_fexp_easy(uint32_t n, const F12Dev* fbuf, int32_t* park) {
  SQ_KERNEL_PROLOGUE(n, SX_SLOTS_FEXP)
  FEXP_PARK
  pk.put(0, sq_fexp_easy(x, fexp_load(fbuf, jc, x.k)));
}

// phase 1 in three launches (the device default): the easy part with the
// launch's Fp inversions batched (dev/sx29.h sq_fexp_easy_a / _b)
__global__ void __launch_bounds__(64, 2) k_fexp_easy_a(uint32_t n, const F12Dev* fbuf, int32_t* park) {
  SQ_KERNEL_PROLOGUE(n, SX_SLOTS_FEXP)
  FEXP_PARK
  sq_fexp_easy_a(x, fexp_load(fbuf, jc, x.k), pk, blockIdx.x * 64 + sx_ * 6);
}
__global__ void __launch_bounds__(64, 2) k_fexp_easy_b(uint32_t n, const F12Dev* fbuf, int32_t* park) {
  SQ_KERNEL_PROLOGUE(n, SX_SLOTS_FEXP)
  FEXP_PARK
  pk.put(0, sq_fexp_easy_b(x, fexp_load(fbuf, jc, x.k), pk, blockIdx.x * 64 + sx_ * 6));
}
// n^-1 for the n of every job of the launch (slot FEXP_EASY_N, lane 0 of the
// job's sextet; stride = the fexp launches' lane count), 256 jobs per
// workgroup (dev/binv.h); a zero n stays zero
__global__ void __launch_bounds__(256) k_fexp_binv(uint32_t n, int32_t* park, uint32_t stride) {
  __shared__ uint32_t tree[512][8];
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  const uint32_t lane0 = (j / SX_JOBS_PER_WAVE) * 64 + (j % SX_JOBS_PER_WAVE) * 6;
  const Park pk{park, 0, stride, true};
  binv_tree256(
      tree, threadIdx.x, j < n, [&] { return pk.get_fp(FEXP_EASY_N, lane0); },
      [&](const fp& v) { pk.put_fp(FEXP_EASY_N, lane0, v); });
}

// phase 2 (three launches): slot dst = (slot src)^x, a^3, a^5, a^7 parked
// from slot ps (a is re-read from src).  24 LDS slots (A, AX, B, BX): 17.4 KB
// per workgroup, so LDS admits the two waves per SIMD that the registers allow
// (the 30-slot region's 21.7 KB admitted 1.75).
#ifndef FTS_EXPT_SLOTS
#define FTS_EXPT_SLOTS 24
#endif
#if FTS_EXPT_SLOTS == 18
// 18 LDS slots (A, AX = B, BX: the multiplier republished after every
// squaring), 13 KB per workgroup: LDS admits three waves per SIMD, but the
// 168 VGPRs of three waves spill (164 B per lane) and the launch ran 4.02-4.06
// against 3.56-3.58 ms per 8192-proof pass (profiles/r05/expt_slots_ab.txt)
__global__ void __launch_bounds__(64, 3) k_fexp_expt(uint32_t n, int32_t* park, int src, int dst, int ps) {
  SQ_KERNEL_PROLOGUE_B(n, 18, 6)
#else
__global__ void __launch_bounds__(64, 2) k_fexp_expt(uint32_t n, int32_t* park, int src, int dst, int ps) {
  SQ_KERNEL_PROLOGUE_B(n, 24, 12)
#endif
  FEXP_PARK
  pk.put(dst, sq_expt(x, pk, src, ps));
}

// phase 3: hard part from slots 0..3 -> GT bytes in the membership transcript
__global__ void __launch_bounds__(64, 1) k_fexp_hard(const PairJob* jobs, uint32_t n, uint8_t* arena,
                                                  int32_t* park) {
  SQ_KERNEL_PROLOGUE(n, SX_SLOTS_FEXP)
  FEXP_PARK
  fp2 g = sq_fexp_hard_exact(x, pk);
  if (valid) sx_gt_bytes(arena + jobs[jc].bytes, x.k, g);
}

// Fuentes-Castaneda glue and hard part
__global__ void __launch_bounds__(64, 2) k_fexp_fc_mid1(uint32_t n, int32_t* park) {
  SQ_KERNEL_PROLOGUE(n, SX_SLOTS_FEXP)
  FEXP_PARK
  sq_fc_mid1(x, pk);
}
__global__ void __launch_bounds__(64, 2) k_fexp_fc_mid2(uint32_t n, int32_t* park) {
  SQ_KERNEL_PROLOGUE(n, SX_SLOTS_FEXP)
  FEXP_PARK
  sq_fc_mid2(x, pk);
}
__global__ void __launch_bounds__(64, 1) k_fexp_fc_hard(const PairJob* jobs, uint32_t n, uint8_t* arena,
                                                     int32_t* park) {
  SQ_KERNEL_PROLOGUE(n, SX_SLOTS_FEXP)
  FEXP_PARK
  fp2 g = sq_fc_hard(x, pk);
  if (valid) sx_gt_bytes(arena + jobs[jc].bytes, x.k, g);
}

// Kernel translation unit (one per kernel family keeps hipcc builds parallel).
#include <hip/hip_runtime.h>

#include "dev/jobs.h"
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

// the fixed Q's lines, in both forms (one lane)
__global__ void k_qlines(const G2Dev* q, LineCoef* out, LineCoef29* out29, int* n) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    int m = precompute_lines(out, g2_load(*q));
    for (int i = 0; i < m; i++) out29[i] = linecoef29(out[i]);
    *n = m;
  }
}

// Kernel translation unit (one per kernel family keeps hipcc builds parallel).
#include <hip/hip_runtime.h>

#include "dev/jobs.h"
#include "launch.h"

using namespace fts;

// 2-pair Miller loops, sextet layout: 10 jobs per 64-lane wave (lanes 60..63
// shadow the last sextet read-only), one wave per workgroup.
__global__ void __launch_bounds__(64, 2) k_miller(const PairJob* jobs, uint32_t n, const LineCoef* qlines,
                                                  const EvLineDev* lines2, const G1Dev* g1out, F12Dev* fbuf) {
  SX_SLOTS_DECL(SX_SLOTS_MILLER_F)
  SX_KERNEL_PROLOGUE(n);
  sx_job_miller(x, jobs[jc], qlines, lines2, g1out, fbuf, jc, n, valid);
}

__global__ void k_qlines(const G2Dev* q, LineCoef* out, int* n) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *n = precompute_lines(out, g2_load(*q));
}

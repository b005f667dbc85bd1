// Kernel translation unit (one per kernel family keeps hipcc builds parallel).
#include <hip/hip_runtime.h>

#include "dev/jobs.h"
#include "launch.h"

using namespace fts;

#define JOB_KERNEL_PROLOGUE(n)                          \
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; \
  if (i >= (n)) return;

__global__ void __launch_bounds__(64) k_miller(const PairJob* jobs, uint32_t n, const LineCoef* qlines,
                                               const G1Dev* g1out, const G1Dev* pts, const G2Dev* g2out,
                                               F12Dev* fbuf) {
  JOB_KERNEL_PROLOGUE(n);
  job_miller(jobs[i], qlines, g1out, pts, g2out, fbuf, i);
}

__global__ void k_qlines(const G2Dev* q, LineCoef* out, int* n) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *n = precompute_lines(out, g2_load(*q));
}

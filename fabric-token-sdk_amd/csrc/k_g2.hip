// Kernel translation unit (one per kernel family keeps hipcc builds parallel).
#include <hip/hip_runtime.h>

#include "dev/jobs.h"
#include "launch.h"

using namespace fts;

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

__global__ void __launch_bounds__(64) k_tab_g2(const G2Dev* bases, uint32_t n, G2Dev* tab) {
  JOB_KERNEL_PROLOGUE(n);
  job_tab_g2(i, bases, tab);
}

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

__global__ void __launch_bounds__(64) k_tab_g2(const G2Dev* bases, uint32_t n, G2Dev* tab) {
  JOB_KERNEL_PROLOGUE(n);
  job_tab_g2(i, bases, tab);
}

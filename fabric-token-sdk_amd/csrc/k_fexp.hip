// Kernel translation unit (one per kernel family keeps hipcc builds parallel).
#include <hip/hip_runtime.h>

#include "dev/jobs.h"
#include "launch.h"

using namespace fts;

#define JOB_KERNEL_PROLOGUE(n)                          \
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; \
  if (i >= (n)) return;

__global__ void __launch_bounds__(64) k_fexp(const PairJob* jobs, uint32_t n, const F12Dev* fbuf,
                                             uint8_t* arena) {
  JOB_KERNEL_PROLOGUE(n);
  job_fexp(jobs[i], fbuf, i, arena);
}

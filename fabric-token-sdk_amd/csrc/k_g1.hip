// Kernel translation unit (one per kernel family keeps hipcc builds parallel).
#include <hip/hip_runtime.h>

#include "dev/jobs.h"
#include "launch.h"

using namespace fts;

#define JOB_KERNEL_PROLOGUE(n)                          \
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; \
  if (i >= (n)) return;

__global__ void __launch_bounds__(128) k_g1(const G1Job* jobs, uint32_t n, const VTerm* vt, const G1Dev* pts,
                                            const uint32_t (*scal)[8], const G1Dev* tab, G1Dev* g1out,
                                            uint8_t* arena) {
  JOB_KERNEL_PROLOGUE(n);
  job_g1(jobs[i], vt, pts, scal, tab, g1out, arena);
}

// Uniform parts of the G1 jobs (fixed-base slots and GLV variable parts), one
// lane per part: lanes [f n, (f+1) n) all run the same code path.
__global__ void __launch_bounds__(128) k_g1_part(const G1Job* jobs, uint32_t n, const VTerm* vt, const G1Dev* pts,
                                                 const uint32_t (*scal)[8], const G1Dev* tab, G1JDev* part) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 4 * n) return;
  job_g1_part(jobs, n, i, vt, pts, scal, tab, part);
}

__global__ void __launch_bounds__(128) k_g1_combine(const G1Job* jobs, uint32_t n, const G1JDev* part,
                                                    G1Dev* g1out, uint8_t* arena) {
  JOB_KERNEL_PROLOGUE(n);
  job_g1_combine(jobs[i], i, n, part, g1out, arena);
}

__global__ void __launch_bounds__(64) k_tab_g1(const G1Dev* bases, uint32_t n, G1Dev* tab) {
  JOB_KERNEL_PROLOGUE(n);
  job_tab_g1(i, bases, tab);
}

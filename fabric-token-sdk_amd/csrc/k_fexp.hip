// Kernel translation unit (one per kernel family keeps hipcc builds parallel).
#include <hip/hip_runtime.h>

#include "dev/jobs.h"
#include "launch.h"

using namespace fts;

// Final exponentiations, sextet layout (see k_miller): k_fexp_exact computes
// f^((p^12-1)/r) (FTZ_FEXP_EXACT, the default), k_fexp the Fuentes-Castaneda
// multiple (FTZ_FEXP_FUENTES); the context's option picks the kernel.
__global__ void __launch_bounds__(64, 2) k_fexp(const PairJob* jobs, uint32_t n, const F12Dev* fbuf,
                                             uint8_t* arena) {
  SX_SLOTS_DECL(SX_SLOTS_FEXP)
  SX_KERNEL_PROLOGUE(n);
  sx_job_fexp<0>(x, jobs[jc], fbuf, jc, arena, valid);
}

__global__ void __launch_bounds__(64, 2) k_fexp_exact(const PairJob* jobs, uint32_t n, const F12Dev* fbuf,
                                                   uint8_t* arena) {
  SX_SLOTS_DECL(SX_SLOTS_FEXP)
  SX_KERNEL_PROLOGUE(n);
  sx_job_fexp<1>(x, jobs[jc], fbuf, jc, arena, valid);
}

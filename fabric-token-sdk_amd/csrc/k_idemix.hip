// Idemix owner-signature kernels (dev/idemix.h): one lane per NymSignature.
#include "launch.h"

__global__ void __launch_bounds__(64) k_nym(const NymJob* jobs, uint32_t n, uint8_t* blob, const QDev* tab,
                                            uint8_t* ok) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  ok[i] = job_nym(jobs[i], blob, tab);
}

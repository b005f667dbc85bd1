// Microbenchmark of the sextet Fp12 primitives (dev/sextet.h) in isolation:
// each sextet repeats one operation `iters` times on resident data.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../dev/jobs.h"
#include "../launch.h"

using namespace fts;

template <int OP>
__global__ void __launch_bounds__(64, 2) k_sxbench(const fp2* seed, fp2* out, int iters) {
  SX_SLOTS_DECL(SX_SLOTS_FEXP)
  uint32_t n = gridDim.x * SX_JOBS_PER_WAVE;
  SX_KERNEL_PROLOGUE(n);
  fp2 a = seed[(jc * 6 + k_) & 1023], b = seed[(jc * 6 + k_ + 7) & 1023];
  if (OP == 2) {
    if (k_ < 3) x.put(SX_L + k_, b);
    x.sync();
  }
#pragma nounroll
  for (int i = 0; i < iters; i++) {
    if (OP == 0) a = sx_mulv(x, a, b);
    if (OP == 1) a = sx_sqr(x, a);
    if (OP == 2) a = sx_mul_line(x, a, SX_L);
    if (OP == 3) a = sx_cyc_sqr(x, a);
    if (OP == 4) a = a * b;  // one reduced Fp2 product per lane (reference point)
  }
  if (valid) out[jc * 6 + k_] = a;
}

// returns sextet operations per second (op: 0 mul, 1 sqr, 2 mul_line, 3 cyc_sqr, 4 fp2 mul per lane)
extern "C" double ftz_sxbench(int device, int op, int blocks, int iters) {
  if (hipSetDevice(device) != hipSuccess) return -1;
  fp2 *seed, *out;
  if (hipMalloc(&seed, 1024 * sizeof(fp2)) != hipSuccess) return -1;
  if (hipMalloc(&out, (size_t)blocks * 64 * sizeof(fp2)) != hipSuccess) return -1;
  (void)hipMemset(seed, 0x11, 1024 * sizeof(fp2));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 2; rep++) {
    (void)hipEventRecord(e0);
    switch (op) {
      case 0: k_sxbench<0><<<blocks, 64>>>(seed, out, iters); break;
      case 1: k_sxbench<1><<<blocks, 64>>>(seed, out, iters); break;
      case 2: k_sxbench<2><<<blocks, 64>>>(seed, out, iters); break;
      case 3: k_sxbench<3><<<blocks, 64>>>(seed, out, iters); break;
      default: k_sxbench<4><<<blocks, 64>>>(seed, out, iters); break;
    }
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  (void)hipFree(seed);
  (void)hipFree(out);
  return (double)blocks * SX_JOBS_PER_WAVE * iters / (ms * 1e-3);
}

// Microbenchmark: Montgomery products/s vs independent chains per lane and
// waves per SIMD (design data for the lane-per-job vs lanes-per-job choice).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../dev/fp_wide.h"

using namespace fts;

template <int IMPL, int CH>
__global__ void __launch_bounds__(256) k_fpmicro(fp* io, int iters) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  fp x[CH];
  fp y = io[i + CH];
#pragma unroll
  for (int c = 0; c < CH; c++) x[c] = io[i + c];
#pragma nounroll
  for (int k = 0; k < iters; k++) {
#pragma unroll
    for (int c = 0; c < CH; c++) {
      if (IMPL == 0) {
        x[c] = mont_mul_cios(x[c], y);
      } else if (IMPL == 2) {
        uint32_t t[16];
        mul_wide(t, x[c].v, y.v);
        x[c] = redc_wide(t);
      } else {
#if defined(__HIP_DEVICE_COMPILE__)
        x[c] = mont_mul_fips(x[c], y);
#endif
      }
    }
  }
  fp s = x[0];
#pragma unroll
  for (int c = 1; c < CH; c++) s = s + x[c];
  io[i] = s;
}

template <int IMPL, int CH>
static float run(fp* io, int blocks, int threads, int iters) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  k_fpmicro<IMPL, CH><<<blocks, threads>>>(io, 4);
  (void)hipEventRecord(e0);
  k_fpmicro<IMPL, CH><<<blocks, threads>>>(io, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms;
}

// total_waves: waves in the grid (1024 = one per SIMD).  Returns products/s.
extern "C" double ftz_fpmicro(int device, int impl, int chains, int total_waves, int iters) {
  if (hipSetDevice(device) != hipSuccess) return -1;
  int threads = 64, blocks = total_waves;
  size_t n = (size_t)threads * blocks + 8;
  fp* io;
  if (hipMalloc(&io, n * sizeof(fp)) != hipSuccess) return -1;
  (void)hipMemset(io, 1, n * sizeof(fp));
  float ms = -1;
#define R(I, C) if (impl == I && chains == C) ms = run<I, C>(io, blocks, threads, iters);
  R(0, 1) R(0, 2) R(0, 4) R(1, 1) R(1, 2) R(1, 4) R(2, 1) R(2, 2) R(2, 4)
#undef R
  (void)hipFree(io);
  return (double)threads * blocks * chains * (double)iters / (ms * 1e-3);
}

// Integer-VALU roofline probe for gfx950: sustained rate of the
// u32 x u32 + u64 -> u64 multiply-add (v_mad_u64_u32) that every Montgomery
// product in dev/fp.h is built from.  8 independent accumulator chains per
// lane, enough waves to fill every SIMD.  Exposed as a C function for bench.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(256) k_madpeak(uint64_t* out, uint32_t iters, uint32_t seed) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t m[8];
  uint64_t acc[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    m[k] = (t + k) * 2654435761u + seed;
    acc[k] = (uint64_t)(t + k) * 0x100000001b3ull;
  }
  for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      // acc = m * hi(acc) + acc  -> exactly one v_mad_u64_u32 per step
      acc[k] = (uint64_t)m[k] * (uint32_t)(acc[k] >> 32) + acc[k];
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s ^= acc[k];
  out[t] = s;
}

// returns sustained MADs per second (wall time of one launch, after a warm-up)
extern "C" double ftz_madpeak(int device, uint32_t iters) {
  if (hipSetDevice(device) != hipSuccess) return -1;
  int blocks = 256 * 8 * 4, threads = 256;  // 8 waves per SIMD
  uint64_t* out;
  if (hipMalloc(&out, (size_t)blocks * threads * 8) != hipSuccess) return -1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  k_madpeak<<<blocks, threads>>>(out, iters / 8 + 1, 1);
  (void)hipEventRecord(e0);
  k_madpeak<<<blocks, threads>>>(out, iters, 2);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipFree(out);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return (double)blocks * threads * iters * 8 / (ms * 1e-3);
}

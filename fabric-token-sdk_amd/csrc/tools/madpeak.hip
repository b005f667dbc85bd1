// Integer-VALU ceilings for gfx950 (the roofline of every kernel on this path).
//
// ftz_madpeak: sustained rate of the u32 x u32 + u64 -> u64 multiply-add
// (v_mad_u64_u32) that the 32-bit Montgomery products in dev/fp.h are built
// from; 8 independent accumulator chains per lane, 8 waves per SIMD.
//
// ftz_valu_rate: sustained wave-instruction rate of one instruction stream
// (each loop body checked in the ISA to be exactly the named instructions), 8
// independent chains per lane, at a chosen number of waves per SIMD:
//   0 v_mad_u64_u32     1 v_mad_i64_i32 (the 29-bit code of dev/fp29.h, sx29.h)
//   2 v_add_co_u32 + v_addc_co_u32 pairs (32-bit carry chains)
//   3 v_lshl_add_u64 (64-bit add)       4 v_cndmask_b32     5 v_mov_b32
//   6 v_bfe_i32          7 v_ashrrev_i64    8 v_sub_co_u32 + v_subb_co_u32 pairs
//   9 the k_fexp_expt mix: per 16 instructions 9 v_mad_i64_i32, 2 v_lshl_add_u64,
//     1 v_bfe_i32, 1 v_ashrrev_i64, 1 sub/subb pair, 1 v_mov_b32
//  10 the 32-bit Montgomery mix (k_g1_part): per 8, 3 v_mad_u64_u32, 4 carry
//     adds (2 add_co/addc pairs), 1 v_cndmask_b32
// Returns wave-instructions per second over the whole chip.
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

// ---------------------------------------------------------------- streams
// C forms that compile to exactly the named instruction (checked in the ISA:
// hipcc pads inline-asm arithmetic with s_nop hazard guards the real kernels
// do not have); v_cndmask, v_mov and v_ashrrev_i64 in asm (their C forms fold away).
#define MADU(a, m) a = (uint64_t)(m) * (uint32_t)((a) >> 32) + (a)
#define MADI(a, m) a = (uint64_t)((int64_t)(int32_t)(m) * (int32_t)((a) >> 32) + (int64_t)(a))
#define ADDC(lo, hi, x)                      \
  {                                          \
    uint32_t c_;                             \
    lo = __builtin_addc(lo, x, 0u, &c_);     \
    hi = __builtin_addc(hi, x, c_, &c_);     \
  }
#define SUBB(lo, hi, x)                      \
  {                                          \
    uint32_t c_;                             \
    lo = __builtin_subc(lo, x, 0u, &c_);     \
    hi = __builtin_subc(hi, x, c_, &c_);     \
  }
#define ADD64(a, b) a = (a) + (b)
#define CND(a, b, s) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(s))
#define MOV(a, b) asm volatile("v_mov_b32 %0, %1" : "=v"(a) : "v"(b))
#define BFE(a) a = (uint32_t)((int32_t)((a) << 3) >> 8)
#define ASHR64(a) asm volatile("v_ashrrev_i64 %0, 29, %0" : "+v"(a))

// one loop iteration: 16 wave-instructions per chain group (8 chains x 2, or
// the mixes' 16), so every op is timed over the same instruction count
template <int OP>
__global__ void __launch_bounds__(256) k_valu(uint64_t* out, uint32_t iters, uint32_t seed) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t a[8];
  uint32_t m[8], lo[8], hi[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    m[k] = (t + k) * 2654435761u + seed;
    a[k] = (uint64_t)(t + k) * 0x100000001b3ull;
    lo[k] = (uint32_t)a[k];
    hi[k] = (uint32_t)(a[k] >> 32);
  }
  uint64_t smask = (uint64_t)seed * 0x9E3779B97F4A7C15ull;
  for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if (OP == 0) { MADU(a[k], m[k]); MADU(a[k], m[k]); }
      if (OP == 1) { MADI(a[k], m[k]); MADI(a[k], m[k]); }
      if (OP == 2) { ADDC(lo[k], hi[k], m[k]); }
      if (OP == 3) { ADD64(a[k], a[(k + 1) & 7]); ADD64(a[k], a[(k + 3) & 7]); }
      if (OP == 4) { CND(lo[k], m[k], smask); CND(hi[k], m[k], smask); }
      if (OP == 5) { MOV(lo[k], hi[k]); MOV(hi[k], lo[k]); }
      if (OP == 6) { BFE(lo[k]); BFE(hi[k]); }
      if (OP == 7) { ASHR64(a[k]); ASHR64(a[k]); }
      if (OP == 8) { SUBB(lo[k], hi[k], m[k]); }
    }
    if (OP == 9) {  // 2 x (9 MADI, 2 ADD64, 1 BFE, 1 ASHR64, 1 SUBB pair, 1 MOV) over the 8 chains
#pragma unroll
      for (int r = 0; r < 2; r++) {
#pragma unroll
        for (int k = 0; k < 8; k++) MADI(a[k], m[k]);
        MADI(a[r], m[r]);
        ADD64(a[2 + r], a[4 + r]);
        ADD64(a[6 + r], a[r]);
        BFE(lo[r]);
        ASHR64(a[4 + r]);
        SUBB(lo[2 + r], hi[2 + r], m[r]);
        MOV(lo[4 + r], hi[4 + r]);
      }
    }
    if (OP == 10) {  // 4 x (3 MADU, 2 ADDC pairs, 1 CND): 24 instructions
#pragma unroll
      for (int r = 0; r < 4; r++) {
        MADU(a[2 * r], m[r]);
        MADU(a[2 * r + 1], m[r + 4]);
        MADU(a[(2 * r + 2) & 7], m[r]);
        ADDC(lo[2 * r], hi[2 * r], m[r]);
        ADDC(lo[2 * r + 1], hi[2 * r + 1], m[r + 4]);
        CND(lo[(2 * r + 3) & 7], m[r], smask);
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s ^= a[k] ^ lo[k] ^ ((uint64_t)hi[k] << 32);
  out[t] = s;
}

// wave-instructions per loop iteration for each stream
static constexpr int VALU_PER_ITER[11] = {16, 16, 16, 16, 16, 16, 16, 16, 16, 32, 24};

template <int OP>
static void launch_valu(int blocks, uint64_t* out, uint32_t iters, uint32_t seed) {
  k_valu<OP><<<blocks, 256>>>(out, iters, seed);
}

extern "C" double ftz_valu_rate(int device, int op, int waves_per_simd, uint32_t iters) {
  if (op < 0 || op > 10 || waves_per_simd < 1 || waves_per_simd > 8) return -1;
  if (hipSetDevice(device) != hipSuccess) return -1;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return -1;
  int blocks = prop.multiProcessorCount * waves_per_simd;  // 256 threads = one wave per SIMD of a CU
  uint64_t* out;
  if (hipMalloc(&out, (size_t)blocks * 256 * 8) != hipSuccess) return -1;
  void (*fn)(int, uint64_t*, uint32_t, uint32_t) = nullptr;
  switch (op) {
    case 0: fn = launch_valu<0>; break;
    case 1: fn = launch_valu<1>; break;
    case 2: fn = launch_valu<2>; break;
    case 3: fn = launch_valu<3>; break;
    case 4: fn = launch_valu<4>; break;
    case 5: fn = launch_valu<5>; break;
    case 6: fn = launch_valu<6>; break;
    case 7: fn = launch_valu<7>; break;
    case 8: fn = launch_valu<8>; break;
    case 9: fn = launch_valu<9>; break;
    default: fn = launch_valu<10>; break;
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  fn(blocks, out, iters / 8 + 1, 1);
  (void)hipEventRecord(e0);
  fn(blocks, out, iters, 2);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipFree(out);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  double waves = (double)blocks * 4;
  return waves * iters * VALU_PER_ITER[op] / (ms * 1e-3);
}

// the shader clock the rates are read against (MHz; hipDeviceProp clockRate)
extern "C" int ftz_clock_mhz(int device) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return -1;
  return prop.clockRate / 1000;
}

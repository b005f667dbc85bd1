// Device self-check and microbenchmark of the two Montgomery multipliers
// (C CIOS vs inline-asm FIPS), used by tests/test_gpu.py and for tuning.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../dev/binv.h"
#include "../dev/fp.h"
#include "../dev/row29.h"

using namespace fts;

__device__ uint32_t xorshift(uint32_t& s) {
  s ^= s << 13;
  s ^= s >> 17;
  s ^= s << 5;
  return s;
}

template <class M>
__device__ Fe<M> rnd_fe(uint32_t& s) {
  Fe<M> x;
  for (int i = 0; i < 8; i++) x.v[i] = xorshift(s);
  x.v[7] &= 0x1FFFFFFFu;  // < 2^253 < m
  return x;
}

template <class M>
__global__ void k_fpcheck(uint32_t seed, uint32_t* bad) {
  uint32_t s = seed ^ (blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u;
  if (!s) s = 1;
  for (int it = 0; it < 64; it++) {
    Fe<M> a = rnd_fe<M>(s), b = rnd_fe<M>(s);
    if (it == 0) {  // edge: m-1 times m-1
      for (int i = 0; i < 8; i++) a.v[i] = M::m[i];
      a.v[0] -= 1;
      b = a;
    }
    Fe<M> x = mont_mul_cios(a, b);
#if defined(__HIP_DEVICE_COMPILE__)
    Fe<M> y = mont_mul_fips(a, b);
#else
    Fe<M> y = x;  // host pass only parses the kernel body
#endif
    if (!fe_eq(x, y)) atomicAdd(bad, 1u);
  }
}

template <int IMPL>
__global__ void k_fpbench(fp* io, int iters) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  fp x = io[i], y = io[i + 1];
  fp z = io[i + 2], w = io[i + 3];
#pragma nounroll
  for (int k = 0; k < iters; k++) {
    if (IMPL == 0) {
      x = mont_mul_cios(x, y);
      z = mont_mul_cios(z, w);
    } else {
#if defined(__HIP_DEVICE_COMPILE__)
      x = mont_mul_fips(x, y);
      z = mont_mul_fips(z, w);
#endif
    }
  }
  io[i] = x + z;
}

extern "C" int ftz_fpcheck(int device, uint32_t seed) {
  if (hipSetDevice(device) != hipSuccess) return -1;
  uint32_t* bad;
  if (hipMalloc(&bad, 8) != hipSuccess) return -1;
  (void)hipMemset(bad, 0, 8);
  k_fpcheck<ModP><<<256, 256>>>(seed, bad);
  k_fpcheck<ModR><<<256, 256>>>(seed + 1, bad + 1);
  uint32_t h[2] = {0, 0};
  (void)hipMemcpy(h, bad, 8, hipMemcpyDeviceToHost);
  (void)hipFree(bad);
  return (int)(h[0] + h[1]);
}

// returns Montgomery products per second for implementation impl (0 C, 1 asm)
extern "C" double ftz_fpbench(int device, int impl, int iters, int waves_per_simd) {
  if (hipSetDevice(device) != hipSuccess) return -1;
  int threads = 256, blocks = 256 * waves_per_simd;
  size_t n = (size_t)threads * blocks + 4;
  fp* io;
  if (hipMalloc(&io, n * sizeof(fp)) != hipSuccess) return -1;
  (void)hipMemset(io, 1, n * sizeof(fp));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 2; rep++) {
    (void)hipEventRecord(e0);
    if (impl == 0)
      k_fpbench<0><<<blocks, threads>>>(io, iters);
    else
      k_fpbench<1><<<blocks, threads>>>(io, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
  }
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipFree(io);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return 2.0 * threads * blocks * (double)iters / (ms * 1e-3);
}

// The batched inversion of dev/binv.h (k_fexp_binv, k_g2_binv) over 256-lane
// workgroups: n values, zero where zmask says so, lanes past n inactive (a
// partial last block), each output against the lane's own fp_inv_var.  Returns
// the number of mismatches (every active output and every untouched inactive
// slot checked), -1 on a HIP error.
__global__ void __launch_bounds__(256) k_binvcheck(uint32_t n, const uint8_t* zmask, uint32_t seed, fp* out,
                                                   uint32_t* bad) {
  __shared__ uint32_t tree[512][8];
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  uint32_t s = seed ^ (j + 1) * 2654435761u;
  if (!s) s = 1;
  fp v = rnd_fe<ModP>(s);
  if (j < n && zmask[j]) v = fe_zero<ModP>();
  binv_tree256(tree, threadIdx.x, j < n, [&] { return v; }, [&](const fp& r) { out[j] = r; });
  if (j >= n) return;
  const fp want = fe_is_zero(v) ? fe_zero<ModP>() : fp_inv_var(v);
  if (!fe_eq(out[j], want)) atomicAdd(bad, 1u);
}

extern "C" int ftz_binvcheck(int device, uint32_t n, const uint8_t* zmask, uint32_t seed) {
  if (hipSetDevice(device) != hipSuccess || n == 0) return -1;
  const uint32_t blocks = (n + 255) / 256;
  uint32_t* bad = nullptr;
  uint8_t* dz = nullptr;
  fp* out = nullptr;
  int rc = -1;
  if (hipMalloc(&bad, 4) == hipSuccess && hipMalloc(&dz, n) == hipSuccess &&
      hipMalloc(&out, sizeof(fp) * (size_t)blocks * 256) == hipSuccess &&
      hipMemset(bad, 0, 4) == hipSuccess && hipMemcpy(dz, zmask, n, hipMemcpyHostToDevice) == hipSuccess &&
      hipMemset(out, 0xA5, sizeof(fp) * (size_t)blocks * 256) == hipSuccess) {
    k_binvcheck<<<blocks, 256>>>(n, dz, seed, out, bad);
    uint32_t h = 0;
    std::vector<uint32_t> tail((size_t)(blocks * 256 - n) * 8);
    if (hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost) == hipSuccess &&
        (tail.empty() || hipMemcpy(tail.data(), out + n, tail.size() * 4, hipMemcpyDeviceToHost) == hipSuccess)) {
      for (uint32_t w : tail) h += w != 0xA5A5A5A5u;  // inactive lanes write nothing
      rc = (int)h;
    }
  }
  (void)hipFree(bad);
  (void)hipFree(dz);
  (void)hipFree(out);
  return rc;
}

// ---- dev/row29.h against dev/fp29.h: every row of every wave multiplies,
// normalises and reduces its own operands (limbs normalised, or signed within
// 2^29) row-wide, every lane the same one-lane, and lane r compares limb r.
__device__ f29 rnd_f29(uint32_t& s, bool sgn) {
  f29 a;
  for (int i = 0; i < 8; i++) {
    uint32_t x = xorshift(s) & (uint32_t)F29_MASK;
    a.l[i] = sgn ? (int32_t)(x >> 0) - (int32_t)(1u << 28) : (int32_t)x;
  }
  a.l[8] = (int32_t)(xorshift(s) & 0x3FFFFFu) - (sgn ? (1 << 21) : 0);
  return a;
}
__global__ void __launch_bounds__(64) k_rowcheck(uint32_t seed, uint32_t* bad) {
  const uint32_t r = row_lane(), q = row_index();
  uint32_t s = seed ^ ((blockIdx.x * 4 + q) + 1) * 2654435761u;
  if (!s) s = 1;
  for (int it = 0; it < 16; it++) {
    const bool sgn = (it & 1) != 0;
    const f29 a = rnd_f29(s, sgn), b = rnd_f29(s, sgn);
    const f29 want_m = f29_mul_c(a, b), want_n = f29_norm(f29_add(a, b)), want_r = f29_reduce(f29_sub(a, b));
    const r29 ra = row_from(a), rb = row_from(b);
    const r29 gm = row_mul(ra, rb), gn = row_norm(row_add(ra, rb)), gr = row_reduce(row_sub(ra, rb));
    int32_t wm = 0, wn = 0, wr = 0;
    for (int i = 0; i < 9; i++) {
      wm = r == (uint32_t)i ? want_m.l[i] : wm;
      wn = r == (uint32_t)i ? want_n.l[i] : wn;
      wr = r == (uint32_t)i ? want_r.l[i] : wr;
    }
    if (gm.v != wm || gn.v != wn || gr.v != wr) atomicAdd(bad, 1u);
    const bool z = row_is_zero(row_sub(ra, ra)), nz = row_is_zero(ra);
    if (!z || nz != f29_is_zero(a)) atomicAdd(bad + 1, 1u);
    // four different products at once through row_level (operands common to
    // the wave's rows, as in the Horner chain: row 0's here), against the one-lane ones
    f29 c0 = a, c1 = b;
    for (int i = 0; i < 9; i++) {
      c0.l[i] = __builtin_amdgcn_readlane(a.l[i], 0);
      c1.l[i] = __builtin_amdgcn_readlane(b.l[i], 0);
    }
    const f29 cm = f29_mul_c(c0, c1), cn = f29_norm(f29_add(c0, c1));
    const r29 r0 = row_from(c0), r1 = row_from(c1), rm = row_from(cm), rn = row_from(cn);
    r29 xa[4] = {r0, r1, rm, rn}, xb[4] = {r1, rm, rn, r0}, o[4];
    row_level<4>(xa, xb, o);
    const f29 fa[4] = {c0, c1, cm, cn}, fb[4] = {c1, cm, cn, c0};
    for (int k = 0; k < 4; k++) {
      const f29 w = f29_mul_c(fa[k], fb[k]);
      int32_t wk = 0;
      for (int i = 0; i < 9; i++) wk = r == (uint32_t)i ? w.l[i] : wk;
      if (o[k].v != wk) atomicAdd(bad + 2, 1u);
    }
  }
}

extern "C" int ftz_rowcheck(int device, uint32_t seed, uint32_t* out3) {
  if (hipSetDevice(device) != hipSuccess) return -1;
  uint32_t* bad;
  if (hipMalloc(&bad, 12) != hipSuccess) return -1;
  (void)hipMemset(bad, 0, 12);
  k_rowcheck<<<1024, 64>>>(seed, bad);
  uint32_t h[3] = {0, 0, 0};
  hipError_t e = hipMemcpy(h, bad, 12, hipMemcpyDeviceToHost);
  (void)hipFree(bad);
  if (e != hipSuccess) return -1;
  for (int k = 0; k < 3; k++) out3[k] = h[k];
  return (int)(h[0] + h[1] + h[2]);
}

// one wave, a chain of n dependent products: row-wide (impl 1) or one-lane
// f29_mul_c (impl 0); returns GPU clock cycles per product
__global__ void __launch_bounds__(64) k_rowbench(int impl, int n, int32_t* io, uint64_t* cyc) {
  f29 a, b;
  for (int i = 0; i < 9; i++) {
    a.l[i] = io[i] & F29_MASK;
    b.l[i] = io[9 + i] & F29_MASK;
  }
  a.l[8] &= 0xFFFF;
  b.l[8] &= 0xFFFF;
  const uint64_t t0 = __builtin_readcyclecounter();
  if (impl == 1) {
    r29 x = row_from(a), y = row_from(b);
    for (int k = 0; k < n; k++) x = row_mul(x, y);
    a = row_to(x);
  } else {
    for (int k = 0; k < n; k++) a = f29_mul_c(a, b);
  }
  const uint64_t t1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) {
    for (int i = 0; i < 9; i++) io[18 + i] = a.l[i];
    *cyc = (t1 - t0) / (uint64_t)n;
  }
}

extern "C" long ftz_rowbench(int device, int impl, int n) {
  if (hipSetDevice(device) != hipSuccess) return -1;
  int32_t* io;
  uint64_t* cyc;
  if (hipMalloc(&io, 27 * 4) != hipSuccess || hipMalloc(&cyc, 8) != hipSuccess) return -1;
  int32_t h[27];
  for (int i = 0; i < 27; i++) h[i] = 123456789 * (i + 1);
  (void)hipMemcpy(io, h, sizeof h, hipMemcpyHostToDevice);
  k_rowbench<<<1, 64>>>(impl, n, io, cyc);
  uint64_t c = 0;
  hipError_t e = hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  (void)hipFree(io);
  (void)hipFree(cyc);
  return e == hipSuccess ? (long)c : -1;
}

// ---- dev/safegcd.h (fp_inv_var) against the binary Euclid (fp_inv_eea): one
// random Montgomery element per lane plus the edge values 1, 2, p - 1 in the
// first lanes; inverse * value must also be one.  Returns the mismatches.
__global__ void __launch_bounds__(256) k_invcheck(uint32_t seed, uint32_t* bad) {
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  uint32_t s = seed ^ (j + 1) * 2654435761u;
  if (!s) s = 1;
  fp v = rnd_fe<ModP>(s);
  if (j < 3) {
    uint32_t k[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (j < 2) {
      k[0] = j + 1;
    } else {
      for (int i = 0; i < 8; i++) k[i] = P_MOD[i];
      k[0] -= 1;
    }
    v = fe_from_int<ModP>(k);
  }
  const fp a = fp_inv_sg<30>(v), a2 = fp_inv_sg<62>(v), b = fp_inv_eea(v);
  if (!fe_eq(a, b) || !fe_eq(a2, b) || !fe_eq(a * v, fe_one<ModP>()) || !fe_eq(fp_inv_var(v), b))
    atomicAdd(bad, 1u);
}

extern "C" int ftz_invcheck(int device, uint32_t blocks, uint32_t seed) {
  if (hipSetDevice(device) != hipSuccess || blocks == 0) return -1;
  uint32_t* bad = nullptr;
  int rc = -1;
  if (hipMalloc(&bad, 4) == hipSuccess && hipMemset(bad, 0, 4) == hipSuccess) {
    k_invcheck<<<blocks, 256>>>(seed, bad);
    uint32_t h = 0;
    if (hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost) == hipSuccess) rc = (int)h;
  }
  (void)hipFree(bad);
  return rc;
}

// one lane, a chain of n dependent inversions: divsteps on 30-bit limbs (impl
// 2), on 62-bit limbs (impl 1) or the binary Euclid (impl 0); returns GPU clock
// cycles per inversion
__global__ void __launch_bounds__(64) k_invbench(int impl, int n, fp* io, uint64_t* cyc) {
  if (threadIdx.x != 0) return;
  fp a = io[0];
  const fp one = fe_one<ModP>();
  const uint64_t t0 = __builtin_readcyclecounter();
  for (int k = 0; k < n; k++)
    a = (impl == 2 ? fp_inv_sg<30>(a) : impl == 1 ? fp_inv_sg<62>(a) : fp_inv_eea(a)) + one;
  const uint64_t t1 = __builtin_readcyclecounter();
  io[1] = a;
  *cyc = (t1 - t0) / (uint64_t)n;
}

extern "C" long ftz_invbench(int device, int impl, int n) {
  if (hipSetDevice(device) != hipSuccess) return -1;
  fp* io;
  uint64_t* cyc;
  if (hipMalloc(&io, 2 * sizeof(fp)) != hipSuccess || hipMalloc(&cyc, 8) != hipSuccess) return -1;
  uint32_t s = 12345;
  fp h[2];
  for (int i = 0; i < 8; i++) h[0].v[i] = 0;
  h[0].v[0] = 7;
  (void)s;
  (void)hipMemcpy(io, h, sizeof h, hipMemcpyHostToDevice);
  k_invbench<<<1, 64>>>(impl, n, io, cyc);
  uint64_t c = 0;
  hipError_t e = hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  (void)hipFree(io);
  (void)hipFree(cyc);
  return e == hipSuccess ? (long)c : -1;
}

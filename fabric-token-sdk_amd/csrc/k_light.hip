// Kernel translation unit (one per kernel family keeps hipcc builds parallel).
#include <hip/hip_runtime.h>

#include "dev/jobs.h"
#include "launch.h"

using namespace fts;

#define JOB_KERNEL_PROLOGUE(n)                          \
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; \
  if (i >= (n)) return;

__global__ void __launch_bounds__(256) k_decode(const DecodeJob* jobs, uint32_t n, const uint8_t* wire,
                                                G1Dev* pts, uint8_t* pt_ok, uint8_t* arena) {
  JOB_KERNEL_PROLOGUE(n);
  DecodeJob j = jobs[i];
  pt_ok[j.out] = job_decode(j, wire, pts, arena);
}

__global__ void __launch_bounds__(256) k_zr(const ZrJob* jobs, uint32_t n, const uint8_t* wire,
                                            uint32_t (*scal)[8], uint8_t* canon) {
  JOB_KERNEL_PROLOGUE(n);
  job_zr(jobs[i], wire, scal, canon);
}

__global__ void __launch_bounds__(256) k_scalar(const ScalJob* jobs, uint32_t n, uint32_t (*scal)[8],
                                                const uint32_t* list) {
  JOB_KERNEL_PROLOGUE(n);
  job_scalar(jobs[i], scal, list);
}

__global__ void __launch_bounds__(128) k_hash(const HashJob* jobs, uint32_t n, const Seg* segs,
                                              const uint8_t* arena, uint32_t (*scal)[8],
                                              const uint8_t* canon, uint8_t* ok) {
  JOB_KERNEL_PROLOGUE(n);
  ok[i] = job_hash(jobs[i], segs, arena, scal, canon);
}

__global__ void __launch_bounds__(256) k_verdict(const TxChecks* tx, uint32_t n, const Check* ck,
                                                 const uint8_t* pt_ok, const uint8_t* hash_ok, int32_t* codes,
                                                 uint32_t* bitmap) {
  JOB_KERNEL_PROLOGUE(n);
  int32_t c = job_verdict(tx[i], ck, pt_ok, hash_ok);
  codes[i] = c;
  if (c == E_OK) atomicOr(&bitmap[i >> 5], 1u << (i & 31));
}

// ---- prover
__global__ void __launch_bounds__(128) k_rand(const RandJob* jobs, uint32_t n, const uint8_t* arena,
                                              uint32_t (*scal)[8]) {
  JOB_KERNEL_PROLOGUE(n);
  job_rand(jobs[i], arena, scal);
}

__global__ void __launch_bounds__(256) k_emit(const EmitJob* jobs, uint32_t n, const uint32_t (*scal)[8],
                                              uint8_t* arena) {
  JOB_KERNEL_PROLOGUE(n);
  job_emit(jobs[i], scal, arena);
}

// one workgroup per copy job (the prover's device-initialised arena / output
// pools, dev/jobs.h CopyJob): lanes stride over its bytes
__global__ void __launch_bounds__(64) k_copy(const CopyJob* jobs, uint32_t n, const uint8_t* wire, uint8_t* arena,
                                             uint8_t* out) {
  if (blockIdx.x >= n) return;
  CopyJob j = jobs[blockIdx.x];
  for (uint32_t b = threadIdx.x; b < j.len; b += blockDim.x) job_copy_byte(j, b, wire, arena, out);
}

// one workgroup per inner document: threads stride over its 3-byte groups
__global__ void __launch_bounds__(256) k_b64(const B64Job* jobs, uint32_t n, const uint8_t* arena, uint8_t* out) {
  if (blockIdx.x >= n) return;
  B64Job j = jobs[blockIdx.x];
  uint32_t groups = (j.len + 2) / 3;
  for (uint32_t g = threadIdx.x; g < groups; g += blockDim.x) b64_group(out + j.dst + 4 * g, arena + j.src, j.len, g);
}

// context construction

__global__ void k_pp_decode(const uint8_t* raw, const uint32_t* g1off, uint32_t n1, const uint32_t* g2off,
                            uint32_t n2, G1Dev* g1, G2Dev* g2, uint8_t* g1bytes, uint8_t* g2bytes, uint8_t* ok) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n1) {
    DecodeJob j;
    j.raw = g1off[i];
    j.len = 64;
    j.out = i;
    j.bytes = NONE;
    j.b64 = NONE;
    ok[i] = job_decode(j, raw, g1, nullptr);
    g1a a = g1_load(g1[i]);
    g1_to_bytes(g1bytes + 64 * i, a);
  } else if (i < n1 + n2) {
    uint32_t k = i - n1;
    ok[i] = decode_g2(raw + g2off[k], 128, g2[k], g2bytes + 128 * k);
  }
}

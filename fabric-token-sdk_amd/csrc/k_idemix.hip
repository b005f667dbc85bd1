// Idemix owner-signature kernels (dev/idemix.h), one set per idemix curve
// (FP256BN_AMCL: fq, BN254: fp): k_nym_part runs the four parts of
// t = s_sk HSk + s_rnym HRand - c Nym on four lanes per signature (part-major:
// lanes [p n, (p+1) n) run part p, so every wave runs one part), k_nym_fin adds
// them and hashes the transcript, one lane per signature.
#include "launch.h"

template <class F>
__device__ __forceinline__ void nym_part(const NymJob* jobs, uint32_t n, const uint8_t* blob, const QDev* tab,
                                         QJDev* part) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 4 * n) return;
  uint32_t p = i / n, j = i - p * n;
  qj_store(part[i], job_nym_part<F>(jobs[j], blob, tab, p));
}

template <class F>
__device__ __forceinline__ void nym_fin(const NymJob* jobs, uint32_t n, uint8_t* blob, const QJDev* part,
                                        uint8_t* ok) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Jac<F> t = jac_add(jac_add(qj_load<F>(part[i]), qj_load<F>(part[n + i])),
                     jac_add(qj_load<F>(part[2 * n + i]), qj_load<F>(part[3 * n + i])));
  ok[i] = job_nym_fin<F>(jobs[i], blob, t);
}

__global__ void __launch_bounds__(64) k_nym_part(const NymJob* jobs, uint32_t n, const uint8_t* blob,
                                                 const QDev* tab, QJDev* part) {
  nym_part<fq>(jobs, n, blob, tab, part);
}
__global__ void __launch_bounds__(64) k_nym_fin(const NymJob* jobs, uint32_t n, uint8_t* blob, const QJDev* part,
                                                uint8_t* ok) {
  nym_fin<fq>(jobs, n, blob, part, ok);
}
__global__ void __launch_bounds__(64) k_nym_part_bn(const NymJob* jobs, uint32_t n, const uint8_t* blob,
                                                    const QDev* tab, QJDev* part) {
  nym_part<fp>(jobs, n, blob, tab, part);
}
__global__ void __launch_bounds__(64) k_nym_fin_bn(const NymJob* jobs, uint32_t n, uint8_t* blob,
                                                   const QJDev* part, uint8_t* ok) {
  nym_fin<fp>(jobs, n, blob, part, ok);
}

// Auditor owner match (dev/idemix.h job_eid): one lane per token
__global__ void __launch_bounds__(64) k_eid(const uint8_t* in, uint32_t n, const QDev* tab, uint8_t* ok) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  ok[i] = job_eid<fq>(in + (size_t)i * EID_JOB_BYTES, tab);
}
__global__ void __launch_bounds__(64) k_eid_bn(const uint8_t* in, uint32_t n, const QDev* tab, uint8_t* ok) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  ok[i] = job_eid<fp>(in + (size_t)i * EID_JOB_BYTES, tab);
}

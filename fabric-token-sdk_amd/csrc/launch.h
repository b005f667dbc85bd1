// Kernel declarations (definitions live in k_*.hip, one TU per kernel family,
// so the heavy pairing TUs compile in parallel).
#pragma once
#include <hip/hip_runtime.h>

#include "dev/jobs.h"
#include "dev/msm.h"
#include "dev/idemix.h"
#include "dev/sx29.h"

using namespace fts;

// Sextet kernels (dev/sextet.h): 10 jobs per one-wave workgroup.
static constexpr uint32_t SX_JOBS_PER_WAVE = 10;
struct SyncWave {
  __device__ __forceinline__ void operator()() const { __syncthreads(); }
};
// LDS of the sextets of one workgroup: region i holds sextet i's NS slots plus
// 16 bytes of padding, so the regions of the sextets that share a ds_read_b128
// lane group start on different 16-byte bank slots (64 B slots and 1152 / 1920 B
// regions would put them on the same banks: 3-way conflicts measured by
// SQ_LDS_BANK_CONFLICT; the padded layout is conflict-free for broadcast reads).
#define SX_SLOTS_DECL(NS)                                                          \
  static constexpr uint32_t sx_stride_ = (NS) * (sizeof(F2Slot) / 16) + 1;          \
  __shared__ uint4 sx_raw_[SX_JOBS_PER_WAVE * sx_stride_];
// Lane -> (sextet, role); lanes 60..63 are ghosts that shadow sextet 9 without
// writing its slots.  Every lane runs the whole program (barriers inside).
#define SX_KERNEL_PROLOGUE(n)                                           \
  uint32_t lane_ = threadIdx.x, sx_ = lane_ / 6;                        \
  bool ghost_ = sx_ >= SX_JOBS_PER_WAVE;                                \
  int k_ = ghost_ ? (int)(lane_ - 6 * SX_JOBS_PER_WAVE) : (int)(lane_ - 6 * sx_); \
  if (ghost_) sx_ = SX_JOBS_PER_WAVE - 1;                               \
  uint32_t job_ = blockIdx.x * SX_JOBS_PER_WAVE + sx_;                  \
  bool valid = !ghost_ && job_ < (n);                                   \
  uint32_t jc = job_ < (n) ? job_ : (n) - 1;                            \
  Sx<SyncWave> x{k_, (SlotT*)(sx_raw_ + sx_ * sx_stride_), !ghost_, {}};

// The same for the carry-free sextet kernels (dev/sx29.h): NS Q2 slots per
// sextet in a region of sq_region_dwords(NS) dwords.
#define SQ_KERNEL_PROLOGUE(n, NS) SQ_KERNEL_PROLOGUE_B(n, NS, SX_B)
#define SQ_KERNEL_PROLOGUE_B(n, NS, BOFS)                                         \
  static constexpr uint32_t sq_stride_ = sq_region_dwords(NS) / 2;               \
  __shared__ uint2 sq_raw_[SX_JOBS_PER_WAVE * sq_stride_];                       \
  uint32_t lane_ = threadIdx.x, sx_ = lane_ / 6;                                 \
  bool ghost_ = sx_ >= SX_JOBS_PER_WAVE;                                         \
  int k_ = ghost_ ? (int)(lane_ - 6 * SX_JOBS_PER_WAVE) : (int)(lane_ - 6 * sx_); \
  if (ghost_) sx_ = SX_JOBS_PER_WAVE - 1;                                        \
  uint32_t job_ = blockIdx.x * SX_JOBS_PER_WAVE + sx_;                           \
  bool valid = !ghost_ && job_ < (n);                                            \
  uint32_t jc = job_ < (n) ? job_ : (n) - 1;                                     \
  Sq<SyncWave, BOFS> x{k_, (QSlotT*)(sq_raw_ + sx_ * sq_stride_), !ghost_, {}};

__global__ void k_decode(const DecodeJob* jobs, uint32_t n, const uint8_t* wire, G1Dev* pts, uint8_t* pt_ok,
                         uint8_t* arena);
__global__ void k_zr(const ZrJob* jobs, uint32_t n, const uint8_t* wire, uint32_t (*scal)[8], uint8_t* canon);
__global__ void k_scalar(const ScalJob* jobs, uint32_t n, uint32_t (*scal)[8], const uint32_t* list);
__global__ void k_hash(const HashJob* jobs, uint32_t n, const Seg* segs, const uint8_t* arena, uint32_t (*scal)[8],
                       const uint8_t* canon, uint8_t* ok);
__global__ void k_verdict(const TxChecks* tx, uint32_t n, const Check* ck, const uint8_t* pt_ok,
                          const uint8_t* hash_ok, int32_t* codes, uint32_t* bitmap);
__global__ void k_pp_decode(const uint8_t* raw, const uint32_t* g1off, uint32_t n1, const uint32_t* g2off,
                            uint32_t n2, G1Dev* g1, G2Dev* g2, uint8_t* g1bytes, uint8_t* g2bytes, uint8_t* ok);
__global__ void k_g1_part(const G1Job* jobs, uint32_t n, const VTerm* vt, const G1Dev* pts,
                          const uint32_t (*scal)[8], const G1Dev* tab, G1JDev* part, G1Dev* vtab);
__global__ void k_g1_combine(const G1Job* jobs, uint32_t n, const G1JDev* part, G1Dev* g1out, uint8_t* arena,
                             G1Dev* pnorm);
__global__ void k_tab_g1(const G1Dev* bases, uint32_t n, G1Dev* tab);
__global__ void k_tab_g1_bw(const G1Dev* bases, uint32_t nb, G1Dev* bw);
__global__ void k_tab_g1_fill(const G1Dev* bw, uint32_t nb, uint32_t chunk, G1JDev* jtmp, uint32_t (*zs)[8], G1Dev* tab);
__global__ void k_g2(const G2Job* jobs, uint32_t n, const uint32_t (*scal)[8], const G2Dev* tab, G2Dev* g2out);
__global__ void k_g2lines(const G2Job* g2, const PairJob* pr, uint32_t n, const uint32_t (*scal)[8], const G2Dev* tab,
                          G2Dev* g2out, const G1Dev* pts, EvLineDev* lines);
__global__ void k_g2_part(const G2Job* g2, uint32_t n, const uint32_t (*scal)[8], const G2Dev* tab, G2PartDev* part);
#ifndef FTS_G2LINES_X29
#define FTS_G2LINES_X29 1  // k_g2lines1's line chain on the carry-free form (dev/g2lines29.h)
#endif
#ifndef FTS_G2_BINV
#define FTS_G2_BINV 1  // k_g2_sum + k_g2_binv before k_g2lines1 (k_g2.hip)
#endif
__global__ void k_g2_sum(uint32_t n, G2PartDev* part);
__global__ void k_g2_binv(uint32_t n, G2PartDev* part);
__global__ void k_g2lines1(const G2Job* g2, const PairJob* pr, uint32_t n, const G2PartDev* part, G2Dev* g2out,
                           const G1Dev* pts, EvLineDev* lines);
__global__ void k_tab_g2(const G2Dev* bases, uint32_t n, G2Dev* tab);
__global__ void k_tab_g2_bw(const G2Dev* bases, G2Dev* bw);
__global__ void k_tab_g2_fill(const G2Dev* bw, uint32_t chunk, uint32_t (*jt)[48], uint32_t (*zs)[16], G2Dev* tab);
__global__ void k_miller(const PairJob* jobs, uint32_t n, const LineCoef29* qlines, const EvLineDev* lines2,
                         const G1Dev* g1out, F12Dev* fbuf);
__global__ void k_qlines(const G2Dev* q, LineCoef* out, LineCoef29* out29, LineCoef29* out29n, int* n, int* norm);
__global__ void k_miller_n(const PairJob* jobs, uint32_t n, const LineCoef29* qlines_n, const EvLineDev* lines2,
                           const G1Dev* g1out, const G1Dev* pnorm, F12Dev* fbuf);
__global__ void k_miller_f3(const PairJob* jobs, uint32_t n, const LineCoef29* qlines_n, const LineCoef29* pklines_n,
                            const G1Dev* g1out, const G1Dev* pnorm, F12Dev* fbuf);
// final exponentiation phases (k_fexp.hip); park: fexp_park_bytes(n) of scratch (dev/sx29.h Park).
// FTS_FEXP_EASY_BATCH (default 1): the easy part in three launches with the
// launch's Fp inversions batched (k_fexp_easy_a, k_fexp_binv, k_fexp_easy_b)
#ifndef FTS_FEXP_EASY_BATCH
#define FTS_FEXP_EASY_BATCH 1
#endif
__global__ void k_fexp_easy(uint32_t n, const F12Dev* fbuf, int32_t* park);
__global__ void k_fexp_easy_a(uint32_t n, const F12Dev* fbuf, int32_t* park);
__global__ void k_fexp_easy_b(uint32_t n, const F12Dev* fbuf, int32_t* park);
__global__ void k_fexp_binv(uint32_t n, int32_t* park, uint32_t stride);
__global__ void k_fexp_expt(uint32_t n, int32_t* park, int src, int dst, int ps);
__global__ void k_fexp_hard(const PairJob* jobs, uint32_t n, uint8_t* arena, int32_t* park);
__global__ void k_fexp_fc_mid1(uint32_t n, int32_t* park);
__global__ void k_fexp_fc_mid2(uint32_t n, int32_t* park);
__global__ void k_fexp_fc_hard(const PairJob* jobs, uint32_t n, uint8_t* arena, int32_t* park);
inline size_t fexp_park_bytes(size_t n_pr) {
  return ((n_pr + SX_JOBS_PER_WAVE - 1) / SX_JOBS_PER_WAVE) * 64 * (size_t)FEXP_PARK_SLOTS * 18 * sizeof(int32_t);
}
// exact (FTZ_FEXP_EXACT): easy part, three x-powers, hard part; Fuentes-Castaneda
// (FTZ_FEXP_FUENTES): easy part and x-powers with its two glue steps
inline void launch_fexp(bool exact, const PairJob* jobs, uint32_t n, const F12Dev* fbuf, uint8_t* arena,
                        int32_t* park, hipStream_t s) {
  if (!n) return;
  const uint32_t nb = (n + SX_JOBS_PER_WAVE - 1) / SX_JOBS_PER_WAVE;
#if FTS_FEXP_EASY_BATCH
  k_fexp_easy_a<<<nb, 64, 0, s>>>(n, fbuf, park);
  k_fexp_binv<<<(n + 255) / 256, 256, 0, s>>>(n, park, nb * 64);
  k_fexp_easy_b<<<nb, 64, 0, s>>>(n, fbuf, park);
#else
  k_fexp_easy<<<nb, 64, 0, s>>>(n, fbuf, park);
#endif
  if (exact) {
    for (int e = 0; e < 3; e++) k_fexp_expt<<<nb, 64, 0, s>>>(n, park, e, e + 1, 4);
    k_fexp_hard<<<nb, 64, 0, s>>>(jobs, n, arena, park);
    return;
  }
  k_fexp_expt<<<nb, 64, 0, s>>>(n, park, 0, 1, FC_EXPT_SLOT);
  k_fexp_fc_mid1<<<nb, 64, 0, s>>>(n, park);
  k_fexp_expt<<<nb, 64, 0, s>>>(n, park, 3, 4, FC_EXPT_SLOT);
  k_fexp_fc_mid2<<<nb, 64, 0, s>>>(n, park);
  k_fexp_expt<<<nb, 64, 0, s>>>(n, park, 5, 6, FC_EXPT_SLOT);
  k_fexp_fc_hard<<<nb, 64, 0, s>>>(jobs, n, arena, park);
}

// prover (k_light.hip)
__global__ void k_rand(const RandJob* jobs, uint32_t n, const uint8_t* arena, uint32_t (*scal)[8]);
__global__ void k_emit(const EmitJob* jobs, uint32_t n, const uint32_t (*scal)[8], uint8_t* arena);
__global__ void k_b64(const B64Job* jobs, uint32_t n, const uint8_t* arena, uint8_t* out);
__global__ void k_copy(const CopyJob* jobs, uint32_t n, const uint8_t* wire, uint8_t* arena, uint8_t* out);

// standalone MSM (k_msm.hip)
__global__ void k_msm_load_pts(uint32_t n, const uint8_t* raw_pts, G1Dev* pts, uint8_t* ok);
__global__ void k_g1_sum(uint32_t n, const uint8_t* raw, uint8_t* out, uint32_t* status);
__global__ void k_g1_check(uint32_t n, const uint8_t* slots, uint8_t* ok);
__global__ void k_msm_load_scal(uint32_t n, const uint8_t* raw_scal, uint32_t (*scal)[8]);
__global__ void k_msm_keys(MsmPlan p, const uint32_t (*scal)[8], uint32_t* key, uint32_t* val, uint32_t* cnt);
__global__ void k_msm_scatter(MsmPlan p, const uint32_t* key, const uint32_t* val, const uint32_t* start,
                              uint32_t* cnt, uint32_t* perm);
__global__ void k_msm_keys_raw(MsmPlan p, uint32_t i0, uint32_t i1, const uint8_t* raw, uint32_t (*scal)[8],
                               uint32_t* key, uint32_t* val, uint32_t* cnt);
__global__ void k_msm_bounds(MsmPlan p, uint64_t total, const uint32_t* skey, const uint32_t* sval, uint32_t* start,
                             uint32_t* end);
__global__ void k_scan_block(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* tot);
__global__ void k_scan_add(uint32_t* out, uint32_t n, const uint32_t* add);
__global__ void k_msm_counts_scan(MsmPlan p, const uint32_t* start, const uint32_t* end, uint32_t* count,
                                  uint32_t* soff, uint32_t* tot);
__global__ void k_msm_owner(MsmPlan p, const uint32_t* count, const uint32_t* soff, uint32_t* owner, uint32_t* wlo,
                            uint32_t* whi);
__global__ void k_msm_phi(MsmPlan p, G1Dev* pts);
__global__ void k_msm_precompute(MsmPlan p, G1Dev* pts);
__global__ void k_msm_len_hist(MsmPlan p, const uint32_t* whi, const uint32_t* owner, const uint32_t* soff,
                               const uint32_t* count, uint32_t* hist);
__global__ void k_msm_len_scan(MsmPlan p, uint32_t* hist);
__global__ void k_msm_len_scatter(MsmPlan p, const uint32_t* whi, const uint32_t* owner, const uint32_t* soff,
                                  const uint32_t* count, uint32_t* cursor, uint32_t* order);
__global__ void k_msm_bucket(MsmPlan p, const uint32_t* whi, const uint32_t* order, const uint32_t* owner,
                             const uint32_t* soff, const uint32_t* start, const uint32_t* count,
                             const uint32_t* perm, const G1Dev* pts, G1JDev* slot_sum);
__global__ void k_msm_segment(MsmPlan p, uint32_t w0, uint32_t w1, const uint32_t* wlo, const uint32_t* whi,
                              const uint32_t* owner, const G1JDev* slot_sum, G1JDev* part);
__global__ void k_msm_tree(const G1JDev* in, uint32_t m, G1JDev* out);
__global__ void k_msm_horner(MsmPlan p, uint32_t w_hi, uint32_t w_lo, const G1JDev* wparts, uint32_t per,
                             G1JDev* acc_buf);
__global__ void k_msm_genpoints(uint32_t n, uint32_t off, uint32_t chunk, const G1Dev* gtab, G1JDev* jtmp,
                                uint32_t (*zs)[8], G1Dev* pts);

// idemix owner signatures (k_idemix.hip)
__global__ void k_nym_part(const NymJob* jobs, uint32_t n, const uint8_t* blob, const QDev* tab, QJDev* part);
__global__ void k_nym_fin(const NymJob* jobs, uint32_t n, uint8_t* blob, const QJDev* part, uint8_t* ok);
__global__ void k_eid(const uint8_t* in, uint32_t n, const QDev* tab, uint8_t* ok);
__global__ void k_nym_part_bn(const NymJob* jobs, uint32_t n, const uint8_t* blob, const QDev* tab, QJDev* part);
__global__ void k_nym_fin_bn(const NymJob* jobs, uint32_t n, uint8_t* blob, const QJDev* part, uint8_t* ok);
__global__ void k_eid_bn(const uint8_t* in, uint32_t n, const QDev* tab, uint8_t* ok);

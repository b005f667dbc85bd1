// Host-runtime internals shared by runtime.hip (contexts, batch slots, the
// staged batch API), engine.hip (the job engine / micro-batcher behind
// ftz_verify_*) and msm_rt.hip (standalone MSM): device buffers, the per-GPU
// context, errors.
#pragma once
#include <hip/hip_runtime.h>

#include <array>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ftsamd.h"
#include "dev/jobs.h"
#include "dev/sx29.h"
#include "host/planner.h"

using namespace fts;
using namespace ftsh;

// ------------------------------------------------------------------ host runtime
extern thread_local std::string g_err;
int set_err(int code, const std::string& msg);
#define HC(expr)                                                                                    \
  do {                                                                                              \
    hipError_t e_ = (expr);                                                                         \
    if (e_ != hipSuccess)                                                                           \
      return set_err(FTZ_E_DEVICE, std::string(#expr " failed: ") + hipGetErrorString(e_));        \
  } while (0)

template <class T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(size_t cnt) {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = cnt;
    if (cnt == 0) return hipSuccess;
    return hipMalloc(&p, cnt * sizeof(T));
  }
  hipError_t upload(const std::vector<T>& v, hipStream_t s) {
    hipError_t e = alloc(v.size());
    if (e != hipSuccess || v.empty()) return e;
    return hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s);
  }
};

// Grow-only device / pinned-host byte buffers (batch slots are reused, so
// steady-state batches neither hipMalloc nor page-lock).
struct DevMem {
  uint8_t* p = nullptr;
  size_t cap = 0;
  ~DevMem() {
    if (p) (void)hipFree(p);
  }
  hipError_t reserve(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = n + n / 4 + 4096;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
};
struct PinnedMem {
  uint8_t* p = nullptr;
  size_t cap = 0;
  ~PinnedMem() {
    if (p) (void)hipHostFree(p);
  }
  hipError_t reserve(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = n + n / 4 + 4096;
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) cap = want;
    return e;
  }
};

struct Engine;
struct ftz_prover;

struct ftz_ctx {
  int device = 0;
  hipStream_t stream = nullptr;  // context-level work (setup, MSM)
  PPInfo pp;
  PPInfo pp_var;                     // pp without the prover's table set (no_sigtab, no fixed pairs)
  std::vector<uint8_t> const_bytes;  // C_SIZE bytes, canonical PP RawBytes
  DBuf<G1Dev> g1tab;
  // the prover's table set: g1tab's bases, then the PS signature points of the
  // range digits (G1B_SIG0 ..), built on the first proving call
  std::vector<G1Dev> pp_g1;          // decoded PP G1 points: PedGen, Ped0..2, G, then R_d, S_d per digit
  std::mutex ptab_mu;
  DBuf<G1Dev> g1tab_p;
  bool ptab_ready = false;
  bool ptab_failed = false;          // its allocation failed once: the prover stays on the variable-base path
  // pp.fixed_pairs: the normalised Miller lines of PK1 then PK2 (k_miller_f3)
  std::vector<G2Dev> pp_g2;          // decoded PK0, PK1, PK2, Q
  DBuf<LineCoef29> pklines29n;
  DBuf<G2Dev> g2tab;
  DBuf<LineCoef> qlines;
  DBuf<LineCoef29> qlines29;         // the same lines in the balanced 29-bit form (k_miller)
  DBuf<LineCoef29> qlines29n;        // normalised by r0 (k_miller_n); used when qnorm
  bool qnorm = false;               // every fixed line has r0 != 0: k_miller_n, else k_miller
  ftz_options opt;                   // resolved options (ftz_ctx_create_ex)
  int serial = 0;                    // profiling: every kernel of a batch on one stream
  // t' + pair-2 lines: k_g2lines1 (one lane per job) or the sextet k_g2lines
  // (ftz_ctx_set_layout).  The verifier's pipeline is throughput bound (one lane:
  // fewest instructions).  The prover's pass was latency bound (t' waits for R')
  // and took the sextet (profiles/r02g_prover_layout.txt); with R' and S'' on
  // fixed-base tables (round 3) its passes fill the device and one lane is ahead
  // (profiles/r03s_prover_layout.txt)
  int g2lanes = FTZ_LAYOUT_ONE_LANE;
  bool g2lanes_set = false;
  std::atomic<const uint8_t*> debug_poison{nullptr};  // ftz_ctx_debug_poison (engine failure-isolation tests)  // ftz_ctx_set_layout chose it: small passes keep it too
  int g2lanes_prover = FTZ_LAYOUT_ONE_LANE;
  WorkPool* pool = nullptr;          // host planning threads
  std::mutex mu;                     // context-level device work (MSM, setup)
  // raw token requests: decoding threads of their own (the engine plans on `pool`
  // concurrently) and grow-only element-check buffers (no hipMalloc / hipFree --
  // which would wait on the engine's device work -- per call)
  std::mutex req_mu;
  WorkPool* req_pool = nullptr;
  double req_ms[6] = {};  // ftz_ctx_request_stats (under req_mu)
  hipStream_t chk_stream = nullptr;
  std::mutex chk_mu;
  PinnedMem chk_h;
  DevMem chk_d;
  // Stream triples (pairing chain / side G1 jobs / G2 + lines) shared by every
  // batch slot of the context round-robin, so the number of HIP streams -- and
  // of hardware queues they need (GPU_MAX_HW_QUEUES) -- stays 3 x opt.slots + 1
  // however many staged batches, prover slots and engine slots exist.
  std::vector<std::array<hipStream_t, 3>> triples;
  std::atomic<uint32_t> next_triple{0};
  // job engine behind ftz_verify_* (created on first use)
  std::mutex eng_mu;
  Engine* eng = nullptr;
  // reusable prover slots behind ftz_prove_* (one one-shot prove call at a time)
  std::mutex prove_mu;
  ftz_prover_host_stats pstats{};  // under prove_mu
  std::vector<ftz_prover*> pslots;
  // slot behind ftz_commit_tokens / ftz_audit_openings
  std::mutex aux_mu;
  struct ftz_batch* aux = nullptr;
};

// ------------------------------------------------------------------ batch slots
// Device scratch of a batch (values the kernels produce), sub-allocated from
// one grow-only buffer.
struct ScratchLayout {
  size_t pts, pt_ok, scal, canon, g1out, pnorm, g2out, fbuf, fxpark, lines2, part1, part1p, part2, vtab1, vtab1p, hash_ok, hash_ok_pre,
      codes, bitmap, total;
};

// One batch: its planning state, pinned staging blob, device blob + scratch,
// its three HIP streams and events.  The staged API hands one out per
// ftz_batch_load_*; the engine cycles a fixed set of them.
struct ftz_batch {
  ftz_ctx* ctx = nullptr;
  bool prover = false;
  size_t n = 0;
  PlanWork work;
  FlatPlan fp;
  ScratchLayout sl{};
  PinnedMem h_blob, h_res;  // staging (host -> device) and results (device -> host)
  DevMem d_blob, d_scr;
  hipEvent_t ev[20];
  bool ev_init = false;
  hipStream_t st[3] = {nullptr, nullptr, nullptr};
  bool pending = false;
  uint64_t jobs_last[FTZ_NKERNELS] = {};
  ftz_stats stats{};
  // engine bookkeeping: which caller requests this batch's items belong to
  struct Part {
    struct Request* req;
    size_t start, count;
  };
  std::vector<Part> parts;
  std::vector<PlanItem> items;
};
struct ftz_prover : ftz_batch {};

int slot_init(ftz_batch* b);                                      // streams + events (once)
int slot_plan_items(ftz_batch* b, size_t n, const PlanItem* items);  // plan + flatten into pinned staging
int slot_submit(ftz_batch* b, bool upload, bool fetch_codes);      // enqueue (optionally the H2D copy first)
int slot_wait(ftz_batch* b);                                       // block, collect stats
void slot_free(ftz_batch* b);                                      // sync + release everything
int prover_plan(ftz_batch* b, size_t n, const void* wit, int kind);  // kind 0 transfer / 1 issue
int prover_submit(ftz_batch* b, bool upload, bool fetch);
int prover_wait(ftz_batch* b);
// results of the last submission that fetched them (valid after slot_wait)
inline const int32_t* slot_codes(const ftz_batch* b) { return reinterpret_cast<const int32_t*>(b->h_res.p); }
inline const uint8_t* slot_out(const ftz_batch* b) {
  return b->h_res.p + ((b->n * sizeof(int32_t) + 255) & ~(size_t)255);
}

// gnark SetBytes check of n 64-byte element slots on the device (msm_rt.hip)
int g1_check_slots(ftz_ctx* c, size_t n, const uint8_t* slots, uint8_t* ok);

// ------------------------------------------------------------------ engine (engine.hip)
int engine_verify(ftz_ctx* c, size_t n, const ftz_transfer* tx, const ftz_issue* is, int32_t* codes);
void engine_destroy(ftz_ctx* c);

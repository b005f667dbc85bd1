// Host-runtime internals shared by runtime.hip (verification batches) and
// msm_rt.hip (standalone MSM): device buffers, the per-GPU context, errors.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../include/ftsamd.h"
#include "dev/jobs.h"
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

struct ftz_ctx {
  int device = 0;
  hipStream_t stream = nullptr, stream2 = nullptr, stream3 = nullptr;
  PPInfo pp;
  std::vector<uint8_t> const_bytes;  // C_SIZE bytes, canonical PP RawBytes
  DBuf<G1Dev> g1tab;
  DBuf<G2Dev> g2tab;
  DBuf<LineCoef> qlines;
  int threads = 8;
  std::mutex mu;
};


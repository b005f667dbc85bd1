// C ABI of the raw token-request path (include/ftsamd.h, host/request.h):
// ASN.1 + action JSON decoding on the context's request threads, element checks
// on the device, ZK verification of every action through the context's job
// engine -- pipelined over chunks of requests (ftsh::verify_token_requests).
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "host/request.h"
#include "rt_internal.h"

extern "C" int ftz_token_request_decode(const uint8_t* raw, size_t len, size_t counts[4], ftz_bytes* elems,
                                        size_t cap) {
  if (!counts || (!raw && len)) return set_err(FTZ_E_INVALID, "null argument");
  std::vector<ftsh::Slice> f[4];
  std::string e = ftsh::der_token_request(raw, len, f);
  if (!e.empty()) return set_err(FTZ_E_INVALID, e);
  size_t tot = 0;
  for (int k = 0; k < 4; k++) counts[k] = f[k].size(), tot += f[k].size();
  if (tot > cap || (tot && !elems)) return set_err(FTZ_E_INVALID, "elems capacity " + std::to_string(cap) +
                                                                      " < " + std::to_string(tot));
  size_t o = 0;
  for (int k = 0; k < 4; k++)
    for (const ftsh::Slice& s : f[k]) elems[o++] = ftz_bytes{s.p, s.len};
  return FTZ_SUCCESS;
}

namespace {
int verify_requests(ftz_ctx* ctx, size_t n, const ftz_bytes* reqs, ftz_get_state_fn get_state,
                    ftz_get_states_fn get_states, void* user, int32_t* codes, int32_t* failed_action) {
  if (!ctx || (n && (!reqs || !codes))) return set_err(FTZ_E_INVALID, "null argument");
  for (size_t i = 0; i < n; i++)
    if (!reqs[i].p && reqs[i].len) return set_err(FTZ_E_INVALID, "null request with non-zero length");
  WorkPool* pool;
  {
    std::lock_guard<std::mutex> lk(ctx->req_mu);
    if (!ctx->req_pool)
      ctx->req_pool = new WorkPool((int)std::max<uint32_t>(
          4, ctx->opt.request_threads ? ctx->opt.request_threads : ctx->opt.threads));
    pool = ctx->req_pool;
  }
  ftsh::RequestHooks h;
  // gnark SetBytes checks: uncompressed and infinity-flag encodings on the host
  // threads (a few field products each), compressed ones -- a square root each,
  // rare on the wire -- in one device pass (all of them on the device measured
  // slower: the calling thread then waits on each chunk's check pass,
  // profiles/r06/req_decode.txt)
  h.check = [ctx, pool](size_t m, const uint8_t* slots, uint8_t* ok) {
    std::atomic<size_t> ncomp{0};
    pool->run((m + 255) / 256, [&](size_t p) {
      for (size_t i = p * 256; i < m && i < (p + 1) * 256; i++) {
        if (slots[64 * i] & 0x80) {
          ok[i] = 2;
          ncomp.fetch_add(1, std::memory_order_relaxed);
          continue;
        }
        fts::g1a a;
        ok[i] = fts::g1_setbytes(slots + 64 * i, 64, a) ? 1 : 0;
      }
    });
    if (ncomp.load() == 0) return (int)FTZ_SUCCESS;
    std::vector<uint32_t> at;
    std::vector<uint8_t> cs;
    for (size_t i = 0; i < m; i++)
      if (ok[i] == 2) {
        at.push_back((uint32_t)i);
        cs.insert(cs.end(), slots + 64 * i, slots + 64 * i + 64);
      }
    std::vector<uint8_t> cok(at.size());
    int rc = g1_check_slots(ctx, at.size(), cs.data(), cok.data());
    for (size_t k = 0; k < at.size(); k++) ok[at[k]] = rc == FTZ_SUCCESS ? cok[k] : 0;
    return rc;
  };
  h.verify_transfers = [ctx](size_t m, const ftz_transfer* tx, int32_t* c) { return ftz_verify_transfers(ctx, m, tx, c); };
  h.verify_issues = [ctx](size_t m, const ftz_issue* is, int32_t* c) { return ftz_verify_issues(ctx, m, is, c); };
  h.get_state = get_state;
  h.get_states = get_states;
  h.user = user;
  h.par = [pool](size_t k, const std::function<void(size_t)>& f) { pool->run(k, f); };
  ftsh::RequestStats st;
  h.stats = &st;
  std::string err;
  int rc = ftsh::verify_token_requests(n, reqs, h, codes, failed_action, err);
  {
    std::lock_guard<std::mutex> lk(ctx->req_mu);
    const double v[6] = {st.decode, st.check, st.lookup, st.tokens, st.build, st.drain};
    for (int k = 0; k < 6; k++) ctx->req_ms[k] += v[k];
  }
  if (rc != FTZ_SUCCESS && !err.empty()) {
    std::string last = ftz_last_error();
    return set_err(rc, err + (last.empty() ? "" : ": " + last));
  }
  return rc;
}
}  // namespace

extern "C" int ftz_ctx_request_stats(ftz_ctx* ctx, double ms[6], int reset) {
  if (!ctx || !ms) return set_err(FTZ_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(ctx->req_mu);
  for (int k = 0; k < 6; k++) {
    ms[k] = ctx->req_ms[k];
    if (reset) ctx->req_ms[k] = 0;
  }
  return FTZ_SUCCESS;
}

extern "C" int ftz_verify_token_requests(ftz_ctx* ctx, size_t n, const ftz_bytes* reqs, ftz_get_state_fn get_state,
                                         void* user, int32_t* codes, int32_t* failed_action) {
  return verify_requests(ctx, n, reqs, get_state, nullptr, user, codes, failed_action);
}

extern "C" int ftz_verify_token_requests_batched(ftz_ctx* ctx, size_t n, const ftz_bytes* reqs,
                                                 ftz_get_states_fn get_states, void* user, int32_t* codes,
                                                 int32_t* failed_action) {
  if (!get_states) return set_err(FTZ_E_INVALID, "null get_states");
  return verify_requests(ctx, n, reqs, nullptr, get_states, user, codes, failed_action);
}

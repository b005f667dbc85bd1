// Closed-loop caller driver for the drop-in seam (bench.py "seam" leg).
//
// The Go shim calls ftz_verify_transfers with ONE TransferAction per call
// (validator_transfer.go:84-98); a peer validating many
// transactions at once has many such calls in flight.  ftz_callers_run starts
// `callers` threads, each calling ftz_verify_transfers(ctx, 1, ...) in a loop
// over `pool` for `seconds`, and reports the throughput and the per-call
// latency distribution -- measured from native threads, so the numbers are the
// engine's, not a Python loop's.
//
// out[0] calls per second, out[1] p50 ms, out[2] p99 ms, out[3] calls,
// out[4] verdicts that differ from expect[] (0 expected), out[5] max ms.
// A failing call's return code is returned and its ftz_last_error() text
// copied to err; -100: no call completed.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "../../../include/ftsamd.h"

extern "C" int ftz_callers_run(ftz_ctx* ctx, const ftz_transfer* pool, const int32_t* expect, size_t pool_n,
                               int callers, double seconds, double* out, char* err, size_t errlen) {
  if (!ctx || !pool || !out || pool_n == 0 || callers < 1 || seconds <= 0) return FTZ_E_INVALID;
  using Clock = std::chrono::steady_clock;
  std::vector<std::vector<float>> lat((size_t)callers);
  std::atomic<uint64_t> bad{0};
  std::atomic<int> rc_any{FTZ_SUCCESS};
  std::atomic<bool> err_set{false};
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  // the window opens once every caller thread exists (starting thousands of
  // threads takes longer than the window itself)
  Clock::time_point t_start, t_end;
  std::vector<std::thread> th;
  th.reserve((size_t)callers);
  for (int c = 0; c < callers; c++) {
    th.emplace_back([&, c]() {
      std::vector<float>& L = lat[(size_t)c];
      L.reserve(4096);
      size_t j = (size_t)c * 7919 % pool_n;
      ready++;
      while (!go.load()) std::this_thread::yield();
      std::this_thread::sleep_until(t_start);
      while (Clock::now() < t_end) {
        int32_t code = -1;
        Clock::time_point t0 = Clock::now();
        int rc = ftz_verify_transfers(ctx, 1, &pool[j], &code);
        Clock::time_point t1 = Clock::now();
        if (rc != FTZ_SUCCESS) {
          if (!err_set.exchange(true) && err && errlen) snprintf(err, errlen, "%s", ftz_last_error());
          rc_any = rc;
          return;
        }
        if (expect && code != expect[j]) bad++;
        L.push_back((float)std::chrono::duration<double, std::milli>(t1 - t0).count());
        j = (j + 1) % pool_n;
      }
    });
  }
  while (ready.load() < callers) std::this_thread::yield();
  t_start = Clock::now() + std::chrono::milliseconds(50);
  t_end = t_start + std::chrono::microseconds((int64_t)(seconds * 1e6));
  if (getenv("FTZ_CALLERS_DEBUG"))
    fprintf(stderr, "callers: %d ready, %.1f ms to start, window %.1f ms\n", callers,
            std::chrono::duration<double, std::milli>(t_start - Clock::now()).count(),
            std::chrono::duration<double, std::milli>(t_end - t_start).count());
  go = true;
  for (auto& t : th) t.join();
  if (getenv("FTZ_CALLERS_DEBUG")) {
    size_t tot = 0;
    for (auto& L : lat) tot += L.size();
    fprintf(stderr, "callers: joined, %zu calls, rc %d\n", tot, rc_any.load());
  }
  if (rc_any != FTZ_SUCCESS) return rc_any;
  std::vector<float> all;
  for (auto& L : lat) all.insert(all.end(), L.begin(), L.end());
  if (all.empty()) return -100;
  std::sort(all.begin(), all.end());
  auto pct = [&](double q) { return (double)all[std::min(all.size() - 1, (size_t)(q * (double)all.size()))]; };
  out[0] = (double)all.size() / seconds;
  out[1] = pct(0.50);
  out[2] = pct(0.99);
  out[3] = (double)all.size();
  out[4] = (double)bad.load();
  out[5] = (double)all.back();
  return FTZ_SUCCESS;
}

// ---- a native ledger for the block-level binding leg (bench.py "requests"):
// what a committer's state snapshot hands the library -- a hash map from the
// token key to json(token.Token), read by ftz_get_state_fn / ftz_get_states_fn
// callbacks that cost what a native lookup costs (no Python in the timed call).
#include <string>
#include <string_view>
#include <unordered_map>

namespace {
struct Ledger {
  std::string store;  // every key and value, back to back
  std::unordered_map<std::string_view, std::pair<size_t, size_t>> kv;  // key -> (value offset, length)
  uint64_t lookups = 0;  // calls (get_state) / keys (get_states), for the bench's report
  uint64_t calls = 0;
};
}  // namespace

extern "C" void* ftz_ledger_create(size_t n, const ftz_bytes* keys, const ftz_bytes* vals) {
  Ledger* l = new Ledger();
  size_t tot = 0;
  for (size_t i = 0; i < n; i++) tot += keys[i].len + vals[i].len;
  l->store.reserve(tot);
  std::vector<std::pair<size_t, size_t>> ko(n);
  for (size_t i = 0; i < n; i++) {
    ko[i] = {l->store.size(), keys[i].len};
    l->store.append((const char*)keys[i].p, keys[i].len);
    l->store.append((const char*)vals[i].p, vals[i].len);
  }
  l->kv.reserve(n);
  for (size_t i = 0; i < n; i++)
    l->kv.emplace(std::string_view(l->store.data() + ko[i].first, ko[i].second),
                  std::make_pair(ko[i].first + ko[i].second, vals[i].len));
  return l;
}

extern "C" void ftz_ledger_destroy(void* p) { delete (Ledger*)p; }

extern "C" void ftz_ledger_counts(void* p, uint64_t* calls, uint64_t* lookups) {
  Ledger* l = (Ledger*)p;
  *calls = l->calls;
  *lookups = l->lookups;
}

extern "C" int ftz_ledger_get_state(void* user, const char* key, size_t key_len, const uint8_t** val,
                                    size_t* val_len) {
  Ledger* l = (Ledger*)user;
  l->calls++;
  l->lookups++;
  auto it = l->kv.find(std::string_view(key, key_len));
  if (it == l->kv.end()) {
    *val = nullptr;
    *val_len = 0;
    return 0;  // GetState of a missing key: nil value, no error
  }
  *val = (const uint8_t*)l->store.data() + it->second.first;
  *val_len = it->second.second;
  return 0;
}

extern "C" int ftz_ledger_get_states(void* user, size_t n, const ftz_bytes* keys, ftz_bytes* vals) {
  Ledger* l = (Ledger*)user;
  l->calls++;
  l->lookups += n;
  for (size_t i = 0; i < n; i++) {
    auto it = l->kv.find(std::string_view((const char*)keys[i].p, keys[i].len));
    vals[i] = it == l->kv.end() ? ftz_bytes{nullptr, 0}
                                : ftz_bytes{(const uint8_t*)l->store.data() + it->second.first, it->second.second};
  }
  return 0;
}

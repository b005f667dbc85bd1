// Job engine behind ftz_verify_transfers / ftz_verify_issues: one per context.
//
// The reference verifies one action per call and fans out goroutines inside
// it (validator_transfer.go:84-98, range/proof.go:247-257); concurrency comes
// from the peer running many validations at once (tcc.go:223-237) and the
// client-side double-checks (token/request.go:295-298).  A GPU pass only pays
// off on thousands of proofs, so every call becomes a *request* in one queue
// per context and a dispatcher thread cuts the queue into device batches:
//
//   * a big call (a block, a 1M-transfer job) is split into batches of at most
//     opt.batch proofs -- which also keeps every 32-bit job index of a batch in
//     range -- and fills the pipeline by itself;
//   * small concurrent calls (the Go shim verifies ONE TransferAction per call)
//     are coalesced: while the GPU has >= opt.hold_inflight batches in flight a
//     partial batch waits up to opt.window_us (from its oldest request) for more
//     callers, otherwise it goes at once (hold_inflight 0: it always waits, so
//     callers that resubmit together after a batch completes share the next
//     batch instead of splitting into a lone first request and the rest); with
//     every slot busy, callers accumulate for the next free slot anyway;
//   * transfers and issues share batches (the planner emits the same jobs).
//
// Batches cycle through opt.slots reusable slots (pinned staging blob, device
// buffers, streams, events): the dispatcher plans batch k+1 on the host pool
// while batches k, k-1, ... run on the device; a completion thread waits for
// the oldest batch in flight, scatters its verdict codes back to the requests
// and recycles the slot.  A request returns when all its proofs are done.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ftsamd.h"
#include "rt_internal.h"

using Clock = std::chrono::steady_clock;

struct Request {
  const ftz_transfer* tx = nullptr;  // exactly one of tx / is
  const ftz_issue* is = nullptr;
  size_t n = 0;
  int32_t* codes = nullptr;
  size_t next = 0;         // next proof to hand to a batch (dispatcher, under mu)
  size_t outstanding = 0;  // proofs not yet completed (under mu)
  int rc = FTZ_SUCCESS;
  std::string err;
  bool finished = false;    // all proofs completed (under the engine mu)
  bool solo = false;        // planned in batches of its own (after a shared batch failed to plan; under mu)
  Clock::time_point t0;
  // the caller's own wake-up: it sleeps on m / cv, not on the engine lock, so a
  // completing pass wakes exactly its callers and they do not queue on one mutex
  std::mutex m;
  std::condition_variable cv;
  bool done = false;  // under m
};

// proof bytes per batch stay well below the 2^31 arena / wire limits
static constexpr size_t BATCH_PROOF_BYTES = (size_t)256 << 20;

struct Engine {
  ftz_ctx* ctx = nullptr;
  std::mutex mu;
  std::condition_variable cv_q, cv_free, cv_comp;
  std::deque<Request*> q;
  size_t pending = 0;        // proofs queued and not yet handed to a batch (under mu)
  bool disp_holding = false;  // the dispatcher is waiting out a window (under mu)
  bool tail_split_done = false;  // the queue's last pass was cut in two (under mu; reset by new requests)
  uint32_t ramp_step = 0;        // passes since the engine was last idle (FTS_ENGINE_RAMP2)
  std::vector<ftz_batch*> slots;
  std::deque<ftz_batch*> free_slots, inflight;
  ftz_engine_stats st{};
  Clock::time_point first, last;
  bool stop = false;
  bool disp_done = false;  // the dispatcher has exited (nothing more will be put in flight)
  std::thread disp, comp;

  void dispatcher();
  void completer();
  void fail_parts(ftz_batch* b, int rc, const std::string& err, std::vector<Request*>& wake);
  void requeue_solo(ftz_batch* b);
};

static PlanItem item_of(const Request* r, size_t i) {
  PlanItem it;
  memset(&it, 0, sizeof(it));
  if (r->tx) {
    const ftz_transfer& t = r->tx[i];
    it.kind = 0;
    it.t = {t.inputs, t.n_in, t.outputs, t.n_out, t.proof, t.proof_len};
  } else {
    const ftz_issue& s = r->is[i];
    it.kind = 1;
    it.i = {s.outputs, s.n_out, s.proof, s.proof_len, s.anonymous};
  }
  return it;
}

// membership proofs (= pairing jobs) an item brings: one per range-proof digit
// of every output (range/proof.go:228-257)
static uint64_t item_pairs(const Request* r, size_t i, uint64_t exponent) {
  return exponent * (r->tx ? r->tx[i].n_out : r->is[i].n_out);
}

static size_t item_bytes(const Request* r, size_t i) {
  return r->tx ? r->tx[i].proof_len + 64 * ((size_t)r->tx[i].n_in + r->tx[i].n_out)
               : r->is[i].proof_len + 64 * (size_t)r->is[i].n_out;
}

// A batch part of request r completed (mu held): collect the caller when it was the last.
static void finish_part(Request* r, size_t count, std::vector<Request*>& wake) {
  r->outstanding -= count;
  if (r->outstanding == 0 && r->next == r->n && !r->finished) {
    r->finished = true;
    wake.push_back(r);
  }
}

// Wake collected callers (engine mu NOT held).  done is set and notified under
// the request's own mutex, so the caller cannot return and free r before we
// let go of it; r is not touched afterwards.
static void wake_all(std::vector<Request*>& wake) {
  for (Request* r : wake) {
    std::lock_guard<std::mutex> g(r->m);
    r->done = true;
    r->cv.notify_one();
  }
  wake.clear();
}

// Deliver a failed batch's error to its requests (mu held).
void Engine::fail_parts(ftz_batch* b, int rc, const std::string& err, std::vector<Request*>& wake) {
  for (auto& p : b->parts) {
    if (p.req->rc == FTZ_SUCCESS) {
      p.req->rc = rc;
      p.req->err = err;
    }
    finish_part(p.req, p.count, wake);
  }
  b->parts.clear();
}

// Undo the hand-out of a batch that failed to plan (mu held): each part goes
// back to the front of the queue in its old order, its request marked solo.
// Parts follow queue order and only the last one's request can still be queued.
void Engine::requeue_solo(ftz_batch* b) {
  for (size_t k = b->parts.size(); k-- > 0;) {
    const auto& p = b->parts[k];
    Request* r = p.req;
    bool queued = r->next < r->n;  // not popped: it is q.front()
    r->next = p.start;
    pending += p.count;
    r->solo = true;
    if (!queued) q.push_front(r);
  }
  b->parts.clear();
  b->items.clear();
}

void Engine::dispatcher() {
  (void)hipSetDevice(ctx->device);
  const size_t B = ctx->opt.batch;
  const auto window = std::chrono::microseconds(ctx->opt.window_us);
  std::unique_lock<std::mutex> lk(mu);
  while (true) {
    cv_q.wait(lk, [&]() { return stop || !q.empty(); });
    if (q.empty()) {
      if (stop) {
        disp_done = true;
        cv_comp.notify_all();
        return;
      }
      continue;
    }
    if (pending < B && inflight.size() >= ctx->opt.hold_inflight && !stop) {
      // the device is busy: let a partial batch wait (a bounded time) for company
      Clock::time_point deadline = q.front()->t0 + window;
      if (Clock::now() < deadline) {
        disp_holding = true;  // enqueuers now notify only once a full batch is pending
        cv_q.wait_until(lk, deadline);
        disp_holding = false;
        continue;  // re-evaluate: a full batch, a completion, or the deadline
      }
    }
    cv_free.wait(lk, [&]() { return !free_slots.empty(); });
    ftz_batch* b = free_slots.front();
    free_slots.pop_front();
    b->parts.clear();
    b->items.clear();
    // A pass closes at B items, BATCH_PROOF_BYTES of proofs, or B * 4 pairing
    // jobs -- a PP-A pass of B 2-output transfers (e = 2): wider range proofs
    // (PP-B: e = 16, 8x the pairings per transfer) get proportionally fewer
    // proofs per pass, so their passes cost what a PP-A pass costs.
    // The first pass of a job (nothing in flight) may be smaller: it reaches the
    // device after a shorter planning step (ftz_options.first_pass, default
    // 4096 of the 8192-proof batch: +2.5 % on a 20-step job, profiles/r05/
    // first_pass_ab.txt).  Passes much smaller than that throughout the job were
    // slower (round 2: 420-442k vs 676-688k transfers/s): a pass's planning and
    // kernel chain have a fixed latency that small passes do not shed.
    const size_t fp1 = ctx->opt.first_pass, ts = ctx->opt.tail_split;
#ifndef FTS_ENGINE_RAMP2
#define FTS_ENGINE_RAMP2 0
#endif
    size_t Bp = (fp1 && fp1 < B && inflight.empty()) ? fp1 : B;
    // (doubling passes from fp1 while few are in flight -- fp1, 2 fp1, ... --
    // measured 0.43-0.55M against 0.76-0.80M transfers/s on the 20-step job,
    // profiles/r06/engine_ramp.txt: the small passes' fixed latency again)
    // FTS_ENGINE_RAMP2: doubling from fp1 only for the passes that follow an
    // idle engine (fp1, 2 fp1, ... up to B, then B until it is idle again);
    // with first_pass 1024 it measured within noise of the default on two
    // boxes (means 808k against 784k, medians 815k against 803k), so it is off
    if (FTS_ENGINE_RAMP2 && fp1 && fp1 < B) {
      if (inflight.empty() && ramp_step > 0 && (fp1 << std::min<uint32_t>(ramp_step, 20)) >= B) ramp_step = 0;
      Bp = std::min(B, fp1 << std::min<uint32_t>(ramp_step, 20));
      ramp_step++;
    }
    // the queue's last pass in two halves whose kernel chains overlap
    // (ftz_options.tail_split)
    if (ts && !tail_split_done && !inflight.empty() && pending <= Bp && pending >= 2 * (size_t)ts) {
      Bp = (pending + 1) / 2;
      tail_split_done = true;  // the second half goes whole
    }
    size_t bytes = 0;
    uint64_t pairs = 0;
    const uint64_t pair_budget = 4 * (uint64_t)Bp, ex = (uint64_t)std::max<int64_t>(1, ctx->pp.exponent);
    auto room = [&]() {
      return b->items.empty() || (bytes < BATCH_PROOF_BYTES && pairs < pair_budget);
    };
    while (!q.empty() && b->items.size() < Bp && room()) {
      Request* r = q.front();
      if (r->solo && !b->items.empty()) break;  // a solo request never shares a batch
      size_t start = r->next;
      while (r->next < r->n && b->items.size() < Bp && room()) {
        bytes += item_bytes(r, r->next);
        pairs += item_pairs(r, r->next, ex);
        b->items.push_back(item_of(r, r->next));
        r->next++;
        pending--;
      }
      if (r->next > start) b->parts.push_back({r, start, r->next - start});
      if (r->next == r->n) q.pop_front();
      if (!room() || r->solo) break;
    }
    lk.unlock();
    Clock::time_point t0 = Clock::now();
    int rc = slot_plan_items(b, b->items.size(), b->items.data());
    Clock::time_point t1 = Clock::now();
    if (rc != FTZ_SUCCESS && b->parts.size() > 1) {
      // a planning error is one caller's bad input (a limit, a null pointer):
      // hand every request of the batch back and plan each on its own, so
      // that the error reaches only the request that caused it
      lk.lock();
      requeue_solo(b);
      free_slots.push_back(b);
      cv_free.notify_one();
      continue;
    }
    if (rc == FTZ_SUCCESS) rc = slot_submit(b, true, true);
    Clock::time_point t2 = Clock::now();
    std::string err = rc == FTZ_SUCCESS ? std::string() : g_err;
    lk.lock();
    if (st.batches == 0 && inflight.empty()) first = t1;
    st.batches++;
    st.proofs += b->items.size();
    st.plan_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
    st.submit_ms += std::chrono::duration<double, std::milli>(t2 - t1).count();
    st.max_in_flight = std::max<uint32_t>(st.max_in_flight, (uint32_t)inflight.size() + 1);
    if (rc != FTZ_SUCCESS) {
      if (b->pending) {  // enqueued part of the work before failing: let it drain first
        lk.unlock();
        (void)slot_wait(b);
        lk.lock();
      }
      std::vector<Request*> wake;
      fail_parts(b, rc, err, wake);
      free_slots.push_back(b);
      cv_free.notify_one();
      lk.unlock();
      wake_all(wake);
      lk.lock();
      continue;
    }
    inflight.push_back(b);
    cv_comp.notify_one();
  }
}

void Engine::completer() {
  (void)hipSetDevice(ctx->device);
  std::unique_lock<std::mutex> lk(mu);
  std::vector<Request*> wake;
  while (true) {
    cv_comp.wait(lk, [&]() { return disp_done || !inflight.empty(); });
    if (inflight.empty()) return;  // disp_done: nothing more will arrive
    ftz_batch* b = inflight.front();
    lk.unlock();
    int rc = slot_wait(b);
    std::string err = rc == FTZ_SUCCESS ? std::string() : g_err;
    if (rc == FTZ_SUCCESS) {
      const int32_t* codes = slot_codes(b);
      size_t off = 0;
      for (auto& p : b->parts) {  // each request's range is written by this thread only
        memcpy(p.req->codes + p.start, codes + off, p.count * sizeof(int32_t));
        off += p.count;
      }
    }
    float dev_ms = 0;
    if (rc == FTZ_SUCCESS) (void)hipEventElapsedTime(&dev_ms, b->ev[18], b->ev[13]);
    lk.lock();
    st.device_ms += dev_ms;
    last = Clock::now();
    st.wall_ms = std::chrono::duration<double, std::milli>(last - first).count();
    inflight.pop_front();
    if (rc != FTZ_SUCCESS) {
      fail_parts(b, rc, err, wake);
    } else {
      for (auto& p : b->parts) finish_part(p.req, p.count, wake);
      b->parts.clear();
    }
    free_slots.push_back(b);
    cv_free.notify_one();
    cv_q.notify_one();  // a partial batch may go now that the device has room
    lk.unlock();
    wake_all(wake);
    lk.lock();
  }
}

static Engine* get_engine(ftz_ctx* c, int& rc) {
  std::lock_guard<std::mutex> lk(c->eng_mu);
  rc = FTZ_SUCCESS;
  if (c->eng) return c->eng;
  Engine* e = new Engine();
  e->ctx = c;
  for (uint32_t k = 0; k < c->opt.slots; k++) {
    ftz_batch* b = new ftz_batch();
    b->ctx = c;
    rc = slot_init(b);
    e->slots.push_back(b);
    e->free_slots.push_back(b);
    if (rc != FTZ_SUCCESS) break;
  }
  if (rc != FTZ_SUCCESS) {
    for (ftz_batch* b : e->slots) {
      slot_free(b);
      delete b;
    }
    delete e;
    return nullptr;
  }
  e->disp = std::thread([e]() { e->dispatcher(); });
  e->comp = std::thread([e]() { e->completer(); });
  c->eng = e;
  return e;
}

int engine_verify(ftz_ctx* c, size_t n, const ftz_transfer* tx, const ftz_issue* is, int32_t* codes) {
  int rc;
  Engine* e = get_engine(c, rc);
  if (!e) return rc;
  Request r;
  r.tx = tx;
  r.is = is;
  r.n = n;
  r.codes = codes;
  r.outstanding = n;
  r.t0 = Clock::now();
  {
    std::lock_guard<std::mutex> lk(e->mu);
    if (e->stop) return set_err(FTZ_E_INVALID, "context is being destroyed");
    e->q.push_back(&r);
    e->pending += n;
    e->tail_split_done = false;
    // a dispatcher waiting out a window only needs waking for a full batch
    if (!e->disp_holding || e->pending >= e->ctx->opt.batch) e->cv_q.notify_one();
  }
  {
    std::unique_lock<std::mutex> lk(r.m);
    r.cv.wait(lk, [&]() { return r.done; });
  }
  if (r.rc != FTZ_SUCCESS) return set_err(r.rc, r.err);
  return FTZ_SUCCESS;
}

void engine_destroy(ftz_ctx* c) {
  Engine* e;
  {
    std::lock_guard<std::mutex> lk(c->eng_mu);
    e = c->eng;
    c->eng = nullptr;
  }
  if (!e) return;
  {
    std::lock_guard<std::mutex> lk(e->mu);
    e->stop = true;
  }
  e->cv_q.notify_all();
  e->cv_comp.notify_all();
  e->cv_free.notify_all();
  e->disp.join();
  e->comp.join();
  for (ftz_batch* b : e->slots) {
    slot_free(b);
    delete b;
  }
  delete e;
}

extern "C" int ftz_ctx_engine_stats(ftz_ctx* c, ftz_engine_stats* out, int reset) {
  if (!c || !out) return set_err(FTZ_E_INVALID, "null argument");
  memset(out, 0, sizeof(*out));
  std::lock_guard<std::mutex> lk(c->eng_mu);
  Engine* e = c->eng;
  if (!e) return FTZ_SUCCESS;
  std::lock_guard<std::mutex> lk2(e->mu);
  *out = e->st;
  if (reset) e->st = ftz_engine_stats{};
  return FTZ_SUCCESS;
}

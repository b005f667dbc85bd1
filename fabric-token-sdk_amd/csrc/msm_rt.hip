// C ABI of the standalone G1 MSM (include/ftsamd.h, dev/msm.h).
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <rocprim/device/device_radix_sort.hpp>

#include "launch.h"
#include "rt_internal.h"

struct ftz_msm {
  ftz_ctx* ctx = nullptr;
  MsmPlan p{};
  DBuf<G1Dev> pts;
  DBuf<uint32_t> scal, key, skey, val, perm, count, tot, soff, owner, wlo, whi, order;
  // start[wb], end[wb] and the slot-length histogram[1024] in one buffer: one
  // memset clears the three before the bounds pass (nothing writes the
  // histogram before k_msm_len_hist), two dependent launches fewer per run
  DBuf<uint32_t> zb;
  uint32_t *start_p = nullptr, *end_p = nullptr, *lenhist_p = nullptr;
  DBuf<uint8_t> sort_tmp;
  size_t sort_tmp_bytes = 0;
  uint32_t key_bits = 0;
  DBuf<G1JDev> slot_sum, part, tree;
  DBuf<G1JDev> hacc;
  G1JDev* hwin = nullptr;  // page-locked: the window sums read back for the host Horner
  DBuf<uint8_t> ok;
  hipEvent_t ev[2];
  bool ev_init = false;
  // ftz_msm_run_scalars: raw big-endian scalars on the device, a copy stream and
  // one event per chunk (created on first use)
  DBuf<uint8_t> raw;
  hipStream_t cstream = nullptr;
  static constexpr int RAW_CHUNKS = 8;
  hipEvent_t cev[RAW_CHUNKS + 1];
  bool cev_init = false;
  float last_ms = 0;
  // ftz_msm_run's launch chain (keys .. Horner, ~25 kernels and memsets) as one
  // graph, captured on the first run: the short launches of a 2^16 MSM ran
  // behind the host's enqueue rate (15-18 us gaps); graph_state 0 = not tried,
  // 1 = captured, -1 = capture failed (direct launches)
  hipGraph_t graph = nullptr;
  hipGraphExec_t graph_exec = nullptr;
  int graph_state = 0;
  uint32_t radix_bits = 8;  // digit bits per radix-sort pass (8: rocPRIM's gfx950 default; 9: Radix9)
  // FTS_MSM_CSORT=1, small plans (dev/msm.h MSM_SMALL_LG): a counting sort
  // instead of rocPRIM's radix sort -- the keys kernel counts each (window,
  // bucket) group with an atomic, a scan gives the group starts, one scatter
  // places the values by returning atomics (end[] holds the counts).  It
  // saves ~9 of the radix sort's and bounds pass's ~5 us dependent launches
  // but measured slower from 2^16 points up (2^16 0.71 against 0.61-0.64 ms,
  // 2^18 1.66 against 1.16-1.19: the scatter's 1.3M returning atomics take
  // 95 us), faster only at 2^14 (0.51 against 0.56), profiles/r06/msm_csort.txt
  bool csort = false;
};

static int blocks(uint64_t n, int bs) { return (int)((n + bs - 1) / bs); }

// The (key, value) sort uses rocPRIM's gfx950 onesweep default (8 key bits per
// pass) or, where 9-bit digits save a pass (17- and 18-bit keys: 2^24 points at
// c = 19), the same kernel shape with 512 digit bins.  An 11-bit config (2048
// digit bins, 256-thread blocks, match ranking) measured slower in round 3:
// 2^20 3.29 -> 4.33 ms, 2^24 29.0 -> 44.6 ms.
using Radix9 = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 12>, rocprim::kernel_config<1024, 12>, 9,
                                        rocprim::block_radix_rank_algorithm::match>>;

static hipError_t msm_sort(ftz_msm* m, void* tmp, size_t& tb, size_t wn, hipStream_t s) {
  if (m->radix_bits == 9)
    return rocprim::radix_sort_pairs<Radix9>(tmp, tb, m->key.p, m->skey.p, m->val.p, m->perm.p, wn, 0, m->key_bits, s);
  return rocprim::radix_sort_pairs(tmp, tb, m->key.p, m->skey.p, m->val.p, m->perm.p, wn, 0, m->key_bits, s);
}

static int msm_alloc(ftz_msm* m, size_t n) {
  const MsmPlan& p = m->p;
  size_t wb = (size_t)p.rw * p.buckets, wn = (size_t)p.windows * p.nv, ws = (size_t)p.rw * p.max_slots;
  HC(m->pts.alloc(p.pts));  // P_i, then phi(P_i) for GLV (pre: then 2^(c w) of both, then the identity)
  HC(m->scal.alloc(8 * n));
  HC(m->key.alloc(wn));
  HC(m->skey.alloc(wn));
  HC(m->val.alloc(wn));
  HC(m->perm.alloc(wn));
  HC(m->count.alloc(wb));
  HC(m->zb.alloc(2 * wb + 1024));
  m->start_p = m->zb.p;
  m->end_p = m->zb.p + wb;
  m->lenhist_p = m->zb.p + 2 * wb;
  m->key_bits = msm_key_bits(p);
#ifndef FTS_MSM_CSORT
#define FTS_MSM_CSORT 0
#endif
  m->csort = FTS_MSM_CSORT && !p.pre && msm_lg(p.nv) <= MSM_SMALL_LG;
  // 9-bit digits where they save a pass (17-18 bits: two passes instead of three)
  if (p.rw > 32) return set_err(FTZ_E_INVALID, "MSM plan has more than 32 windows");
  const uint32_t rb = m->ctx->opt.msm_radix_bits;
  m->radix_bits = rb ? rb : (m->key_bits > 16 && m->key_bits <= 18 ? 9u : 8u);
  HC(msm_sort(m, nullptr, m->sort_tmp_bytes, wn, m->ctx->stream));
  HC(m->sort_tmp.alloc(m->sort_tmp_bytes ? m->sort_tmp_bytes : 1));
  HC(m->tot.alloc(2 * ((wb + 1023) / 1024) + 2048));
  HC(m->soff.alloc(wb));
  HC(m->owner.alloc(ws));
  HC(m->wlo.alloc(p.rw));
  HC(m->whi.alloc(p.rw));
  HC(m->slot_sum.alloc(ws));
  HC(m->order.alloc(ws));
  HC(m->part.alloc((size_t)p.rw * p.segs));
  HC(m->tree.alloc((size_t)p.rw * ((p.segs + MSM_TREE_CHUNK - 1) / MSM_TREE_CHUNK) * 2));
  HC(m->hacc.alloc(1));
  HC(hipHostMalloc(reinterpret_cast<void**>(&m->hwin), (size_t)p.rw * sizeof(G1JDev), hipHostMallocDefault));
  HC(m->ok.alloc(n));
  for (int k = 0; k < 2; k++) HC(hipEventCreate(&m->ev[k]));
  m->ev_init = true;

  return FTZ_SUCCESS;
}

// exclusive scan of n counters in place of `out` (recursive over block totals)
static int scan(uint32_t* in, uint32_t* out, size_t n, uint32_t* tmp, hipStream_t s) {
  uint32_t nb = (uint32_t)((n + 1023) / 1024);
  k_scan_block<<<nb, 1024, 0, s>>>(in, out, (uint32_t)n, tmp);
  if (nb > 1) {
    uint32_t* sums = tmp + nb;
    int rc = scan(tmp, sums, nb, sums + nb + 1, s);
    if (rc != FTZ_SUCCESS) return rc;
    k_scan_add<<<nb, 1024, 0, s>>>(out, (uint32_t)n, sums);
  }
  return FTZ_SUCCESS;
}

static int msm_new(ftz_ctx* c, size_t n, ftz_msm** out) {
  if (!c || !out) return set_err(FTZ_E_INVALID, "null argument");
  if (n == 0 || n > (1u << 28)) return set_err(FTZ_E_INVALID, "MSM size must be in [1, 2^28]");
  HC(hipSetDevice(c->device));
  ftz_msm* m = new ftz_msm();
  m->ctx = c;
  // planner overrides from the context's options (window bits, slot cap, slots per
  // segment; 0 = the planner's choice) and the GLV switch
  const ftz_options& o = c->opt;
  m->p = msm_make_plan(n, o.msm_window_bits, o.msm_slot_cap, o.msm_seg_slots, o.msm_glv != 0, o.msm_precompute != 0);
  // sort values carry a point index in 31 bits (pre) or an entry index in 30
  if (m->p.pre && (uint64_t)m->p.windows * m->p.nv + 1 >= (1ull << 31)) {
    delete m;
    return set_err(FTZ_E_INVALID, "msm_precompute: windows x points exceeds 2^31 resident points");
  }
  if (!m->p.pre && (uint64_t)m->p.windows * m->p.nv >= (1ull << 30)) {
    delete m;
    return set_err(FTZ_E_INVALID, "MSM too large: windows x points exceeds 2^30 sort entries");
  }
  int rc = msm_alloc(m, n);
  if (rc != FTZ_SUCCESS) {
    ftz_msm_destroy(m);
    return rc;
  }
  *out = m;
  return FTZ_SUCCESS;
}

// resident points from P_i: phi(P_i) = (beta x_i, y_i) next to P_i for the GLV
// halves; with pre the window multiples 2^(c w) of both and the identity last
static int prepare_points(ftz_msm* m) {
  hipStream_t s = m->ctx->stream;
  const MsmPlan& p = m->p;
  if (p.glv) k_msm_phi<<<blocks(p.n, 256), 256, 0, s>>>(p, m->pts.p);
  if (p.pre) k_msm_precompute<<<blocks(p.nv, 256), 256, 0, s>>>(p, m->pts.p);
  HC(hipMemsetAsync(m->pts.p + (p.pts - 1), 0, sizeof(G1Dev), s));  // the identity: zero digits
  HC(hipGetLastError());
  return FTZ_SUCCESS;
}

static int upload_scalars(ftz_msm* m, const uint8_t* scalars) {
  hipStream_t s = m->ctx->stream;
  size_t n = m->p.n;
  DBuf<uint8_t> raw;
  HC(raw.alloc(32 * n));
  HC(hipMemcpyAsync(raw.p, scalars, 32 * n, hipMemcpyHostToDevice, s));
  k_msm_load_scal<<<blocks(n, 256), 256, 0, s>>>((uint32_t)n, raw.p, reinterpret_cast<uint32_t (*)[8]>(m->scal.p));
  HC(hipStreamSynchronize(s));
  return FTZ_SUCCESS;
}

extern "C" int ftz_msm_load(ftz_ctx* c, size_t n, const uint8_t* points, const uint8_t* scalars, ftz_msm** out) {
  if (!points || !scalars) return set_err(FTZ_E_INVALID, "null argument");
  if (!c) return set_err(FTZ_E_INVALID, "null context");
  std::lock_guard<std::mutex> lk(c->mu);
  ftz_msm* m = nullptr;
  int rc = msm_new(c, n, &m);
  if (rc != FTZ_SUCCESS) return rc;
  hipStream_t s = c->stream;
  {
    DBuf<uint8_t> raw;
    if (raw.alloc(64 * n) != hipSuccess ||
        hipMemcpyAsync(raw.p, points, 64 * n, hipMemcpyHostToDevice, s) != hipSuccess) {
      ftz_msm_destroy(m);
      return set_err(FTZ_E_NOMEM, "point upload failed");
    }
    k_msm_load_pts<<<blocks(n, 256), 256, 0, s>>>((uint32_t)n, raw.p, m->pts.p, m->ok.p);
    std::vector<uint8_t> ok(n);
    if (hipMemcpyAsync(ok.data(), m->ok.p, n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      ftz_msm_destroy(m);
      return set_err(FTZ_E_DEVICE, "point decode failed");
    }
    for (size_t i = 0; i < n; i++)
      if (!ok[i]) {
        ftz_msm_destroy(m);
        return set_err(FTZ_E_INVALID, "point " + std::to_string(i) + " is not a canonical BN254 G1 point");
      }
  }
  rc = prepare_points(m);
  if (rc == FTZ_SUCCESS) rc = upload_scalars(m, scalars);
  if (rc != FTZ_SUCCESS) {
    ftz_msm_destroy(m);
    return rc;
  }
  *out = m;
  return FTZ_SUCCESS;
}

extern "C" int ftz_msm_load_gen(ftz_ctx* c, size_t n, uint32_t offset, const uint8_t* scalars, ftz_msm** out) {
  if (!scalars) return set_err(FTZ_E_INVALID, "null argument");
  if (!c) return set_err(FTZ_E_INVALID, "null context");
  if ((uint64_t)offset + n >= (1ull << 32) || offset == 0) return set_err(FTZ_E_INVALID, "bad point offset");
  std::lock_guard<std::mutex> lk(c->mu);
  ftz_msm* m = nullptr;
  int rc = msm_new(c, n, &m);
  if (rc != FTZ_SUCCESS) return rc;
  hipStream_t s = c->stream;
  {
    const uint32_t chunk = 64;
    DBuf<G1JDev> jtmp;
    DBuf<uint32_t> zs;
    if (jtmp.alloc(n) != hipSuccess || zs.alloc(8 * n) != hipSuccess) {
      ftz_msm_destroy(m);
      return set_err(FTZ_E_NOMEM, "scratch allocation failed");
    }
    k_msm_genpoints<<<blocks((n + chunk - 1) / chunk, 128), 128, 0, s>>>(
        (uint32_t)n, offset, chunk, c->g1tab.p, jtmp.p, reinterpret_cast<uint32_t (*)[8]>(zs.p), m->pts.p);
    if (hipStreamSynchronize(s) != hipSuccess) {
      ftz_msm_destroy(m);
      return set_err(FTZ_E_DEVICE, "point generation failed");
    }
  }
  rc = prepare_points(m);
  if (rc == FTZ_SUCCESS) rc = upload_scalars(m, scalars);
  if (rc != FTZ_SUCCESS) {
    ftz_msm_destroy(m);
    return rc;
  }
  *out = m;
  return FTZ_SUCCESS;
}

extern "C" int ftz_msm_set_scalars(ftz_msm* m, const uint8_t* scalars) {
  if (!m || !scalars) return set_err(FTZ_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(m->ctx->mu);
  HC(hipSetDevice(m->ctx->device));
  return upload_scalars(m, scalars);
}

// the pipeline after the sort keys, enqueued on s
static int msm_enqueue_tail(ftz_msm* m, hipStream_t s) {
  const MsmPlan& p = m->p;
  size_t wb = (size_t)p.rw * p.buckets;
  size_t wn = (size_t)p.windows * p.nv;
  int rc;
  if (m->csort) {
    // counting sort: end[] = the group counts from the keys kernel
    rc = scan(m->end_p, m->start_p, wb, m->tot.p, s);
    if (rc != FTZ_SUCCESS) return rc;
    k_msm_counts_scan<<<blocks(wb, 1024), 1024, 0, s>>>(p, nullptr, m->end_p, m->count.p, m->soff.p, m->tot.p);
    k_msm_scatter<<<blocks(p.n, 256), 256, 0, s>>>(p, m->key.p, m->val.p, m->start_p, m->end_p, m->perm.p);
  } else {
    // (window, bucket)-sorted point lists: stable radix sort, bucket ranges
    size_t tb = m->sort_tmp_bytes;
    HC(msm_sort(m, m->sort_tmp.p, tb, wn, s));
    HC(hipMemsetAsync(m->zb.p, 0, (2 * wb + 1024) * sizeof(uint32_t), s));  // start, end, histogram
    k_msm_bounds<<<blocks(wn, 256), 256, 0, s>>>(p, (uint64_t)wn, m->skey.p, m->perm.p, m->start_p, m->end_p);
    k_msm_counts_scan<<<blocks(wb, 1024), 1024, 0, s>>>(p, m->start_p, m->end_p, m->count.p, m->soff.p, m->tot.p);
  }
  // the slot-count scan's higher levels (its first level ran fused above)
  const uint32_t nb = (uint32_t)((wb + 1023) / 1024);
  if (nb > 1) {
    uint32_t* sums = m->tot.p + nb;
    rc = scan(m->tot.p, sums, nb, sums + nb + 1, s);
    if (rc != FTZ_SUCCESS) return rc;
    k_scan_add<<<nb, 1024, 0, s>>>(m->soff.p, (uint32_t)wb, sums);
  }
  k_msm_owner<<<blocks(wb, 256), 256, 0, s>>>(p, m->count.p, m->soff.p, m->owner.p, m->wlo.p, m->whi.p);
  // bucket slots in length order, then one lane per slot
  size_t sl = (size_t)p.rw * p.max_slots;
  if (m->csort) HC(hipMemsetAsync(m->lenhist_p, 0, 1024 * sizeof(uint32_t), s));
  k_msm_len_hist<<<blocks(sl, 256), 256, 0, s>>>(p, m->whi.p, m->owner.p, m->soff.p, m->count.p, m->lenhist_p);
  k_msm_len_scan<<<1, 1024, 0, s>>>(p, m->lenhist_p);
  k_msm_len_scatter<<<blocks(sl, 256), 256, 0, s>>>(p, m->whi.p, m->owner.p, m->soff.p, m->count.p,
                                                     m->lenhist_p, m->order.p);
  k_msm_bucket<<<blocks(sl, 128), 128, 0, s>>>(p, m->whi.p, m->order.p, m->owner.p, m->soff.p, m->start_p,
                                               m->count.p, m->perm.p, m->pts.p, m->slot_sum.p);
  k_msm_segment<<<blocks((size_t)p.rw * p.segs, MSM_SEG_PER_BLOCK), MSM_SEG_THREADS, 0, s>>>(p, 0, p.rw, m->wlo.p, m->whi.p,
                                                                       m->owner.p, m->slot_sum.p, m->part.p);
  // tree passes: segs -> ceil(segs / chunk) -> ... until one part per window
  // (host Horner) or at most HORNER_PARTS, which the Horner wave adds up itself
  // (quads in parallel)
  const uint32_t HORNER_PARTS = FTS_MSM_HOST_HORNER ? 1 : 8;
  G1JDev* bufs[2] = {m->tree.p, m->tree.p + (size_t)p.rw * ((p.segs + MSM_TREE_CHUNK - 1) / MSM_TREE_CHUNK)};
  const G1JDev* in = m->part.p;
  uint32_t cnt = p.segs;
  int which = 0;
  while (cnt > HORNER_PARTS) {
    uint32_t chunks = (cnt + MSM_TREE_CHUNK - 1) / MSM_TREE_CHUNK;
    G1JDev* out = bufs[which];
    k_msm_tree<<<p.rw * chunks, 256, 0, s>>>(in, cnt, out);
    in = out;
    which ^= 1;
    cnt = chunks;
  }
#if FTS_MSM_HOST_HORNER
  HC(hipMemcpyAsync(m->hwin, in, (size_t)p.rw * sizeof(G1JDev), hipMemcpyDeviceToHost, s));
#else
  k_msm_horner<<<1, 64, 0, s>>>(p, p.rw, 0, in, cnt, m->hacc.p);
#endif
  return FTZ_SUCCESS;
}

// The window combination sum_w 2^(c w) W_w on the host, from the rw window sums
// the pipeline read back (rw * 96 bytes): c (rw - 1) dependent doublings (120 at
// 2^16 and 2^20) are one serial chain whatever the device does, and a host core
// runs a doubling in 4x64-bit Montgomery limbs (FTS_HOST64) several times faster
// than one wave's latency-bound chain (k_msm_horner: 284-298 us per MSM,
// profiles/r06/msm_trace.txt) -- the split sppark's Pippenger also makes.  The
// affine result is unique, so the bytes are those of the device chain.
// Counted in last_ms.
static fts::g1j msm_horner_host(const MsmPlan& p, const G1JDev* win) {
  fts::g1j acc = fts::jac_inf<fts::fp>();
  bool started = false;
  for (int w = (int)p.rw - 1; w >= 0; w--) {
    if (started)
      for (uint32_t q = 0; q < p.c; q++) acc = fts::jac_dbl(acc);
    const fts::g1j x = fts::g1j_load(win[w]);
    if (!fts::is_zero(x.z)) {
      acc = fts::jac_add(acc, x);
      started = !fts::is_zero(acc.z);
    }
  }
  return acc;
}

// the result after the enqueued pipeline (event ev[0] recorded at its start)
static int msm_finish(ftz_msm* m, uint8_t out[64]) {
  hipStream_t s = m->ctx->stream;
  HC(hipEventRecord(m->ev[1], s));
  HC(hipGetLastError());
#if FTS_MSM_HOST_HORNER
  HC(hipStreamSynchronize(s));
  auto t0 = std::chrono::steady_clock::now();
  fts::g1j_to_raw(msm_horner_host(m->p, m->hwin), out);
#else
  G1JDev acc;
  HC(hipMemcpyAsync(&acc, m->hacc.p, sizeof(acc), hipMemcpyDeviceToHost, s));
  HC(hipStreamSynchronize(s));
  // affine conversion + RawBytes on the host (one inverse: a few microseconds
  // here, ~40k single-lane instructions on the device); counted in last_ms
  auto t0 = std::chrono::steady_clock::now();
  fts::g1j_to_raw(fts::g1j_load(acc), out);
#endif
  double host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  HC(hipEventElapsedTime(&m->last_ms, m->ev[0], m->ev[1]));
  m->last_ms += (float)host_ms;
  return FTZ_SUCCESS;
}

static int msm_enqueue_all(ftz_msm* m, hipStream_t s) {
  const MsmPlan& p = m->p;
  const uint32_t(*scal)[8] = reinterpret_cast<const uint32_t(*)[8]>(m->scal.p);
  if (m->csort) HC(hipMemsetAsync(m->end_p, 0, (size_t)p.rw * p.buckets * sizeof(uint32_t), s));
  k_msm_keys<<<blocks(p.n, 256), 256, 0, s>>>(p, scal, m->key.p, m->val.p, m->csort ? m->end_p : nullptr);
  return msm_enqueue_tail(m, s);
}

// capture keys .. Horner once (relaxed mode: the context's other threads may
// allocate meanwhile); on failure the handle keeps launching directly
static void msm_capture(ftz_msm* m, hipStream_t s) {
  m->graph_state = -1;
  if (hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  int rc = msm_enqueue_all(m, s);
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(s, &g);
  if (rc != FTZ_SUCCESS || e != hipSuccess || !g) {
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    return;
  }
  if (hipGraphInstantiate(&m->graph_exec, g, nullptr, nullptr, 0) != hipSuccess) {
    (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    m->graph_exec = nullptr;
    return;
  }
  m->graph = g;
  m->graph_state = 1;
}

extern "C" int ftz_msm_run(ftz_msm* m, uint8_t out[64]) {
  if (!m || !out) return set_err(FTZ_E_INVALID, "null argument");
  ftz_ctx* c = m->ctx;
  std::lock_guard<std::mutex> lk(c->mu);
  HC(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  if (m->graph_state == 0 && c->opt.msm_graph) msm_capture(m, s);
  HC(hipEventRecord(m->ev[0], s));
  if (m->graph_state == 1) {
    HC(hipGraphLaunch(m->graph_exec, s));
  } else {
    int rc = msm_enqueue_all(m, s);
    if (rc != FTZ_SUCCESS) return rc;
  }
  return msm_finish(m, out);
}

// ftz_msm_run with the scalars copied from host memory in RAW_CHUNKS pieces on a
// stream of the handle's own; the compute stream runs the key kernel of each
// piece as soon as its copy has landed.  last_ms spans the first copy to the
// result (events on both streams).
extern "C" int ftz_msm_run_scalars(ftz_msm* m, const uint8_t* scalars, uint8_t out[64]) {
  if (!m || !scalars || !out) return set_err(FTZ_E_INVALID, "null argument");
  ftz_ctx* c = m->ctx;
  std::lock_guard<std::mutex> lk(c->mu);
  HC(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const MsmPlan& p = m->p;
  if (!m->raw.p) HC(m->raw.alloc(32 * (size_t)p.n));
  if (!m->cstream) HC(hipStreamCreateWithFlags(&m->cstream, hipStreamNonBlocking));
  if (!m->cev_init) {
    for (int k = 0; k <= ftz_msm::RAW_CHUNKS; k++) HC(hipEventCreateWithFlags(&m->cev[k], hipEventDisableTiming));
    m->cev_init = true;
  }
  // the copies must not overwrite raw scalars a previous run still reads
  HC(hipEventRecord(m->cev[ftz_msm::RAW_CHUNKS], s));
  HC(hipStreamWaitEvent(m->cstream, m->cev[ftz_msm::RAW_CHUNKS], 0));
  HC(hipEventRecord(m->ev[0], m->cstream));
  uint32_t(*scal)[8] = reinterpret_cast<uint32_t(*)[8]>(m->scal.p);
  if (m->csort) HC(hipMemsetAsync(m->end_p, 0, (size_t)p.rw * p.buckets * sizeof(uint32_t), s));
  const uint32_t per = (p.n + ftz_msm::RAW_CHUNKS - 1) / ftz_msm::RAW_CHUNKS;
  for (int k = 0; k < ftz_msm::RAW_CHUNKS; k++) {
    uint32_t i0 = k * per, i1 = std::min<uint32_t>(p.n, i0 + per);
    if (i0 >= i1) break;
    HC(hipMemcpyAsync(m->raw.p + 32 * (size_t)i0, scalars + 32 * (size_t)i0, 32 * (size_t)(i1 - i0),
                      hipMemcpyHostToDevice, m->cstream));
    HC(hipEventRecord(m->cev[k], m->cstream));
    HC(hipStreamWaitEvent(s, m->cev[k], 0));
    k_msm_keys_raw<<<blocks(i1 - i0, 256), 256, 0, s>>>(p, i0, i1, m->raw.p, scal, m->key.p, m->val.p,
                                                        m->csort ? m->end_p : nullptr);
  }
  int rc = msm_enqueue_tail(m, s);
  if (rc != FTZ_SUCCESS) return rc;
  return msm_finish(m, out);
}

extern "C" int ftz_host_alloc(size_t bytes, void** out) {
  if (!out) return set_err(FTZ_E_INVALID, "null argument");
  *out = nullptr;
  if (!bytes) return FTZ_SUCCESS;
  if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) {
    *out = nullptr;
    return set_err(FTZ_E_NOMEM, "page-locked host allocation failed");
  }
  return FTZ_SUCCESS;
}

extern "C" void ftz_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

extern "C" int ftz_msm_info(const ftz_msm* m, float* last_ms, uint32_t* window_bits) {
  if (!m) return set_err(FTZ_E_INVALID, "null argument");
  if (last_ms) *last_ms = m->last_ms;
  if (window_bits) *window_bits = m->p.c;
  return FTZ_SUCCESS;
}

extern "C" void ftz_msm_destroy(ftz_msm* m) {
  if (!m) return;
  (void)hipSetDevice(m->ctx->device);
  if (m->ev_init)
  {
    for (int k = 0; k < 2; k++) (void)hipEventDestroy(m->ev[k]);
  }
  if (m->cev_init)
    for (int k = 0; k <= ftz_msm::RAW_CHUNKS; k++) (void)hipEventDestroy(m->cev[k]);
  if (m->cstream) {
    (void)hipStreamSynchronize(m->cstream);
    (void)hipStreamDestroy(m->cstream);
  }
  if (m->graph_exec) (void)hipGraphExecDestroy(m->graph_exec);
  if (m->hwin) (void)hipHostFree(m->hwin);
  if (m->graph) (void)hipGraphDestroy(m->graph);
  delete m;
}

// gnark SetBytes check of n 64-byte slots on the context's device (rt_internal.h)
// gnark SetBytes checks of n 64-byte slots on the device, on a stream and
// grow-only buffers of their own: a check never waits on the job engine's
// batches (no hipMalloc / hipFree per call) nor on MSM / setup work
int g1_check_slots(ftz_ctx* c, size_t n, const uint8_t* slots, uint8_t* ok) {
  if (!n) return FTZ_SUCCESS;
  if (n > (1u << 26)) return set_err(FTZ_E_INVALID, "too many elements in one check");
  std::lock_guard<std::mutex> lk(c->chk_mu);
  HC(hipSetDevice(c->device));
  if (!c->chk_stream) HC(hipStreamCreateWithFlags(&c->chk_stream, hipStreamNonBlocking));
  hipStream_t s = c->chk_stream;
  HC(c->chk_h.reserve(65 * n));
  HC(c->chk_d.reserve(65 * n));
  memcpy(c->chk_h.p, slots, 64 * n);
  HC(hipMemcpyAsync(c->chk_d.p, c->chk_h.p, 64 * n, hipMemcpyHostToDevice, s));
  k_g1_check<<<blocks(n, 256), 256, 0, s>>>((uint32_t)n, c->chk_d.p, c->chk_d.p + 64 * n);
  HC(hipGetLastError());
  HC(hipMemcpyAsync(c->chk_h.p + 64 * n, c->chk_d.p + 64 * n, n, hipMemcpyDeviceToHost, s));
  HC(hipStreamSynchronize(s));
  memcpy(ok, c->chk_h.p + 64 * n, n);
  return FTZ_SUCCESS;
}

extern "C" int ftz_g1_sum(ftz_ctx* c, size_t n, const uint8_t* points, uint8_t out[64]) {
  if (!c || !out || (n && !points)) return set_err(FTZ_E_INVALID, "null argument");
  if (n > 4096) return set_err(FTZ_E_INVALID, "ftz_g1_sum takes at most 4096 points");
  std::lock_guard<std::mutex> lk(c->mu);
  HC(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  DBuf<uint8_t> buf;
  HC(buf.alloc(64 * n + 64 + 16));
  uint8_t* d_out = buf.p + 64 * n;
  uint32_t* d_status = reinterpret_cast<uint32_t*>(buf.p + 64 * n + 64);
  if (n) HC(hipMemcpyAsync(buf.p, points, 64 * n, hipMemcpyHostToDevice, s));
  k_g1_sum<<<1, 64, 0, s>>>((uint32_t)n, buf.p, d_out, d_status);
  HC(hipGetLastError());
  uint8_t res[64 + 16];
  HC(hipMemcpyAsync(res, d_out, sizeof(res), hipMemcpyDeviceToHost, s));
  HC(hipStreamSynchronize(s));
  uint32_t st;
  memcpy(&st, res + 64, 4);
  if (st != n) return set_err(FTZ_E_INVALID, "point " + std::to_string(st) + " is not a canonical BN254 G1 point");
  memcpy(out, res, 64);
  return FTZ_SUCCESS;
}

extern "C" int ftz_msm_g1(ftz_ctx* c, size_t n, const uint8_t* points, const uint8_t* scalars, uint8_t out[64]) {
  ftz_msm* m = nullptr;
  int rc = ftz_msm_load(c, n, points, scalars, &m);
  if (rc == FTZ_SUCCESS) rc = ftz_msm_run(m, out);
  ftz_msm_destroy(m);
  return rc;
}

// ftsamd: HIP runtime + C ABI (include/ftsamd.h) -- contexts, batch slots and
// the staged batch / prover API.  The job engine behind ftz_verify_* is in
// engine.hip, the standalone MSM in msm_rt.hip.
//
// One context per GPU holds the public parameters in device form: fixed-base
// tables for Ped0..2, PedGen, the G1 generator and PK0..2, Q; the precomputed
// Miller lines of Q; and the canonical RawBytes of the PP points that every
// transcript hashes.  A batch is planned on host threads (host/planner.cpp)
// straight into a pinned staging blob, copied to the device in ONE transfer,
// and executed as a fixed sequence of job kernels on the batch's own three
// HIP streams (see dev/jobs.h for the job model).
#include <hip/hip_runtime.h>

#include <chrono>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ftsamd.h"
#include "dev/jobs.h"
#include "host/planner.h"
#include "launch.h"

using namespace fts;
using namespace ftsh;

#include "rt_internal.h"

thread_local std::string g_err;
int set_err(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

static int blocks_for(uint32_t n, int bs) { return (int)((n + bs - 1) / bs); }

extern "C" const char* ftz_last_error(void) { return g_err.c_str(); }

extern "C" void ftz_options_default(ftz_options* o) {
  if (!o) return;
  memset(o, 0, sizeof(*o));
  o->struct_size = sizeof(ftz_options);
  o->batch = 8192;
  o->slots = 4;
  o->window_us = 1000;
  o->threads = 0;
  o->fexp = FTZ_FEXP_EXACT;
  o->hold_inflight = 2;
  o->small_pass = 4096;
  o->first_pass = 4096;
  o->msm_glv = 1;
  o->prover_tables = 1;
  o->msm_graph = 0;
}

extern "C" int ftz_ctx_create(const uint8_t* pp, size_t pp_len, int device, ftz_ctx** out) {
  return ftz_ctx_create_ex(pp, pp_len, device, nullptr, out);
}

extern "C" int ftz_ctx_create_ex(const uint8_t* pp, size_t pp_len, int device, const ftz_options* opt,
                                 ftz_ctx** out) {
  if (!pp || !out) return set_err(FTZ_E_INVALID, "null argument");
  *out = nullptr;
  ftz_options o;
  ftz_options_default(&o);
  if (opt) {
    if (opt->struct_size != sizeof(ftz_options)) return set_err(FTZ_E_INVALID, "ftz_options.struct_size mismatch");
    o = *opt;
    if (o.batch == 0) o.batch = 8192;
    if (o.slots == 0) o.slots = 4;
    if (o.fexp != FTZ_FEXP_EXACT && o.fexp != FTZ_FEXP_FUENTES) return set_err(FTZ_E_INVALID, "unknown fexp variant");
    if (o.batch > (1u << 20) || o.slots > 64) return set_err(FTZ_E_INVALID, "batch / slots out of range");
    if (o.msm_window_bits > 24) return set_err(FTZ_E_INVALID, "msm_window_bits out of range (0..24)");
    if (o.msm_glv > 1 || o.msm_precompute > 1 || o.prover_tables > 1 || o.msm_graph > 1)
      return set_err(FTZ_E_INVALID, "msm_glv / msm_precompute / prover_tables / msm_graph must be 0 or 1");
    if (o.request_threads > 1024) return set_err(FTZ_E_INVALID, "request_threads out of range (0..1024)");
    if (o.msm_radix_bits && o.msm_radix_bits != 8 && o.msm_radix_bits != 9)
      return set_err(FTZ_E_INVALID, "msm_radix_bits must be 0, 8 or 9");
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return set_err(FTZ_E_DEVICE, "no HIP device available (ftsamd requires an MI355X / gfx950 GPU)");
  if (device < 0 || device >= ndev) return set_err(FTZ_E_DEVICE, "device ordinal out of range");
  HC(hipSetDevice(device));
  hipDeviceProp_t prop;
  HC(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return set_err(FTZ_E_DEVICE, std::string("unsupported GPU architecture ") + prop.gcnArchName +
                                     " (code objects are built for gfx950)");
  ftz_ctx* c = new ftz_ctx();
  c->device = device;
  c->opt = o;
  unsigned hc = std::thread::hardware_concurrency();
  int threads = o.threads ? (int)o.threads : (int)std::max(1u, std::min(16u, hc ? hc : 8u));
  c->opt.threads = (uint32_t)threads;
  c->pool = new WorkPool(threads);
  std::string e = parse_pp(pp, pp_len, "zkatdlog", c->pp);
  if (!e.empty()) {
    ftz_ctx_destroy(c);
    return set_err(FTZ_E_PP, e);
  }
  c->pp_var = c->pp;
  c->pp_var.no_sigtab = true;
  c->pp_var.fixed_pairs = false;
  int prio_lo = 0, prio_hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  if (hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, prio_hi) != hipSuccess) {
    ftz_ctx_destroy(c);
    return set_err(FTZ_E_DEVICE, "hipStreamCreate failed");
  }
  // at most 4 triples (13 streams with the context's own: fits 16 hardware
  // queues); engine slots beyond that share them round-robin, i.e. are planned
  // ahead and queue behind the batch 4 slots earlier
  for (uint32_t k = 0; k < std::min<uint32_t>(c->opt.slots, 4); k++) {
    std::array<hipStream_t, 3> t{};
    bool ok = hipStreamCreateWithPriority(&t[0], hipStreamNonBlocking, prio_hi) == hipSuccess &&
              hipStreamCreateWithPriority(&t[1], hipStreamNonBlocking, prio_lo) == hipSuccess &&
              hipStreamCreateWithPriority(&t[2], hipStreamNonBlocking, prio_hi) == hipSuccess;
    c->triples.push_back(t);
    if (!ok) {
      ftz_ctx_destroy(c);
      return set_err(FTZ_E_DEVICE, "hipStreamCreate failed");
    }
  }
  // decode PP points on the GPU: G1 [PedGen, Ped0, Ped1, Ped2, G1 generator], G2 [PK0, PK1, PK2, Q]
  std::vector<uint8_t> raw;
  std::vector<uint32_t> g1off, g2off;
  auto push = [&](const std::vector<uint8_t>& v, size_t need, std::vector<uint32_t>& offs) {
    offs.push_back((uint32_t)raw.size());
    std::vector<uint8_t> t = v;
    t.resize(std::max(need, v.size()), 0);
    raw.insert(raw.end(), t.begin(), t.end());
  };
  push(c->pp.pedgen, 64, g1off);
  for (int k = 0; k < 3; k++) push(c->pp.ped[k], 64, g1off);
  std::vector<uint8_t> gen(64, 0);
  gen[31] = 1;
  gen[63] = 2;
  push(gen, 64, g1off);
  for (int k = 0; k < 3; k++) push(c->pp.pk[k], 128, g2off);
  push(c->pp.q, 128, g2off);
  // SignedValues (setup.go:168-184): decoded to check Validate's point rules
  size_t nsig = c->pp.sig_r.size();
  for (size_t k = 0; k < nsig; k++) {
    push(c->pp.sig_r[k], 64, g1off);
    push(c->pp.sig_s[k], 64, g1off);
  }
  raw.resize(raw.size() + 128, 0);
  const uint32_t n1 = (uint32_t)g1off.size();
  DBuf<uint8_t> d_raw, d_g1b, d_g2b, d_ok;
  DBuf<uint32_t> d_g1off, d_g2off;
  DBuf<G1Dev> d_g1;
  DBuf<G2Dev> d_g2;
  int rc = FTZ_SUCCESS;
  auto fail = [&](int code, const std::string& m) {
    rc = set_err(code, m);
    return rc;
  };
  do {
    if (d_raw.upload(raw, c->stream) != hipSuccess || d_g1off.upload(g1off, c->stream) != hipSuccess ||
        d_g2off.upload(g2off, c->stream) != hipSuccess || d_g1.alloc(n1) != hipSuccess ||
        d_g2.alloc(4) != hipSuccess || d_g1b.alloc(64 * (size_t)n1) != hipSuccess ||
        d_g2b.alloc(128 * 4) != hipSuccess || d_ok.alloc(n1 + 4) != hipSuccess) {
      fail(FTZ_E_NOMEM, "device allocation failed");
      break;
    }
    k_pp_decode<<<blocks_for(n1 + 4, 64), 64, 0, c->stream>>>(d_raw.p, d_g1off.p, n1, d_g2off.p, 4, d_g1.p, d_g2.p,
                                                               d_g1b.p, d_g2b.p, d_ok.p);
    std::vector<uint8_t> ok(n1 + 4);
    std::vector<uint8_t> g1b(64 * (size_t)n1), g2b(128 * 4);
    if (hipMemcpyAsync(ok.data(), d_ok.p, ok.size(), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipMemcpyAsync(g1b.data(), d_g1b.p, g1b.size(), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipMemcpyAsync(g2b.data(), d_g2b.p, g2b.size(), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
      fail(FTZ_E_DEVICE, std::string("public-parameter decode failed: ") + hipGetErrorString(hipGetLastError()));
      break;
    }
    bool allok = true;
    for (size_t k = 0; k < ok.size(); k++) allok = allok && ok[k];
    if (!allok) {
      fail(FTZ_E_PP, "public parameters hold an invalid curve point");
      break;
    }
    c->pp_g2.resize(4);
    if (hipMemcpy(c->pp_g2.data(), d_g2.p, 4 * sizeof(G2Dev), hipMemcpyDeviceToHost) != hipSuccess) {
      fail(FTZ_E_DEVICE, "copy failed");
      break;
    }
    c->const_bytes.assign(C_SIZE, 0);
    memcpy(&c->const_bytes[C_PEDGEN], &g1b[0], 64);
    memcpy(&c->const_bytes[C_PED0], &g1b[64], 192);
    memcpy(&c->const_bytes[C_Q_PK], &g2b[384], 128);        // Q
    memcpy(&c->const_bytes[C_Q_PK + 128], &g2b[0], 384);    // PK0..2
    memcpy(&c->const_bytes[C_PK_Q + 384], &g2b[384], 128);  // Q again (PK0..2 shared)
    // fixed-base tables: G1 base order must follow G1Base: PED0, PED1, PED2, PEDGEN, GEN
    std::vector<G1Dev> hb(5);
    std::vector<G1Dev>& got = c->pp_g1;  // kept: the prover's signature-point tables (g1tab_p)
    got.resize(n1);
    if (hipMemcpy(got.data(), d_g1.p, n1 * sizeof(G1Dev), hipMemcpyDeviceToHost) != hipSuccess) {
      fail(FTZ_E_DEVICE, "copy failed");
      break;
    }
    hb[G1B_PED0] = got[1];
    hb[G1B_PED1] = got[2];
    hb[G1B_PED2] = got[3];
    hb[G1B_PEDGEN] = got[0];
    hb[G1B_GEN] = got[4];
    DBuf<G1Dev> d_b1;
    if (d_b1.upload(hb, c->stream) != hipSuccess) {
      fail(FTZ_E_NOMEM, "alloc");
      break;
    }
    uint32_t t1 = G1B_COUNT * G1TAB_WINDOWS * G1TAB_DIGITS, t2 = G2B_COUNT * G2TAB_WINDOWS * G2TAB_DIGITS;
    if (c->g1tab.alloc(t1) != hipSuccess || c->g2tab.alloc(t2) != hipSuccess ||
        c->qlines.alloc(MILLER_LINES) != hipSuccess || c->qlines29.alloc(MILLER_LINES) != hipSuccess ||
        c->qlines29n.alloc(MILLER_LINES) != hipSuccess) {
      fail(FTZ_E_NOMEM, "table allocation failed");
      break;
    }
    DBuf<G1Dev> d_bw;
    DBuf<G1JDev> d_jt;
    DBuf<uint32_t> d_zs;
    if (G1TAB_C <= 8) {
      k_tab_g1<<<blocks_for(t1, 64), 64, 0, c->stream>>>(d_b1.p, t1, c->g1tab.p);
    } else {
      const uint32_t chunk = 128, lanes = G1B_COUNT * G1TAB_WINDOWS * (G1TAB_DIGITS / chunk);
      if (d_bw.alloc(G1B_COUNT * G1TAB_WINDOWS) != hipSuccess || d_jt.alloc(t1) != hipSuccess ||
          d_zs.alloc(8 * (size_t)t1) != hipSuccess) {
        fail(FTZ_E_NOMEM, "table scratch allocation failed");
        break;
      }
      k_tab_g1_bw<<<blocks_for(G1B_COUNT * G1TAB_WINDOWS, 64), 64, 0, c->stream>>>(d_b1.p, G1B_COUNT, d_bw.p);
      k_tab_g1_fill<<<blocks_for(lanes, 128), 128, 0, c->stream>>>(
          d_bw.p, G1B_COUNT, chunk, d_jt.p, reinterpret_cast<uint32_t (*)[8]>(d_zs.p), c->g1tab.p);
    }
    DBuf<G2Dev> d_bw2;
    DBuf<uint32_t> d_jt2, d_zs2;
    if (G2TAB_C <= 8) {
      k_tab_g2<<<blocks_for(t2, 64), 64, 0, c->stream>>>(d_g2.p, t2, c->g2tab.p);  // PK0, PK1, PK2, Q
    } else {
      const uint32_t chunk = 64, lanes = G2B_COUNT * G2TAB_WINDOWS * (G2TAB_DIGITS / chunk);
      if (d_bw2.alloc(G2B_COUNT * G2TAB_WINDOWS) != hipSuccess || d_jt2.alloc(48 * (size_t)t2) != hipSuccess ||
          d_zs2.alloc(16 * (size_t)t2) != hipSuccess) {
        fail(FTZ_E_NOMEM, "table scratch allocation failed");
        break;
      }
      k_tab_g2_bw<<<blocks_for(G2B_COUNT * G2TAB_WINDOWS, 64), 64, 0, c->stream>>>(d_g2.p, d_bw2.p);
      k_tab_g2_fill<<<blocks_for(lanes, 128), 128, 0, c->stream>>>(
          d_bw2.p, chunk, reinterpret_cast<uint32_t (*)[48]>(d_jt2.p), reinterpret_cast<uint32_t (*)[16]>(d_zs2.p),
          c->g2tab.p);
    }
    DBuf<int> d_n;
    if (d_n.alloc(2) != hipSuccess) {
      fail(FTZ_E_NOMEM, "alloc");
      break;
    }
    k_qlines<<<1, 64, 0, c->stream>>>(d_g2.p + 3, c->qlines.p, c->qlines29.p, c->qlines29n.p, d_n.p, d_n.p + 1);
    int nl[2] = {0, 0};
    if (hipMemcpyAsync(nl, d_n.p, 2 * sizeof(int), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess || nl[0] != MILLER_LINES) {
      fail(FTZ_E_DEVICE, std::string("context setup kernels failed: ") + hipGetErrorString(hipGetLastError()));
      break;
    }
    c->qnorm = nl[1] != 0;
  } while (0);
  if (rc != FTZ_SUCCESS) {
    ftz_ctx_destroy(c);
    return rc;
  }
  *out = c;
  return FTZ_SUCCESS;
}

extern "C" void ftz_ctx_destroy(ftz_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  engine_destroy(c);
  for (ftz_prover* p : c->pslots) {
    slot_free(p);
    delete p;
  }
  c->pslots.clear();
  if (c->aux) {
    slot_free(c->aux);
    delete c->aux;
    c->aux = nullptr;
  }
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto& t : c->triples)
    for (hipStream_t x : t)
      if (x) {
        (void)hipStreamSynchronize(x);
        (void)hipStreamDestroy(x);
      }
  c->triples.clear();
  c->g1tab.alloc(0);
  c->g2tab.alloc(0);
  c->qlines.alloc(0);
  c->qlines29.alloc(0);
  c->qlines29n.alloc(0);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->chk_stream) {
    (void)hipStreamSynchronize(c->chk_stream);
    (void)hipStreamDestroy(c->chk_stream);
  }
  delete c->pool;
  delete c->req_pool;
  delete c;
}

extern "C" int ftz_ctx_set_threads(ftz_ctx* c, int threads) {
  if (!c || threads < 1 || threads > 256) return set_err(FTZ_E_INVALID, "bad argument");
  std::lock_guard<std::mutex> lk(c->eng_mu);
  if (c->eng) return set_err(FTZ_E_INVALID, "ftz_ctx_set_threads: the context's engine is already running");
  delete c->pool;
  c->pool = new WorkPool(threads);
  c->opt.threads = (uint32_t)threads;
  return FTZ_SUCCESS;
}

extern "C" int ftz_ctx_set_serial(ftz_ctx* c, int serial) {
  if (!c) return set_err(FTZ_E_INVALID, "null context");
  c->serial = serial ? 1 : 0;
  return FTZ_SUCCESS;
}

extern "C" int ftz_ctx_debug_poison(ftz_ctx* c, const uint8_t* proof) {
  if (!c) return set_err(FTZ_E_INVALID, "null context");
  c->debug_poison.store(proof);
  return FTZ_SUCCESS;
}

extern "C" int ftz_ctx_set_debug(ftz_ctx* c, int flags) {
  if (!c) return set_err(FTZ_E_INVALID, "null context");
  if (flags & ~FTZ_DEBUG_CHALLENGES) return set_err(FTZ_E_INVALID, "unknown debug flag");
  c->pp.debug_challenges = (flags & FTZ_DEBUG_CHALLENGES) != 0;
  return FTZ_SUCCESS;
}

extern "C" int ftz_ctx_set_layout(ftz_ctx* c, int stage, int layout) {
  if (!c) return set_err(FTZ_E_INVALID, "null context");
  if (layout != FTZ_LAYOUT_ONE_LANE && layout != FTZ_LAYOUT_SEXTET) return set_err(FTZ_E_INVALID, "unknown layout");
  if (stage == FTZ_STAGE_G2LINES) {
    c->g2lanes = layout;
    c->g2lanes_set = true;
  }
  else if (stage == FTZ_STAGE_PROVER_G2LINES)
    c->g2lanes_prover = layout;
  else
    return set_err(FTZ_E_INVALID, "unknown stage");
  return FTZ_SUCCESS;
}

extern "C" int ftz_pp_validate(const uint8_t* pp, size_t pp_len) {
  if (!pp) return set_err(FTZ_E_INVALID, "null argument");
  std::string e = validate_pp(pp, pp_len, "zkatdlog");
  return e.empty() ? FTZ_SUCCESS : set_err(FTZ_E_PP, e);
}

extern "C" int ftz_ctx_options(const ftz_ctx* c, ftz_options* out) {
  if (!c || !out) return set_err(FTZ_E_INVALID, "null argument");
  *out = c->opt;
  return FTZ_SUCCESS;
}

extern "C" int ftz_ctx_info(const ftz_ctx* c, uint32_t* base, uint32_t* exponent) {
  if (!c) return set_err(FTZ_E_INVALID, "null context");
  if (base) *base = c->pp.base;
  if (exponent) *exponent = (uint32_t)c->pp.exponent;
  return FTZ_SUCCESS;
}

// ------------------------------------------------------------------ batch slots
int slot_init(ftz_batch* b) {
  if (b->st[0]) return FTZ_SUCCESS;
  // the next of the context's shared stream triples (pairing chain and G2 /
  // line jobs high priority, side G1 jobs -- which fill the SIMDs the chain
  // leaves idle -- low)
  ftz_ctx* c = b->ctx;
  const auto& t = c->triples[c->next_triple.fetch_add(1) % c->triples.size()];
  for (int k = 0; k < 3; k++) b->st[k] = t[k];
  for (int k = 0; k < 20; k++)
    HC(hipEventCreateWithFlags(&b->ev[k], k == 17 ? (hipEventBlockingSync | hipEventDisableTiming) : 0));
  b->ev_init = true;
  return FTZ_SUCCESS;
}

void slot_free(ftz_batch* b) {
  if (!b) return;
  // the streams are the context's: wait for this slot's last submission only
  if (b->ev_init && b->pending) (void)hipEventSynchronize(b->ev[17]);
  b->pending = false;
  if (b->ev_init)
    for (int k = 0; k < 20; k++) (void)hipEventDestroy(b->ev[k]);
  b->ev_init = false;
  b->st[0] = b->st[1] = b->st[2] = nullptr;
}

static void scratch_layout(ftz_batch* b) {
  const FlatPlan& f = b->fp;
  ScratchLayout& s = b->sl;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    size_t r = o;
    o = (o + std::max<size_t>(bytes, 1) + 255) & ~(size_t)255;
    return r;
  };
  size_t n_pr = f.cnt[PS_PR], n_g1 = f.cnt[PS_G1], n_g1p = f.cnt[PS_G1P];
  s.pts = take(sizeof(G1Dev) * (size_t)f.n_pts);
  s.pt_ok = take(f.n_pts);
  s.scal = take(32 * (size_t)f.n_scal);
  s.canon = take(f.n_scal);
  s.g1out = take(sizeof(G1Dev) * (size_t)f.n_g1out);
  s.pnorm = take(sizeof(G1Dev) * (size_t)f.n_g1out);
  s.g2out = take(sizeof(G2Dev) * (size_t)f.n_g2out);
  s.fbuf = take(sizeof(F12Dev) * n_pr);
  s.fxpark = take(fexp_park_bytes(n_pr));
  s.lines2 = take(sizeof(EvLineDev) * n_pr * MILLER_LINES);
  s.part1 = take(sizeof(G1JDev) * 4 * n_g1);
  s.part1p = take(sizeof(G1JDev) * 4 * n_g1p);
  s.part2 = take(sizeof(G2PartDev) * 4 * n_pr);
  s.vtab1 = take(sizeof(G1Dev) * 16 * n_g1);
  s.vtab1p = take(sizeof(G1Dev) * 16 * n_g1p);
  s.hash_ok = take(f.cnt[PS_HMAIN]);
  s.hash_ok_pre = take(f.cnt[PS_HPRE]);
  s.codes = take(sizeof(int32_t) * b->n);
  s.bitmap = take(sizeof(uint32_t) * ((b->n + 31) / 32 + 1));
  s.total = o;
}

// Flattened plan -> pinned staging blob; device blob and scratch sized.
static int slot_finish_plan(ftz_batch* b, size_t n, bool p2_g1out) {
  ftz_ctx* c = b->ctx;
  std::string e = flat_layout(b->work, p2_g1out, b->fp);
  if (!e.empty()) return set_err(FTZ_E_INVALID, e);
  if (b->fp.n_items != n) return set_err(FTZ_E_INVALID, "planner: item count mismatch");
  const bool fixed3 = p2_g1out && c->pp.fixed_pairs && c->ptab_ready;  // the prover's pairings take no G2 jobs
  if (!fixed3 && b->fp.cnt[PS_G2] != b->fp.cnt[PS_PR])
    return set_err(FTZ_E_INVALID, "planner: G2 and pairing jobs out of step");
  b->n = n;
  HC(b->h_blob.reserve(b->fp.bytes));
  flat_write(b->work, b->fp, b->h_blob.p, c->const_bytes.data(), *c->pool);
  // pairing job i consumes G2 job i's output (k_g2lines computes both)
  const PairJob* pr = b->fp.ptr<PairJob>(b->h_blob.p, PS_PR);
  const G2Job* g2 = b->fp.ptr<G2Job>(b->h_blob.p, PS_G2);
  for (size_t i = 0; i < b->fp.cnt[PS_PR]; i++)
    if (fixed3 ? (pr[i].q2 != NONE || pr[i].p3 == NONE) : pr[i].q2 != g2[i].out)
      return set_err(FTZ_E_INVALID, "planner: G2 and pairing jobs out of step");
  scratch_layout(b);
  HC(b->d_blob.reserve(b->fp.bytes));
  HC(b->d_scr.reserve(b->sl.total));
  size_t res = ((n * sizeof(int32_t) + 255) & ~(size_t)255) + b->fp.cnt[PS_OUT] + 256;
  HC(b->h_res.reserve(res));
  return FTZ_SUCCESS;
}

int slot_plan_items(ftz_batch* b, size_t n, const PlanItem* items) {
  if (const uint8_t* poison = b->ctx->debug_poison.load())
    for (size_t i = 0; i < n; i++)
      if ((items[i].kind == 0 && items[i].t.proof == poison) || (items[i].kind == 1 && items[i].i.proof == poison))
        return set_err(FTZ_E_INVALID, "poisoned item (ftz_ctx_debug_poison)");
  plan_items(b->ctx->pp, n, items, b->work, *b->ctx->pool);
  return slot_finish_plan(b, n, false);
}

// The prover's G1 table set (ftz_ctx.g1tab_p): g1tab's bases, then R_d, S_d of
// every digit (PP SignedValues), 32 MB per base with 16-bit windows (6.4 GB
// for b = 100), built once -- in groups of 16 bases, the same kernels as g1tab
// -- on the first proving call of a context whose PP qualify (pp_sig_tables)
// and whose ftz_options.prover_tables is 1.  When the tables cannot be
// allocated the context records it once and proves on the variable-base path
// (prover_plan plans with pp_var), as it does with prover_tables = 0.
static int ensure_prover_tables(ftz_ctx* c) {
  std::lock_guard<std::mutex> lk(c->ptab_mu);
  if (c->ptab_ready || c->ptab_failed || !c->opt.prover_tables || !pp_sig_tables(c->pp)) return FTZ_SUCCESS;
  HC(hipSetDevice(c->device));
  const uint32_t nsig = 2 * c->pp.base, nb = G1B_SIG0 + nsig;
  const size_t per = (size_t)G1TAB_WINDOWS * G1TAB_DIGITS;
  if (c->pp_g1.size() != G1B_COUNT + (size_t)nsig) return set_err(FTZ_E_PP, "signature points not decoded");
  if (c->g1tab_p.alloc(nb * per) != hipSuccess) {
    (void)hipGetLastError();  // clear the sticky allocation error
    (void)c->g1tab_p.alloc(0);
    c->ptab_failed = true;
    return FTZ_SUCCESS;
  }
  hipStream_t s = c->stream;
  HC(hipMemcpyAsync(c->g1tab_p.p, c->g1tab.p, G1B_COUNT * per * sizeof(G1Dev), hipMemcpyDeviceToDevice, s));
  std::vector<G1Dev> sig(c->pp_g1.begin() + G1B_COUNT, c->pp_g1.end());  // R_0, S_0, R_1, S_1, ...
  DBuf<G1Dev> d_b;
  HC(d_b.upload(sig, s));
  if (G1TAB_C <= 8) {
    const uint32_t t = (uint32_t)(nsig * per);
    k_tab_g1<<<blocks_for(t, 64), 64, 0, s>>>(d_b.p, t, c->g1tab_p.p + G1B_COUNT * per);
  } else {
    const uint32_t group = 16, chunk = 128;
    DBuf<G1Dev> d_bw;
    DBuf<G1JDev> d_jt;
    DBuf<uint32_t> d_zs;
    if (d_bw.alloc(group * G1TAB_WINDOWS) != hipSuccess || d_jt.alloc(group * per) != hipSuccess ||
        d_zs.alloc(8 * group * per) != hipSuccess)
      return set_err(FTZ_E_NOMEM, "prover table scratch allocation failed");
    for (uint32_t g = 0; g < nsig; g += group) {
      const uint32_t m = std::min(group, nsig - g), lanes = m * G1TAB_WINDOWS * (G1TAB_DIGITS / chunk);
      k_tab_g1_bw<<<blocks_for(m * G1TAB_WINDOWS, 64), 64, 0, s>>>(d_b.p + g, m, d_bw.p);
      k_tab_g1_fill<<<blocks_for(lanes, 128), 128, 0, s>>>(d_bw.p, m, chunk, d_jt.p,
                                                           reinterpret_cast<uint32_t (*)[8]>(d_zs.p),
                                                           c->g1tab_p.p + (G1B_COUNT + g) * per);
    }
    HC(hipGetLastError());
    HC(hipStreamSynchronize(s));  // the scratch buffers go out of scope
  }
  if (c->pp.fixed_pairs) {  // PK1, PK2 lines for k_miller_f3 (the host planner checked r0 != 0)
    if (!c->qnorm) return set_err(FTZ_E_PP, "fixed-pair prover needs normalisable Q lines");
    DBuf<G2Dev> d_q;
    DBuf<LineCoef> d_l;
    DBuf<LineCoef29> d_l29;
    DBuf<int> d_n;
    std::vector<G2Dev> pk = {c->pp_g2[G2B_PK1], c->pp_g2[G2B_PK2]};
    if (d_q.upload(pk, s) != hipSuccess || d_l.alloc(MILLER_LINES) != hipSuccess ||
        d_l29.alloc(MILLER_LINES) != hipSuccess || d_n.alloc(4) != hipSuccess ||
        c->pklines29n.alloc(2 * MILLER_LINES) != hipSuccess)
      return set_err(FTZ_E_NOMEM, "prover line allocation failed");
    for (int t = 0; t < 2; t++)
      k_qlines<<<1, 64, 0, s>>>(d_q.p + t, d_l.p, d_l29.p, c->pklines29n.p + t * MILLER_LINES, d_n.p + 2 * t,
                                d_n.p + 2 * t + 1);
    int nl[4] = {0, 0, 0, 0};
    HC(hipMemcpyAsync(nl, d_n.p, sizeof(nl), hipMemcpyDeviceToHost, s));
    HC(hipStreamSynchronize(s));
    if (nl[0] != MILLER_LINES || nl[2] != MILLER_LINES || !nl[1] || !nl[3])
      return set_err(FTZ_E_PP, "PK1 / PK2 lines are not normalisable");
  }
  HC(hipGetLastError());
  HC(hipStreamSynchronize(s));
  c->ptab_ready = true;
  return FTZ_SUCCESS;
}

// fixed-base tables the prover's G1 jobs index (G1B_SIG0 .. only with g1tab_p)
static const G1Dev* prover_g1tab(ftz_ctx* c) { return c->ptab_ready ? c->g1tab_p.p : c->g1tab.p; }

int prover_plan(ftz_batch* b, size_t n, const void* wit, int kind) {
  ftz_ctx* c = b->ctx;
  int trc = ensure_prover_tables(c);
  if (trc != FTZ_SUCCESS) return trc;
  const PPInfo& pp = c->ptab_ready ? c->pp : c->pp_var;  // the table set's bases only when it exists
  std::string e = kind == 0
                      ? plan_prove_items_transfers(pp, n, static_cast<const TransferWit*>(wit), b->work, *c->pool)
                      : plan_prove_items_issues(pp, n, static_cast<const IssueWit*>(wit), b->work, *c->pool);
  if (!e.empty()) return set_err(FTZ_E_INVALID, e);
  return slot_finish_plan(b, n, true);
}

// Device pointers of a slot (blob sections + scratch).
struct SlotPtrs {
  uint8_t *wire, *arena, *out;
  const DecodeJob* dec;
  const ZrJob* zr;
  const ScalJob *sc, *sc1, *sc_post;
  const uint32_t* sclist;
  const VTerm* vt;
  const G1Job *g1, *g1p;
  const G2Job* g2;
  const PairJob* pr;
  const Seg* seg;
  const HashJob *hpre, *hmain;
  const Check* ck;
  const TxChecks* tx;
  const RandJob* rnd;
  const EmitJob* emit;
  const B64Job* b64;
  const CopyJob *cp, *cp2;
  G1Dev* pts;
  uint8_t *pt_ok, *canon, *hash_ok, *hash_ok_pre;
  uint32_t (*scal)[8];
  G1Dev* g1out;
  G1Dev* pnorm;
  G2Dev* g2out;
  F12Dev* fbuf;
  int32_t* fxpark;
  EvLineDev* lines2;
  G1JDev *part1, *part1p;
  G2PartDev* part2;
  G1Dev *vtab1, *vtab1p;
  int32_t* codes;
  uint32_t* bitmap;
  uint32_t n_dec, n_zr, n_sc, n_sc1, n_sp, n_rnd, n_em, n_b64, n_g1, n_g1p, n_g2, n_pr, n_hp, n_hm, n_tx, n_cp, n_cp2;
};

static SlotPtrs slot_ptrs(ftz_batch* b) {
  SlotPtrs p;
  const FlatPlan& f = b->fp;
  uint8_t* d = b->d_blob.p;
  uint8_t* s = b->d_scr.p;
  p.wire = d + f.off[PS_WIRE];
  p.arena = d + f.off[PS_ARENA];
  p.out = d + f.off[PS_OUT];
  p.dec = f.ptr<DecodeJob>(d, PS_DEC);
  p.zr = f.ptr<ZrJob>(d, PS_ZR);
  p.sc = f.ptr<ScalJob>(d, PS_SC);
  p.sc1 = f.ptr<ScalJob>(d, PS_SC1);
  p.sc_post = f.ptr<ScalJob>(d, PS_SCPOST);
  p.sclist = f.ptr<uint32_t>(d, PS_SCLIST);
  p.vt = f.ptr<VTerm>(d, PS_VT);
  p.g1 = f.ptr<G1Job>(d, PS_G1);
  p.g1p = f.ptr<G1Job>(d, PS_G1P);
  p.g2 = f.ptr<G2Job>(d, PS_G2);
  p.pr = f.ptr<PairJob>(d, PS_PR);
  p.seg = f.ptr<Seg>(d, PS_SEG);
  p.hpre = f.ptr<HashJob>(d, PS_HPRE);
  p.hmain = f.ptr<HashJob>(d, PS_HMAIN);
  p.ck = f.ptr<Check>(d, PS_CK);
  p.tx = f.ptr<TxChecks>(d, PS_TX);
  p.rnd = f.ptr<RandJob>(d, PS_RND);
  p.emit = f.ptr<EmitJob>(d, PS_EMIT);
  p.b64 = f.ptr<B64Job>(d, PS_B64);
  p.cp = f.ptr<CopyJob>(d, PS_CP);
  p.cp2 = f.ptr<CopyJob>(d, PS_CP2);
  const ScratchLayout& l = b->sl;
  p.pts = reinterpret_cast<G1Dev*>(s + l.pts);
  p.pt_ok = s + l.pt_ok;
  p.scal = reinterpret_cast<uint32_t (*)[8]>(s + l.scal);
  p.canon = s + l.canon;
  p.g1out = reinterpret_cast<G1Dev*>(s + l.g1out);
  p.pnorm = reinterpret_cast<G1Dev*>(s + l.pnorm);
  p.g2out = reinterpret_cast<G2Dev*>(s + l.g2out);
  p.fbuf = reinterpret_cast<F12Dev*>(s + l.fbuf);
  p.fxpark = reinterpret_cast<int32_t*>(s + l.fxpark);
  p.lines2 = reinterpret_cast<EvLineDev*>(s + l.lines2);
  p.part1 = reinterpret_cast<G1JDev*>(s + l.part1);
  p.part1p = reinterpret_cast<G1JDev*>(s + l.part1p);
  p.part2 = reinterpret_cast<G2PartDev*>(s + l.part2);
  p.vtab1 = reinterpret_cast<G1Dev*>(s + l.vtab1);
  p.vtab1p = reinterpret_cast<G1Dev*>(s + l.vtab1p);
  p.hash_ok = s + l.hash_ok;
  p.hash_ok_pre = s + l.hash_ok_pre;
  p.codes = reinterpret_cast<int32_t*>(s + l.codes);
  p.bitmap = reinterpret_cast<uint32_t*>(s + l.bitmap);
  p.n_dec = (uint32_t)f.cnt[PS_DEC];
  p.n_zr = (uint32_t)f.cnt[PS_ZR];
  p.n_sc = (uint32_t)f.cnt[PS_SC];
  p.n_sc1 = (uint32_t)f.cnt[PS_SC1];
  p.n_sp = (uint32_t)f.cnt[PS_SCPOST];
  p.n_rnd = (uint32_t)f.cnt[PS_RND];
  p.n_em = (uint32_t)f.cnt[PS_EMIT];
  p.n_b64 = (uint32_t)f.cnt[PS_B64];
  p.n_g1 = (uint32_t)f.cnt[PS_G1];
  p.n_g1p = (uint32_t)f.cnt[PS_G1P];
  p.n_g2 = (uint32_t)f.cnt[PS_G2];
  p.n_pr = (uint32_t)f.cnt[PS_PR];
  p.n_hp = (uint32_t)f.cnt[PS_HPRE];
  p.n_hm = (uint32_t)f.cnt[PS_HMAIN];
  p.n_tx = (uint32_t)f.cnt[PS_TX];
  p.n_cp = (uint32_t)f.cnt[PS_CP];
  p.n_cp2 = (uint32_t)f.cnt[PS_CP2];
  return p;
}

// Host -> device copy of a slot's plan: the blob up to fp.upload, and with
// device-initialised pools the const region at the start of the arena (the rest
// of the arena and the proof output are written on the device by k_copy).
static hipError_t upload_plan(ftz_batch* b, hipStream_t s) {
  const FlatPlan& f = b->fp;
  hipError_t e = hipMemcpyAsync(b->d_blob.p, b->h_blob.p, f.upload, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && f.dev_pools)
    e = hipMemcpyAsync(b->d_blob.p + f.off[PS_ARENA], b->h_blob.p + f.off[PS_ARENA], C_SIZE, hipMemcpyHostToDevice, s);
  return e;
}

// t' and the pair-2 lines (R read from `pts`): one lane per job (default;
// k_g2_part four lanes per job for the table sums, then k_g2lines1) or the
// sextet layout (k_g2lines); same bytes either way
static void launch_g2lines(ftz_ctx* c, const SlotPtrs& p, const G1Dev* pts, hipStream_t s, bool prover) {
  // small passes (few callers waiting) take the low-latency sextet layout: six lanes
  // per job cut the stage's per-job chain, which bounds a small pass's latency --
  // unless ftz_ctx_set_layout chose the verifier's layout explicitly
  int layout = prover ? c->g2lanes_prover : c->g2lanes;
  if (!prover && !c->g2lanes_set && p.n_g2 <= c->opt.small_pass) layout = FTZ_LAYOUT_SEXTET;
  if (layout == FTZ_LAYOUT_ONE_LANE) {
    k_g2_part<<<blocks_for(4 * p.n_g2, 64), 64, 0, s>>>(p.g2, p.n_g2, p.scal, c->g2tab.p, p.part2);
#if FTS_G2_BINV && FTS_G2LINES_X29
    k_g2_sum<<<blocks_for(p.n_g2, 64), 64, 0, s>>>(p.n_g2, p.part2);
    k_g2_binv<<<blocks_for(p.n_g2, 256), 256, 0, s>>>(p.n_g2, p.part2);
#endif
    k_g2lines1<<<blocks_for(p.n_g2, 64), 64, 0, s>>>(p.g2, p.pr, p.n_g2, p.part2, p.g2out, pts, p.lines2);
  } else {
    k_g2lines<<<blocks_for(p.n_g2, SX_JOBS_PER_WAVE), 64, 0, s>>>(p.g2, p.pr, p.n_g2, p.scal, c->g2tab.p, p.g2out, pts,
                                                                  p.lines2);
  }
}

static void launch_miller(ftz_ctx* c, const SlotPtrs& p, hipStream_t s) {
  if (c->qnorm) {
    k_miller_n<<<blocks_for(p.n_pr, SX_JOBS_PER_WAVE), 64, 0, s>>>(p.pr, p.n_pr, c->qlines29n.p, p.lines2, p.g1out,
                                                                   p.pnorm, p.fbuf);
    return;
  }
  k_miller<<<blocks_for(p.n_pr, SX_JOBS_PER_WAVE), 64, 0, s>>>(p.pr, p.n_pr, c->qlines29.p, p.lines2, p.g1out,
                                                                 p.fbuf);
}

static void launch_fexp(ftz_ctx* c, const SlotPtrs& p, hipStream_t s) {
  launch_fexp(c->opt.fexp != FTZ_FEXP_FUENTES, p.pr, p.n_pr, p.fbuf, p.arena, p.fxpark, s);
}

// Verification pipeline.  Three streams after the light decode/scalar kernels:
//   st[2]: G2 jobs t' and the pair-2 Miller lines evaluated at R (k_g2lines)
//   st[0]: G1 jobs feeding the pairings (P1 = sbf*P - c*S), then, after st[2],
//          the sextet Miller loops and final exponentiations
//   st[1]: the G1 jobs no pairing depends on (well-formedness, range equality,
//          membership Schnorr commitments)
// The transcript hashes wait for all three.
int slot_submit(ftz_batch* b, bool upload, bool fetch_codes) {
  ftz_ctx* c = b->ctx;
  HC(hipSetDevice(c->device));
  SlotPtrs p = slot_ptrs(b);
  hipStream_t s = b->st[0], s2 = b->st[1], s3 = b->st[2];
  if (c->serial) s2 = s3 = s;
  const uint64_t jobs[FTZ_NKERNELS] = {p.n_dec, p.n_zr, p.n_hp, p.n_sc, p.n_g1p, p.n_g2,
                                       p.n_pr,  p.n_pr, p.n_g1, p.n_hm, p.n_tx, p.n_tx};
  for (int k = 0; k < FTZ_NKERNELS; k++) b->jobs_last[k] = jobs[k];
  hipEvent_t* e = b->ev;
  HC(hipEventRecord(e[18], s));
  if (upload) HC(upload_plan(b, s));
  HC(hipMemsetAsync(p.bitmap, 0, sizeof(uint32_t) * ((b->n + 31) / 32 + 1), s));
  if (b->fp.n_pts) HC(hipMemsetAsync(p.pt_ok, 1, b->fp.n_pts, s));
  HC(hipEventRecord(e[0], s));
  // shape images into every proof's arena block and output, then the witness bytes
  if (p.n_cp) k_copy<<<p.n_cp, 64, 0, s>>>(p.cp, p.n_cp, p.wire, p.arena, p.out);
  if (p.n_cp2) k_copy<<<p.n_cp2, 64, 0, s>>>(p.cp2, p.n_cp2, p.wire, p.arena, p.out);
  if (p.n_dec) k_decode<<<blocks_for(p.n_dec, 256), 256, 0, s>>>(p.dec, p.n_dec, p.wire, p.pts, p.pt_ok, p.arena);
  HC(hipEventRecord(e[1], s));
  if (p.n_zr) k_zr<<<blocks_for(p.n_zr, 256), 256, 0, s>>>(p.zr, p.n_zr, p.wire, p.scal, p.canon);
  HC(hipEventRecord(e[2], s));
  if (p.n_hp)
    k_hash<<<blocks_for(p.n_hp, 128), 128, 0, s>>>(p.hpre, p.n_hp, p.seg, p.arena, p.scal, p.canon, p.hash_ok_pre);
  HC(hipEventRecord(e[3], s));
  if (p.n_sc) k_scalar<<<blocks_for(p.n_sc, 256), 256, 0, s>>>(p.sc, p.n_sc, p.scal, p.sclist);
  HC(hipEventRecord(e[4], s));
  // st[2]: G2 jobs + pair-2 lines
  HC(hipStreamWaitEvent(s3, e[4], 0));
  HC(hipEventRecord(e[14], s3));
  if (p.n_g2)
    launch_g2lines(c, p, p.pts, s3, false);
  HC(hipEventRecord(e[15], s3));
  // st[0]: pairing chain
  HC(hipEventRecord(e[16], s));
  if (p.n_g1p) {
    k_g1_part<<<blocks_for(4 * p.n_g1p, 128), 128, 0, s>>>(p.g1p, p.n_g1p, p.vt, p.pts, p.scal, c->g1tab.p, p.part1p,
                                                           p.vtab1p);
    k_g1_combine<<<blocks_for(p.n_g1p, 256), 256, 0, s>>>(p.g1p, p.n_g1p, p.part1p, p.g1out, p.arena, p.pnorm);
  }
  HC(hipEventRecord(e[5], s));
  // st[1]: pairing-independent G1 jobs, started with the jobs the chain waits for
  HC(hipStreamWaitEvent(s2, e[4], 0));
  HC(hipEventRecord(e[11], s2));
  if (p.n_g1) {
    k_g1_part<<<blocks_for(4 * p.n_g1, 128), 128, 0, s2>>>(p.g1, p.n_g1, p.vt, p.pts, p.scal, c->g1tab.p, p.part1,
                                                           p.vtab1);
    k_g1_combine<<<blocks_for(p.n_g1, 256), 256, 0, s2>>>(p.g1, p.n_g1, p.part1, p.g1out, p.arena, p.pnorm);
  }
  HC(hipEventRecord(e[12], s2));
  HC(hipStreamWaitEvent(s, e[15], 0));
  HC(hipEventRecord(e[6], s));
  if (p.n_pr)
    launch_miller(c, p, s);
  HC(hipEventRecord(e[7], s));
  launch_fexp(c, p, s);
  HC(hipEventRecord(e[8], s));
  HC(hipStreamWaitEvent(s, e[12], 0));
  HC(hipEventRecord(e[9], s));
  if (p.n_hm)
    k_hash<<<blocks_for(p.n_hm, 128), 128, 0, s>>>(p.hmain, p.n_hm, p.seg, p.arena, p.scal, p.canon, p.hash_ok);
  HC(hipEventRecord(e[10], s));
  if (p.n_tx)
    k_verdict<<<blocks_for(p.n_tx, 256), 256, 0, s>>>(p.tx, p.n_tx, p.ck, p.pt_ok, p.hash_ok, p.codes, p.bitmap);
  HC(hipEventRecord(e[13], s));
  if (fetch_codes && b->n) HC(hipMemcpyAsync(b->h_res.p, p.codes, b->n * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HC(hipEventRecord(e[17], s));
  HC(hipGetLastError());
  b->pending = true;
  return FTZ_SUCCESS;
}

// stats slots: decode zr hash_pre scalar g1p g2+lines miller fexp g1(side) hash verdict total
static const int ST_FROM[FTZ_NKERNELS] = {0, 1, 2, 3, 16, 14, 6, 7, 11, 9, 10, 0};
static const int ST_TO[FTZ_NKERNELS] = {1, 2, 3, 4, 5, 15, 7, 8, 12, 10, 13, 13};

int slot_wait(ftz_batch* b) {
  if (!b->pending) return FTZ_SUCCESS;
  HC(hipSetDevice(b->ctx->device));
  HC(hipEventSynchronize(b->ev[17]));
  b->pending = false;
  for (int k = 0; k < FTZ_NKERNELS; k++) {
    float ms = 0;
    HC(hipEventElapsedTime(&ms, b->ev[ST_FROM[k]], b->ev[ST_TO[k]]));
    b->stats.ms[k] = ms;
    b->stats.jobs[k] = b->jobs_last[k];
  }
  return FTZ_SUCCESS;
}

// ------------------------------------------------------------------ staged batch API
static int staged_load(ftz_ctx* c, size_t n, const PlanItem* items, ftz_batch** out) {
  HC(hipSetDevice(c->device));
  ftz_batch* b = new ftz_batch();
  b->ctx = c;
  int rc = slot_init(b);
  if (rc == FTZ_SUCCESS) rc = slot_plan_items(b, n, items);
  if (rc == FTZ_SUCCESS) {
    hipError_t e = hipMemcpyAsync(b->d_blob.p, b->h_blob.p, b->fp.bytes, hipMemcpyHostToDevice, b->st[0]);
    if (e == hipSuccess) e = hipStreamSynchronize(b->st[0]);
    if (e != hipSuccess) rc = set_err(FTZ_E_DEVICE, std::string("batch upload failed: ") + hipGetErrorString(e));
  }
  if (rc != FTZ_SUCCESS) {
    slot_free(b);
    delete b;
    return rc;
  }
  *out = b;
  return FTZ_SUCCESS;
}

static bool transfer_args_ok(size_t n, const ftz_transfer* tx) {
  for (size_t i = 0; i < n; i++)
    if ((tx[i].n_in && !tx[i].inputs) || (tx[i].n_out && !tx[i].outputs) || (tx[i].proof_len && !tx[i].proof))
      return false;
  return true;
}
static bool issue_args_ok(size_t n, const ftz_issue* is) {
  for (size_t i = 0; i < n; i++)
    if ((is[i].n_out && !is[i].outputs) || (is[i].proof_len && !is[i].proof)) return false;
  return true;
}

extern "C" int ftz_batch_load_transfers(ftz_ctx* c, size_t n, const ftz_transfer* tx, ftz_batch** out) {
  if (!c || !out || (n && !tx)) return set_err(FTZ_E_INVALID, "null argument");
  if (!transfer_args_ok(n, tx)) return set_err(FTZ_E_INVALID, "null buffer in transfer");
  std::vector<PlanItem> items(n);
  for (size_t i = 0; i < n; i++) {
    memset(&items[i], 0, sizeof(PlanItem));
    items[i].kind = 0;
    items[i].t = {tx[i].inputs, tx[i].n_in, tx[i].outputs, tx[i].n_out, tx[i].proof, tx[i].proof_len};
  }
  return staged_load(c, n, items.data(), out);
}

extern "C" int ftz_batch_load_issues(ftz_ctx* c, size_t n, const ftz_issue* is, ftz_batch** out) {
  if (!c || !out || (n && !is)) return set_err(FTZ_E_INVALID, "null argument");
  if (!issue_args_ok(n, is)) return set_err(FTZ_E_INVALID, "null buffer in issue");
  std::vector<PlanItem> items(n);
  for (size_t i = 0; i < n; i++) {
    memset(&items[i], 0, sizeof(PlanItem));
    items[i].kind = 1;
    items[i].i = {is[i].outputs, is[i].n_out, is[i].proof, is[i].proof_len, is[i].anonymous};
  }
  return staged_load(c, n, items.data(), out);
}

extern "C" int ftz_batch_submit(ftz_batch* b) {
  if (!b) return set_err(FTZ_E_INVALID, "null batch");
  if (b->pending) return set_err(FTZ_E_INVALID, "batch resubmitted before ftz_batch_wait");
  return slot_submit(b, false, false);
}

extern "C" int ftz_batch_wait(ftz_batch* b) {
  if (!b) return set_err(FTZ_E_INVALID, "null batch");
  return slot_wait(b);
}

extern "C" int ftz_batch_run(ftz_batch* b) {
  int rc = ftz_batch_submit(b);
  return rc == FTZ_SUCCESS ? ftz_batch_wait(b) : rc;
}

extern "C" int ftz_batch_codes(ftz_batch* b, int32_t* codes) {
  if (!b || (b->n && !codes)) return set_err(FTZ_E_INVALID, "null argument");
  int rc = slot_wait(b);
  if (rc != FTZ_SUCCESS) return rc;
  HC(hipSetDevice(b->ctx->device));
  if (b->n) HC(hipMemcpy(codes, b->d_scr.p + b->sl.codes, b->n * sizeof(int32_t), hipMemcpyDeviceToHost));
  return FTZ_SUCCESS;
}

extern "C" int ftz_batch_bitmap(ftz_batch* b, uint8_t* bits) {
  if (!b || (b->n && !bits)) return set_err(FTZ_E_INVALID, "null argument");
  int rc = slot_wait(b);
  if (rc != FTZ_SUCCESS) return rc;
  HC(hipSetDevice(b->ctx->device));
  std::vector<uint32_t> w((b->n + 31) / 32);
  if (!w.empty()) HC(hipMemcpy(w.data(), b->d_scr.p + b->sl.bitmap, w.size() * 4, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < (b->n + 7) / 8; i++) bits[i] = (uint8_t)(w[i / 4] >> (8 * (i % 4)));
  return FTZ_SUCCESS;
}

extern "C" int ftz_batch_stats(const ftz_batch* b, ftz_stats* out) {
  if (!b || !out) return set_err(FTZ_E_INVALID, "null argument");
  *out = b->stats;
  return FTZ_SUCCESS;
}

extern "C" size_t ftz_batch_size(const ftz_batch* b) { return b ? b->n : 0; }

extern "C" int ftz_batch_challenges(ftz_batch* b, size_t i, int32_t* kinds, uint8_t* values, size_t cap,
                                    size_t* count) {
  if (!b || !count || (cap && (!kinds || !values))) return set_err(FTZ_E_INVALID, "null argument");
  if (i >= b->n) return set_err(FTZ_E_INVALID, "proof index out of range");
  int rc = slot_wait(b);
  if (rc != FTZ_SUCCESS) return rc;
  const FlatPlan& f = b->fp;
  const TxChecks* tx = f.ptr<TxChecks>(b->h_blob.p, PS_TX);
  const Check* ck = f.ptr<Check>(b->h_blob.p, PS_CK);
  const HashJob* hm = f.ptr<HashJob>(b->h_blob.p, PS_HMAIN);
  std::vector<int32_t> kd(cap);
  std::vector<uint32_t> slot(cap);
  size_t m = proof_challenge_slots(tx[i], ck, hm, kd.data(), slot.data(), cap);
  *count = m;
  HC(hipSetDevice(b->ctx->device));
  for (size_t k = 0; k < std::min(m, cap); k++) {
    if (slot[k] == NONE) return set_err(FTZ_E_INVALID, "batch not loaded with FTZ_DEBUG_CHALLENGES");
    uint32_t h[8];
    HC(hipMemcpy(h, b->d_scr.p + b->sl.scal + 32 * (size_t)slot[k], 32, hipMemcpyDeviceToHost));
    kinds[k] = kd[k];
    limbs_to_be32(values + 32 * k, h);
  }
  return FTZ_SUCCESS;
}

extern "C" void ftz_batch_destroy(ftz_batch* b) {
  if (!b) return;
  (void)hipSetDevice(b->ctx->device);
  slot_free(b);
  delete b;
}

extern "C" int ftz_verify_transfers(ftz_ctx* c, size_t n, const ftz_transfer* tx, int32_t* codes) {
  if (!c || (n && (!tx || !codes))) return set_err(FTZ_E_INVALID, "null argument");
  if (n == 0) return FTZ_SUCCESS;
  if (!transfer_args_ok(n, tx)) return set_err(FTZ_E_INVALID, "null buffer in transfer");
  return engine_verify(c, n, tx, nullptr, codes);
}

extern "C" int ftz_verify_issues(ftz_ctx* c, size_t n, const ftz_issue* is, int32_t* codes) {
  if (!c || (n && (!is || !codes))) return set_err(FTZ_E_INVALID, "null argument");
  if (n == 0) return FTZ_SUCCESS;
  if (!issue_args_ok(n, is)) return set_err(FTZ_E_INVALID, "null buffer in issue");
  return engine_verify(c, n, nullptr, is, codes);
}

// ------------------------------------------------------------------ prover
// Plans from host/planner_prove.cpp; the pipeline of slot_submit with the
// prover's extra stages: randomness before the group work, responses, JSON
// hole filling and base64 of the inner documents after the transcript hashes.
int prover_submit(ftz_batch* b, bool upload, bool fetch) {
  ftz_ctx* c = b->ctx;
  HC(hipSetDevice(c->device));
  SlotPtrs p = slot_ptrs(b);
  hipStream_t s = b->st[0], s2 = b->st[1], s3 = b->st[2];
  if (c->serial) s2 = s3 = s;
  uint64_t jobs[FTZ_NKERNELS] = {p.n_dec, p.n_zr, (uint64_t)p.n_rnd + p.n_hp, p.n_sc, p.n_g1p, p.n_g2, p.n_pr, p.n_pr,
                                 p.n_g1, (uint64_t)p.n_hm + p.n_sp, (uint64_t)p.n_em + p.n_b64, p.n_tx};
  for (int k = 0; k < FTZ_NKERNELS; k++) b->jobs_last[k] = jobs[k];
  hipEvent_t* e = b->ev;
  HC(hipEventRecord(e[18], s));
  if (upload) HC(upload_plan(b, s));
  HC(hipMemsetAsync(p.bitmap, 0, sizeof(uint32_t) * ((b->n + 31) / 32 + 1), s));
  if (b->fp.n_pts) HC(hipMemsetAsync(p.pt_ok, 1, b->fp.n_pts, s));
  HC(hipEventRecord(e[0], s));
  // shape images into every proof's arena block and output, then the witness bytes
  if (p.n_cp) k_copy<<<p.n_cp, 64, 0, s>>>(p.cp, p.n_cp, p.wire, p.arena, p.out);
  if (p.n_cp2) k_copy<<<p.n_cp2, 64, 0, s>>>(p.cp2, p.n_cp2, p.wire, p.arena, p.out);
  if (p.n_dec) k_decode<<<blocks_for(p.n_dec, 256), 256, 0, s>>>(p.dec, p.n_dec, p.wire, p.pts, p.pt_ok, p.arena);
  HC(hipEventRecord(e[1], s));
  if (p.n_zr) k_zr<<<blocks_for(p.n_zr, 256), 256, 0, s>>>(p.zr, p.n_zr, p.wire, p.scal, p.canon);
  HC(hipEventRecord(e[2], s));
  if (p.n_rnd) k_rand<<<blocks_for(p.n_rnd, 128), 128, 0, s>>>(p.rnd, p.n_rnd, p.arena, p.scal);
  if (p.n_hp)
    k_hash<<<blocks_for(p.n_hp, 128), 128, 0, s>>>(p.hpre, p.n_hp, p.seg, p.arena, p.scal, p.canon, p.hash_ok_pre);
  HC(hipEventRecord(e[3], s));
  if (p.n_sc) k_scalar<<<blocks_for(p.n_sc, 256), 256, 0, s>>>(p.sc, p.n_sc, p.scal, p.sclist);
  if (p.n_sc1) k_scalar<<<blocks_for(p.n_sc1, 256), 256, 0, s>>>(p.sc1, p.n_sc1, p.scal, p.sclist);
  HC(hipEventRecord(e[4], s));
  // st[1]: G1 jobs no pairing depends on
  HC(hipStreamWaitEvent(s2, e[4], 0));
  HC(hipEventRecord(e[11], s2));
  if (p.n_g1) {
    k_g1_part<<<blocks_for(4 * p.n_g1, 128), 128, 0, s2>>>(p.g1, p.n_g1, p.vt, p.pts, p.scal, prover_g1tab(c), p.part1,
                                                           p.vtab1);
    k_g1_combine<<<blocks_for(p.n_g1, 256), 256, 0, s2>>>(p.g1, p.n_g1, p.part1, p.g1out, p.arena, p.pnorm);
  }
  HC(hipEventRecord(e[12], s2));
  // st[0]: R' = rr R and rsbf P (the pairing inputs)
  HC(hipEventRecord(e[16], s));
  if (p.n_g1p) {
    k_g1_part<<<blocks_for(4 * p.n_g1p, 128), 128, 0, s>>>(p.g1p, p.n_g1p, p.vt, p.pts, p.scal, prover_g1tab(c), p.part1p,
                                                           p.vtab1p);
    k_g1_combine<<<blocks_for(p.n_g1p, 256), 256, 0, s>>>(p.g1p, p.n_g1p, p.part1p, p.g1out, p.arena, p.pnorm);
  }
  HC(hipEventRecord(e[5], s));
  // st[2]: t = rv PK1 + rh PK2 and its lines evaluated at R' (pair 2 reads g1out);
  // none with fixed pairs (every G2 argument is a PP point with precomputed lines)
  HC(hipStreamWaitEvent(s3, e[5], 0));
  HC(hipEventRecord(e[14], s3));
  if (p.n_g2)
    launch_g2lines(c, p, p.g1out, s3, true);
  HC(hipEventRecord(e[15], s3));
  HC(hipStreamWaitEvent(s, e[15], 0));
  HC(hipEventRecord(e[6], s));
  if (p.n_pr && p.n_g2 == 0 && c->pp.fixed_pairs && c->ptab_ready)  // e(C, Q) e(A, PK1) e(B, PK2)
    k_miller_f3<<<blocks_for(p.n_pr, SX_JOBS_PER_WAVE), 64, 0, s>>>(p.pr, p.n_pr, c->qlines29n.p, c->pklines29n.p,
                                                                    p.g1out, p.pnorm, p.fbuf);
  else if (p.n_pr)
    launch_miller(c, p, s);
  HC(hipEventRecord(e[7], s));
  launch_fexp(c, p, s);
  HC(hipEventRecord(e[8], s));
  HC(hipStreamWaitEvent(s, e[12], 0));
  HC(hipEventRecord(e[9], s));
  if (p.n_hm)
    k_hash<<<blocks_for(p.n_hm, 128), 128, 0, s>>>(p.hmain, p.n_hm, p.seg, p.arena, p.scal, p.canon, p.hash_ok);
  if (p.n_sp) k_scalar<<<blocks_for(p.n_sp, 256), 256, 0, s>>>(p.sc_post, p.n_sp, p.scal, p.sclist);
  HC(hipEventRecord(e[10], s));
  if (p.n_em) k_emit<<<blocks_for(p.n_em, 256), 256, 0, s>>>(p.emit, p.n_em, p.scal, p.arena);
  if (p.n_b64) k_b64<<<p.n_b64, 256, 0, s>>>(p.b64, p.n_b64, p.arena, p.out);
  if (p.n_tx)
    k_verdict<<<blocks_for(p.n_tx, 256), 256, 0, s>>>(p.tx, p.n_tx, p.ck, p.pt_ok, p.hash_ok, p.codes, p.bitmap);
  HC(hipEventRecord(e[13], s));  // total includes the verdict kernel
  if (fetch) {
    if (b->n) HC(hipMemcpyAsync(b->h_res.p, p.codes, b->n * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if (b->fp.cnt[PS_OUT])
      HC(hipMemcpyAsync(const_cast<uint8_t*>(slot_out(b)), p.out, b->fp.cnt[PS_OUT], hipMemcpyDeviceToHost, s));
  }
  HC(hipEventRecord(e[17], s));
  HC(hipGetLastError());
  b->pending = true;
  return FTZ_SUCCESS;
}

int prover_wait(ftz_batch* b) { return slot_wait(b); }

template <class W>
static int prover_load(ftz_ctx* c, size_t n, const W* w, int kind, ftz_prover** out) {
  if (!c || !out || (n && !w)) return set_err(FTZ_E_INVALID, "null argument");
  HC(hipSetDevice(c->device));
  ftz_prover* b = new ftz_prover();
  b->ctx = c;
  b->prover = true;
  int rc = slot_init(b);
  if (rc == FTZ_SUCCESS) rc = prover_plan(b, n, w, kind);
  if (rc == FTZ_SUCCESS) {
    hipError_t e = upload_plan(b, b->st[0]);
    if (e == hipSuccess) e = hipStreamSynchronize(b->st[0]);
    if (e != hipSuccess) rc = set_err(FTZ_E_DEVICE, std::string("prover upload failed: ") + hipGetErrorString(e));
  }
  if (rc != FTZ_SUCCESS) {
    slot_free(b);
    delete b;
    return rc;
  }
  *out = b;
  return FTZ_SUCCESS;
}

static bool transfer_wit_ok(size_t n, const ftz_transfer_witness* w, std::string& e) {
  for (size_t i = 0; i < n; i++)
    if ((w[i].n_in && (!w[i].inputs || !w[i].in_values || !w[i].in_bfs)) ||
        (w[i].n_out && (!w[i].outputs || !w[i].out_values || !w[i].out_bfs)) || !w[i].seed ||
        (w[i].type_len && !w[i].type)) {
      e = "null buffer in witness " + std::to_string(i);
      return false;
    }
  return true;
}
static bool issue_wit_ok(size_t n, const ftz_issue_witness* w, std::string& e) {
  for (size_t i = 0; i < n; i++)
    if ((w[i].n_out && (!w[i].outputs || !w[i].values || !w[i].bfs)) || !w[i].seed ||
        (w[i].type_len && !w[i].type)) {
      e = "null buffer in witness " + std::to_string(i);
      return false;
    }
  return true;
}

static std::vector<TransferWit> to_wit(size_t n, const ftz_transfer_witness* w) {
  std::vector<TransferWit> t(n);
  for (size_t i = 0; i < n; i++)
    t[i] = {w[i].inputs,     w[i].n_in,    w[i].outputs, w[i].n_out,    w[i].in_values, w[i].in_bfs,
            w[i].out_values, w[i].out_bfs, w[i].type,    w[i].type_len, w[i].seed};
  return t;
}
static std::vector<IssueWit> to_wit(size_t n, const ftz_issue_witness* w) {
  std::vector<IssueWit> t(n);
  for (size_t i = 0; i < n; i++)
    t[i] = {w[i].outputs, w[i].n_out, w[i].values, w[i].bfs, w[i].type, w[i].type_len, w[i].anonymous, w[i].seed};
  return t;
}

extern "C" int ftz_prover_load_transfers(ftz_ctx* c, size_t n, const ftz_transfer_witness* w, ftz_prover** out) {
  std::string e;
  if (w && !transfer_wit_ok(n, w, e)) return set_err(FTZ_E_INVALID, e);
  std::vector<TransferWit> t = w ? to_wit(n, w) : std::vector<TransferWit>();
  return prover_load(c, n, w ? t.data() : (const TransferWit*)nullptr, 0, out);
}

extern "C" int ftz_prover_load_issues(ftz_ctx* c, size_t n, const ftz_issue_witness* w, ftz_prover** out) {
  std::string e;
  if (w && !issue_wit_ok(n, w, e)) return set_err(FTZ_E_INVALID, e);
  std::vector<IssueWit> t = w ? to_wit(n, w) : std::vector<IssueWit>();
  return prover_load(c, n, w ? t.data() : (const IssueWit*)nullptr, 1, out);
}

extern "C" int ftz_prover_submit(ftz_prover* b) {
  if (!b) return set_err(FTZ_E_INVALID, "null prover");
  if (b->pending) return set_err(FTZ_E_INVALID, "prover resubmitted before ftz_prover_wait");
  return prover_submit(b, false, false);
}

extern "C" int ftz_prover_wait(ftz_prover* b) {
  if (!b) return set_err(FTZ_E_INVALID, "null prover");
  return prover_wait(b);
}

extern "C" int ftz_prover_run(ftz_prover* b) {
  int rc = ftz_prover_submit(b);
  return rc == FTZ_SUCCESS ? ftz_prover_wait(b) : rc;
}

extern "C" size_t ftz_prover_bytes(const ftz_prover* b) { return b ? b->fp.cnt[PS_OUT] : 0; }

extern "C" int ftz_prover_proofs(ftz_prover* b, uint8_t* buf, size_t cap, size_t* offsets, int32_t* codes) {
  if (!b) return set_err(FTZ_E_INVALID, "null prover");
  size_t nb = b->fp.cnt[PS_OUT];
  if (cap < nb || (nb && !buf)) return set_err(FTZ_E_INVALID, "proof buffer too small");
  int rc = slot_wait(b);
  if (rc != FTZ_SUCCESS) return rc;
  HC(hipSetDevice(b->ctx->device));
  hipStream_t s = b->st[0];
  if (nb) HC(hipMemcpyAsync(buf, b->d_blob.p + b->fp.off[PS_OUT], nb, hipMemcpyDeviceToHost, s));
  if (codes && b->n) HC(hipMemcpyAsync(codes, b->d_scr.p + b->sl.codes, b->n * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HC(hipStreamSynchronize(s));
  if (offsets) {
    for (size_t i = 0; i < b->n; i++) offsets[i] = b->fp.out_off[i];
    offsets[b->n] = nb;
  }
  return FTZ_SUCCESS;
}

extern "C" int ftz_prover_stats(const ftz_prover* b, ftz_stats* out) {
  if (!b || !out) return set_err(FTZ_E_INVALID, "null argument");
  *out = b->stats;
  return FTZ_SUCCESS;
}

extern "C" void ftz_prover_destroy(ftz_prover* b) {
  if (!b) return;
  (void)hipSetDevice(b->ctx->device);
  slot_free(b);  // syncs and destroys the streams and events (no leak per prove call)
  delete b;
}

// One-shot proving of any n: passes of min(opt.batch, 4096) witnesses pipelined through
// the context's reusable prover slots (plan batch k+1 on the host while batch
// k runs), proofs concatenated into buf in witness order.
template <class W>
static int prove_chunked(ftz_ctx* c, size_t n, const W* w, int kind, uint8_t* buf, size_t cap, size_t* offsets,
                         int32_t* codes) {
  std::lock_guard<std::mutex> lk(c->prove_mu);
  HC(hipSetDevice(c->device));
  using Clk = std::chrono::steady_clock;
  auto ms = [](Clk::time_point a, Clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  const Clk::time_point t_call = Clk::now();
  ftz_prover_host_stats& ps = c->pstats;
  // passes of at most 4096 witnesses: the prover's pass is a latency-bound
  // chain (R' -> t lines -> Miller -> final exponentiation -> challenges ->
  // responses) planned on the calling thread, and 8192-witness passes fill the
  // slots too slowly (65536 proofs: 298k/s vs 426k/s, profiles/r02g_prover_layout.txt);
  // opt.slots of them in flight (clamped to [2, 8])
  const size_t K = std::max<size_t>(2, std::min<size_t>(c->opt.slots, 8)), B = std::min<size_t>(c->opt.batch, 4096);
  while (c->pslots.size() < K) {
    ftz_prover* p = new ftz_prover();
    p->ctx = c;
    p->prover = true;
    int rc = slot_init(p);
    if (rc != FTZ_SUCCESS) {
      slot_free(p);
      delete p;
      return rc;
    }
    c->pslots.push_back(p);
  }
  size_t nchunks = (n + B - 1) / B, written = 0;
  int rc = FTZ_SUCCESS;
  auto finish = [&](size_t k) {
    ftz_prover* p = c->pslots[k % K];
    Clk::time_point t0 = Clk::now();
    int r = prover_wait(p);
    Clk::time_point t1 = Clk::now();
    ps.wait_ms += ms(t0, t1);
    if (r != FTZ_SUCCESS) return r;
    size_t lo = k * B, nb = p->fp.cnt[PS_OUT];
    if (written + nb > cap) return set_err(FTZ_E_INVALID, "proof buffer too small");
    // ~29 MB of proof JSON per 4096-proof pass: copied by the planning threads
    // (one core's memcpy took a third of the host time between passes)
    if (nb) {
      const size_t parts = 16, step = (nb + parts - 1) / parts;
      const uint8_t* src = slot_out(p);
      uint8_t* dst = buf + written;
      c->pool->run(parts, [&](size_t i) {
        size_t a = i * step, e = std::min(nb, a + step);
        if (e > a) memcpy(dst + a, src + a, e - a);
      });
    }
    for (size_t i = 0; i < p->n; i++) {
      if (offsets) offsets[lo + i] = written + p->fp.out_off[i];
      if (codes) codes[lo + i] = slot_codes(p)[i];
    }
    written += nb;
    ps.copy_ms += ms(t1, Clk::now());
    ps.passes++;
    ps.proofs += p->n;
    return FTZ_SUCCESS;
  };
  size_t done = 0;
  for (size_t k = 0; k < nchunks && rc == FTZ_SUCCESS; k++) {
    if (k >= K) {
      rc = finish(done++);
      if (rc != FTZ_SUCCESS) break;
    }
    ftz_prover* p = c->pslots[k % K];
    size_t lo = k * B, cnt = std::min(B, n - lo);
    Clk::time_point t0 = Clk::now();
    rc = prover_plan(p, cnt, w + lo, kind);
    Clk::time_point t1 = Clk::now();
    if (rc == FTZ_SUCCESS) rc = prover_submit(p, true, true);
    ps.plan_ms += ms(t0, t1);
    ps.submit_ms += ms(t1, Clk::now());
  }
  // drain what is in flight (also after an error, so no slot stays pending)
  int rc2 = FTZ_SUCCESS;
  while (done < nchunks) {
    ftz_prover* p = c->pslots[done % K];
    if (!p->pending) break;
    int r = rc == FTZ_SUCCESS ? finish(done) : prover_wait(p);
    if (r != FTZ_SUCCESS && rc2 == FTZ_SUCCESS) rc2 = r;
    done++;
  }
  if (rc == FTZ_SUCCESS) rc = rc2;
  if (rc == FTZ_SUCCESS && offsets) offsets[n] = written;
  ps.wall_ms += ms(t_call, Clk::now());
  return rc;
}

extern "C" int ftz_ctx_prover_stats(ftz_ctx* c, ftz_prover_host_stats* out, int reset) {
  if (!c || !out) return set_err(FTZ_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(c->prove_mu);
  *out = c->pstats;
  if (reset) c->pstats = ftz_prover_host_stats{};
  return FTZ_SUCCESS;
}

extern "C" int ftz_prove_transfers(ftz_ctx* c, size_t n, const ftz_transfer_witness* w, uint8_t* buf, size_t cap,
                                   size_t* offsets, int32_t* codes) {
  if (!c || (n && !w)) return set_err(FTZ_E_INVALID, "null argument");
  std::string e;
  if (!transfer_wit_ok(n, w, e)) return set_err(FTZ_E_INVALID, e);
  if (n == 0) {
    if (offsets) offsets[0] = 0;
    return FTZ_SUCCESS;
  }
  std::vector<TransferWit> t = to_wit(n, w);
  return prove_chunked(c, n, t.data(), 0, buf, cap, offsets, codes);
}

extern "C" int ftz_prove_issues(ftz_ctx* c, size_t n, const ftz_issue_witness* w, uint8_t* buf, size_t cap,
                                size_t* offsets, int32_t* codes) {
  if (!c || (n && !w)) return set_err(FTZ_E_INVALID, "null argument");
  std::string e;
  if (!issue_wit_ok(n, w, e)) return set_err(FTZ_E_INVALID, e);
  if (n == 0) {
    if (offsets) offsets[0] = 0;
    return FTZ_SUCCESS;
  }
  std::vector<IssueWit> t = to_wit(n, w);
  return prove_chunked(c, n, t.data(), 1, buf, cap, offsets, codes);
}

// ------------------------------------------------------------------ token openings
// Batches of up to 2^16 openings on the context's aux slot: H(type) (hash job),
// value / bf (scalar jobs), the 3-base fixed-base G1 job writing RawBytes into
// the arena, and -- for audits -- the commitment's decode job writing its
// canonical RawBytes next to it; the host then compares the two.
static int openings_run(ftz_ctx* c, size_t n, const ftz_token_opening* t, const uint8_t* coms, uint8_t* out,
                        int32_t* codes) {
  if (!c || (n && !t) || (n && !out && !codes)) return set_err(FTZ_E_INVALID, "null argument");
  for (size_t i = 0; i < n; i++)
    if (!t[i].value || !t[i].bf || (t[i].type_len && !t[i].type))
      return set_err(FTZ_E_INVALID, "null buffer in opening " + std::to_string(i));
  if (n == 0) return FTZ_SUCCESS;
  std::lock_guard<std::mutex> lk(c->aux_mu);
  HC(hipSetDevice(c->device));
  if (!c->aux) {
    ftz_batch* b = new ftz_batch();
    b->ctx = c;
    int rc = slot_init(b);
    if (rc != FTZ_SUCCESS) {
      slot_free(b);
      delete b;
      return rc;
    }
    c->aux = b;
  }
  ftz_batch* b = c->aux;
  const size_t B = (size_t)1 << 16;
  std::vector<PlanItem> items;
  std::vector<uint8_t> arena;
  for (size_t lo = 0; lo < n; lo += B) {
    size_t cnt = std::min(B, n - lo);
    items.assign(cnt, PlanItem{});
    for (size_t i = 0; i < cnt; i++) {
      const ftz_token_opening& o = t[lo + i];
      items[i].kind = 2;
      items[i].o = {o.type, o.type_len, o.value, o.bf, coms ? coms + 64 * (lo + i) : nullptr};
    }
    int rc = slot_plan_items(b, cnt, items.data());
    if (rc == FTZ_SUCCESS) rc = slot_submit(b, true, true);
    if (rc == FTZ_SUCCESS) rc = slot_wait(b);
    if (rc != FTZ_SUCCESS) return rc;
    arena.resize(b->fp.cnt[PS_ARENA]);
    HC(hipMemcpy(arena.data(), b->d_blob.p + b->fp.off[PS_ARENA], arena.size(), hipMemcpyDeviceToHost));
    const int32_t* vc = slot_codes(b);
    for (size_t i = 0; i < cnt; i++) {
      const uint8_t* r = arena.data() + b->fp.item_off[i];
      if (out) memcpy(out + 64 * (lo + i), r, 64);
      if (codes) codes[lo + i] = vc[i] != FTZ_OK ? vc[i] : (memcmp(r, r + 64, 64) == 0 ? FTZ_OK : FTZ_ERR_OPENING);
    }
  }
  return FTZ_SUCCESS;
}

extern "C" int ftz_commit_tokens(ftz_ctx* c, size_t n, const ftz_token_opening* t, uint8_t* out) {
  if (n && !out) return set_err(FTZ_E_INVALID, "null output");
  return openings_run(c, n, t, nullptr, out, nullptr);
}

extern "C" int ftz_audit_openings(ftz_ctx* c, size_t n, const uint8_t* commitments, const ftz_token_opening* t,
                                  int32_t* codes) {
  if (n && (!commitments || !codes)) return set_err(FTZ_E_INVALID, "null argument");
  return openings_run(c, n, t, commitments, nullptr, codes);
}

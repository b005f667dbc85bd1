// ftsamd: HIP runtime + kernels + C ABI (include/ftsamd.h).
//
// One context per GPU holds the public parameters in device form: fixed-base
// tables (8-bit windows) for Ped0..2, PedGen, the G1 generator and PK0..2, Q;
// the precomputed Miller lines of Q; and the canonical RawBytes of the PP
// points that every transcript hashes.  A batch is planned on the host
// (host/planner.cpp), uploaded once, and executed as a fixed sequence of
// job kernels on one HIP stream (see dev/jobs.h for the job model).
#include <hip/hip_runtime.h>
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

struct ftz_batch {
  ftz_ctx* ctx = nullptr;
  size_t n = 0;
  Plan plan;
  DBuf<uint8_t> wire, arena, pt_ok, canon, hash_ok_pre, hash_ok;
  DBuf<DecodeJob> dec;
  DBuf<ZrJob> zr;
  DBuf<ScalJob> sc;
  DBuf<uint32_t> sclist;
  DBuf<VTerm> vt;
  DBuf<G1Job> g1, g1p;
  DBuf<G2Job> g2;
  DBuf<PairJob> pr;
  DBuf<Seg> seg;
  DBuf<HashJob> hpre, hmain;
  DBuf<Check> ck;
  DBuf<TxChecks> tx;
  DBuf<G1Dev> pts, g1out;
  DBuf<G2Dev> g2out;
  DBuf<uint32_t> scal;  // 8 limbs per scalar
  DBuf<F12Dev> fbuf;
  DBuf<EvLineDev> lines2;  // pair-2 Miller lines, [line][pair job]
  DBuf<G1JDev> part1, part1p;  // G1 job parts (4 per job) of the side / pairing G1 jobs
  DBuf<G1Dev> vtab1, vtab1p;   // window tables of their variable parts (16 entries per job)
  DBuf<int32_t> codes;
  DBuf<uint32_t> bitmap;
  // prover
  DBuf<RandJob> rnd;
  DBuf<ScalJob> sc1, sc_post;
  DBuf<EmitJob> emit;
  DBuf<B64Job> b64;
  DBuf<uint8_t> out;
  hipEvent_t ev[20];
  bool ev_init = false;
  ftz_stats stats;
  // the batch's own streams (pairing chain, side G1 jobs, G2 jobs + lines), so
  // that several batches can be in flight at once (ftz_batch_submit)
  hipStream_t st[3] = {nullptr, nullptr, nullptr};
  bool pending = false;
  uint64_t jobs_last[FTZ_NKERNELS] = {};
};

// Same priorities as the context streams: the pairing chain high, the side G1
// jobs low.
static int batch_streams(ftz_batch* b) {
  if (b->st[0]) return FTZ_SUCCESS;
  int prio_lo = 0, prio_hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  HC(hipStreamCreateWithPriority(&b->st[0], hipStreamNonBlocking, prio_hi));
  HC(hipStreamCreateWithPriority(&b->st[1], hipStreamNonBlocking, prio_lo));
  HC(hipStreamCreateWithPriority(&b->st[2], hipStreamNonBlocking, prio_hi));
  return FTZ_SUCCESS;
}

static int blocks_for(uint32_t n, int bs) { return (int)((n + bs - 1) / bs); }

extern "C" const char* ftz_last_error(void) { return g_err.c_str(); }

extern "C" int ftz_ctx_create(const uint8_t* pp, size_t pp_len, int device, ftz_ctx** out) {
  if (!pp || !out) return set_err(FTZ_E_INVALID, "null argument");
  *out = nullptr;
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
  unsigned hc = std::thread::hardware_concurrency();
  c->threads = (int)std::max(1u, std::min(16u, hc ? hc : 8u));
  std::string e = parse_pp(pp, pp_len, "zkatdlog", c->pp);
  if (!e.empty()) {
    delete c;
    return set_err(FTZ_E_PP, e);
  }
  // The pairing chain (stream, stream3) gets the higher priority: the G1 jobs
  // no pairing depends on (stream2) fill the SIMDs the chain leaves idle.
  int prio_lo = 0, prio_hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  if (hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, prio_hi) != hipSuccess ||
      hipStreamCreateWithPriority(&c->stream2, hipStreamNonBlocking, prio_lo) != hipSuccess ||
      hipStreamCreateWithPriority(&c->stream3, hipStreamNonBlocking, prio_hi) != hipSuccess) {
    delete c;
    return set_err(FTZ_E_DEVICE, "hipStreamCreate failed");
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
  raw.resize(raw.size() + 128, 0);
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
        d_g2off.upload(g2off, c->stream) != hipSuccess || d_g1.alloc(5) != hipSuccess ||
        d_g2.alloc(4) != hipSuccess || d_g1b.alloc(64 * 5) != hipSuccess || d_g2b.alloc(128 * 4) != hipSuccess ||
        d_ok.alloc(9) != hipSuccess) {
      fail(FTZ_E_NOMEM, "device allocation failed");
      break;
    }
    k_pp_decode<<<1, 64, 0, c->stream>>>(d_raw.p, d_g1off.p, 5, d_g2off.p, 4, d_g1.p, d_g2.p, d_g1b.p, d_g2b.p,
                                         d_ok.p);
    uint8_t ok[9];
    std::vector<uint8_t> g1b(64 * 5), g2b(128 * 4);
    if (hipMemcpyAsync(ok, d_ok.p, 9, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipMemcpyAsync(g1b.data(), d_g1b.p, g1b.size(), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipMemcpyAsync(g2b.data(), d_g2b.p, g2b.size(), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
      fail(FTZ_E_DEVICE, std::string("public-parameter decode failed: ") + hipGetErrorString(hipGetLastError()));
      break;
    }
    bool allok = true;
    for (int k = 0; k < 9; k++) allok = allok && ok[k];
    if (!allok) {
      fail(FTZ_E_PP, "public parameters hold an invalid curve point");
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
    std::vector<G1Dev> got(5);
    if (hipMemcpy(got.data(), d_g1.p, 5 * sizeof(G1Dev), hipMemcpyDeviceToHost) != hipSuccess) {
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
    uint32_t n1 = G1B_COUNT * G1TAB_WINDOWS * G1TAB_DIGITS, n2 = G2B_COUNT * G2TAB_WINDOWS * G2TAB_DIGITS;
    if (c->g1tab.alloc(n1) != hipSuccess || c->g2tab.alloc(n2) != hipSuccess ||
        c->qlines.alloc(MILLER_LINES) != hipSuccess) {
      fail(FTZ_E_NOMEM, "table allocation failed");
      break;
    }
    DBuf<G1Dev> d_bw;
    DBuf<G1JDev> d_jt;
    DBuf<uint32_t> d_zs;
    if (G1TAB_C <= 8) {
      k_tab_g1<<<blocks_for(n1, 64), 64, 0, c->stream>>>(d_b1.p, n1, c->g1tab.p);
    } else {
      const uint32_t chunk = 128, lanes = G1B_COUNT * G1TAB_WINDOWS * (G1TAB_DIGITS / chunk);
      if (d_bw.alloc(G1B_COUNT * G1TAB_WINDOWS) != hipSuccess || d_jt.alloc(n1) != hipSuccess ||
          d_zs.alloc(8 * (size_t)n1) != hipSuccess) {
        fail(FTZ_E_NOMEM, "table scratch allocation failed");
        break;
      }
      k_tab_g1_bw<<<blocks_for(G1B_COUNT * G1TAB_WINDOWS, 64), 64, 0, c->stream>>>(d_b1.p, d_bw.p);
      k_tab_g1_fill<<<blocks_for(lanes, 128), 128, 0, c->stream>>>(
          d_bw.p, chunk, d_jt.p, reinterpret_cast<uint32_t (*)[8]>(d_zs.p), c->g1tab.p);
    }
    DBuf<G2Dev> d_bw2;
    DBuf<uint32_t> d_jt2, d_zs2;
    if (G2TAB_C <= 8) {
      k_tab_g2<<<blocks_for(n2, 64), 64, 0, c->stream>>>(d_g2.p, n2, c->g2tab.p);  // PK0, PK1, PK2, Q
    } else {
      const uint32_t chunk = 64, lanes = G2B_COUNT * G2TAB_WINDOWS * (G2TAB_DIGITS / chunk);
      if (d_bw2.alloc(G2B_COUNT * G2TAB_WINDOWS) != hipSuccess || d_jt2.alloc(48 * (size_t)n2) != hipSuccess ||
          d_zs2.alloc(16 * (size_t)n2) != hipSuccess) {
        fail(FTZ_E_NOMEM, "table scratch allocation failed");
        break;
      }
      k_tab_g2_bw<<<blocks_for(G2B_COUNT * G2TAB_WINDOWS, 64), 64, 0, c->stream>>>(d_g2.p, d_bw2.p);
      k_tab_g2_fill<<<blocks_for(lanes, 128), 128, 0, c->stream>>>(
          d_bw2.p, chunk, reinterpret_cast<uint32_t (*)[48]>(d_jt2.p), reinterpret_cast<uint32_t (*)[16]>(d_zs2.p),
          c->g2tab.p);
    }
    DBuf<int> d_n;
    if (d_n.alloc(1) != hipSuccess) {
      fail(FTZ_E_NOMEM, "alloc");
      break;
    }
    k_qlines<<<1, 64, 0, c->stream>>>(d_g2.p + 3, c->qlines.p, d_n.p);
    int nl = 0;
    if (hipMemcpyAsync(&nl, d_n.p, sizeof(int), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess || nl != MILLER_LINES) {
      fail(FTZ_E_DEVICE, std::string("context setup kernels failed: ") + hipGetErrorString(hipGetLastError()));
      break;
    }
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
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  c->g1tab.alloc(0);
  c->g2tab.alloc(0);
  c->qlines.alloc(0);
  if (c->stream2) (void)hipStreamDestroy(c->stream2);
  if (c->stream3) (void)hipStreamDestroy(c->stream3);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

extern "C" int ftz_ctx_set_threads(ftz_ctx* c, int threads) {
  if (!c || threads < 1) return set_err(FTZ_E_INVALID, "bad argument");
  c->threads = threads;
  return FTZ_SUCCESS;
}

extern "C" int ftz_ctx_info(const ftz_ctx* c, uint32_t* base, uint32_t* exponent) {
  if (!c) return set_err(FTZ_E_INVALID, "null context");
  if (base) *base = c->pp.base;
  if (exponent) *exponent = (uint32_t)c->pp.exponent;
  return FTZ_SUCCESS;
}

static int batch_upload(ftz_batch* b) {
  ftz_ctx* c = b->ctx;
  Plan& p = b->plan;
  int rc = batch_streams(b);
  if (rc != FTZ_SUCCESS) return rc;
  hipStream_t s = b->st[0];
  memcpy(p.arena.data(), c->const_bytes.data(), C_SIZE);
  std::vector<uint8_t> wire = p.wire;
  wire.resize(wire.size() + 64, 0);  // decode jobs may look at 64 bytes past a short element
  HC(b->wire.upload(wire, s));
  HC(b->arena.upload(p.arena, s));
  HC(b->dec.upload(p.dec, s));
  HC(b->zr.upload(p.zr, s));
  HC(b->sc.upload(p.sc, s));
  HC(b->sclist.upload(p.sclist, s));
  HC(b->vt.upload(p.vt, s));
  HC(b->g1.upload(p.g1, s));
  HC(b->g1p.upload(p.g1p, s));
  HC(b->g2.upload(p.g2, s));
  HC(b->pr.upload(p.pr, s));
  HC(b->seg.upload(p.seg, s));
  HC(b->hpre.upload(p.hpre, s));
  HC(b->hmain.upload(p.hmain, s));
  HC(b->ck.upload(p.ck, s));
  HC(b->tx.upload(p.tx, s));
  HC(b->pts.alloc(std::max<uint32_t>(p.n_pts, 1)));
  HC(b->pt_ok.alloc(std::max<uint32_t>(p.n_pts, 1)));
  HC(b->scal.alloc(8 * (size_t)std::max<uint32_t>(p.n_scal, 1)));
  HC(b->canon.alloc(std::max<uint32_t>(p.n_scal, 1)));
  HC(b->g1out.alloc(std::max<uint32_t>(p.n_g1out, 1)));
  HC(b->g2out.alloc(std::max<uint32_t>(p.n_g2out, 1)));
  HC(b->fbuf.alloc(std::max<size_t>(p.pr.size(), 1)));
  HC(b->lines2.alloc(std::max<size_t>(p.pr.size(), 1) * MILLER_LINES));
  HC(b->part1.alloc(4 * std::max<size_t>(p.g1.size(), 1)));
  HC(b->part1p.alloc(4 * std::max<size_t>(p.g1p.size(), 1)));
  HC(b->vtab1.alloc(16 * std::max<size_t>(p.g1.size(), 1)));
  HC(b->vtab1p.alloc(16 * std::max<size_t>(p.g1p.size(), 1)));
  if (p.g2.size() != p.pr.size()) return set_err(FTZ_E_INVALID, "planner: G2 and pairing jobs out of step");
  for (size_t i = 0; i < p.pr.size(); i++)
    if (p.pr[i].q2 != p.g2[i].out) return set_err(FTZ_E_INVALID, "planner: G2 and pairing jobs out of step");
  HC(b->rnd.upload(p.rnd, s));
  HC(b->sc1.upload(p.sc1, s));
  HC(b->sc_post.upload(p.sc_post, s));
  HC(b->emit.upload(p.emit, s));
  HC(b->b64.upload(p.b64, s));
  HC(b->out.upload(p.out, s));
  HC(b->hash_ok.alloc(std::max<size_t>(p.hmain.size(), 1)));
  HC(b->hash_ok_pre.alloc(std::max<size_t>(p.hpre.size(), 1)));
  HC(b->codes.alloc(std::max<size_t>(b->n, 1)));
  HC(b->bitmap.alloc((b->n + 31) / 32 + 1));
  HC(hipMemsetAsync(b->pt_ok.p, 1, std::max<uint32_t>(p.n_pts, 1), s));
  HC(hipStreamSynchronize(s));
  if (!b->ev_init) {
    for (int k = 0; k < 20; k++) HC(hipEventCreate(&b->ev[k]));
    b->ev_init = true;
  }
  return FTZ_SUCCESS;
}

extern "C" int ftz_batch_load_transfers(ftz_ctx* c, size_t n, const ftz_transfer* tx, ftz_batch** out) {
  if (!c || !out || (n && !tx)) return set_err(FTZ_E_INVALID, "null argument");
  for (size_t i = 0; i < n; i++)
    if ((tx[i].n_in && !tx[i].inputs) || (tx[i].n_out && !tx[i].outputs) || (tx[i].proof_len && !tx[i].proof))
      return set_err(FTZ_E_INVALID, "null buffer in transfer");
  std::lock_guard<std::mutex> lk(c->mu);
  HC(hipSetDevice(c->device));
  ftz_batch* b = new ftz_batch();
  b->ctx = c;
  b->n = n;
  std::vector<TransferIn> t(n);
  for (size_t i = 0; i < n; i++)
    t[i] = {tx[i].inputs, tx[i].n_in, tx[i].outputs, tx[i].n_out, tx[i].proof, tx[i].proof_len};
  plan_transfers(c->pp, n, t.data(), b->plan, c->threads);
  int rc = batch_upload(b);
  if (rc != FTZ_SUCCESS) {
    ftz_batch_destroy(b);
    return rc;
  }
  *out = b;
  return FTZ_SUCCESS;
}

extern "C" int ftz_batch_load_issues(ftz_ctx* c, size_t n, const ftz_issue* is, ftz_batch** out) {
  if (!c || !out || (n && !is)) return set_err(FTZ_E_INVALID, "null argument");
  for (size_t i = 0; i < n; i++)
    if ((is[i].n_out && !is[i].outputs) || (is[i].proof_len && !is[i].proof))
      return set_err(FTZ_E_INVALID, "null buffer in issue");
  std::lock_guard<std::mutex> lk(c->mu);
  HC(hipSetDevice(c->device));
  ftz_batch* b = new ftz_batch();
  b->ctx = c;
  b->n = n;
  std::vector<IssueIn> t(n);
  for (size_t i = 0; i < n; i++) t[i] = {is[i].outputs, is[i].n_out, is[i].proof, is[i].proof_len, is[i].anonymous};
  plan_issues(c->pp, n, t.data(), b->plan, c->threads);
  int rc = batch_upload(b);
  if (rc != FTZ_SUCCESS) {
    ftz_batch_destroy(b);
    return rc;
  }
  *out = b;
  return FTZ_SUCCESS;
}

// Three streams after the light decode/scalar kernels:
//   stream3: G2 jobs t' and the pair-2 Miller lines evaluated at R (k_g2lines)
//   stream : G1 jobs feeding the pairings (P1 = sbf*P - c*S), then, after
//            stream3, the sextet Miller loops and final exponentiations
//   stream2: the G1 jobs no pairing depends on (well-formedness, range
//            equality, membership Schnorr commitments)
// The transcript hashes wait for all three.
extern "C" int ftz_batch_submit(ftz_batch* b) {
  if (!b) return set_err(FTZ_E_INVALID, "null batch");
  ftz_ctx* c = b->ctx;
  std::lock_guard<std::mutex> lk(c->mu);
  HC(hipSetDevice(c->device));
  Plan& p = b->plan;
  hipStream_t s = b->st[0], s2 = b->st[1], s3 = b->st[2];
  // FTZ_SERIAL=1: run every kernel on one stream (per-kernel timings without
  // overlap, for profiling)
  const bool serial = getenv("FTZ_SERIAL") && getenv("FTZ_SERIAL")[0] == '1';  // read per run (bench toggles it)
  // FTZ_BATCH_STREAMS=1: the whole batch on its pairing-chain stream (several
  // batches in flight then overlap each other instead)
  const bool one = getenv("FTZ_BATCH_STREAMS") && getenv("FTZ_BATCH_STREAMS")[0] == '1';
  if (serial || one) s2 = s3 = s;
  uint32_t (*scal)[8] = reinterpret_cast<uint32_t (*)[8]>(b->scal.p);
  uint32_t n_dec = (uint32_t)p.dec.size(), n_zr = (uint32_t)p.zr.size(), n_sc = (uint32_t)p.sc.size();
  uint32_t n_g1 = (uint32_t)p.g1.size(), n_g1p = (uint32_t)p.g1p.size(), n_g2 = (uint32_t)p.g2.size();
  uint32_t n_pr = (uint32_t)p.pr.size();
  uint32_t n_hp = (uint32_t)p.hpre.size(), n_hm = (uint32_t)p.hmain.size(), n_tx = (uint32_t)p.tx.size();
  const uint64_t jobs[FTZ_NKERNELS] = {n_dec, n_zr, n_hp, n_sc, n_g1p, n_g2, n_pr, n_pr, n_g1, n_hm, n_tx, n_tx};
  for (int k = 0; k < FTZ_NKERNELS; k++) b->jobs_last[k] = jobs[k];
  hipEvent_t* e = b->ev;
  HC(hipMemsetAsync(b->bitmap.p, 0, b->bitmap.n * sizeof(uint32_t), s));
  HC(hipEventRecord(e[0], s));
  if (n_dec) k_decode<<<blocks_for(n_dec, 256), 256, 0, s>>>(b->dec.p, n_dec, b->wire.p, b->pts.p, b->pt_ok.p, b->arena.p);
  HC(hipEventRecord(e[1], s));
  if (n_zr) k_zr<<<blocks_for(n_zr, 256), 256, 0, s>>>(b->zr.p, n_zr, b->wire.p, scal, b->canon.p);
  HC(hipEventRecord(e[2], s));
  if (n_hp)
    k_hash<<<blocks_for(n_hp, 128), 128, 0, s>>>(b->hpre.p, n_hp, b->seg.p, b->arena.p, scal, b->canon.p,
                                                 b->hash_ok_pre.p);
  HC(hipEventRecord(e[3], s));
  if (n_sc) k_scalar<<<blocks_for(n_sc, 256), 256, 0, s>>>(b->sc.p, n_sc, scal, b->sclist.p);
  HC(hipEventRecord(e[4], s));
  // stream3: G2 jobs + pair-2 lines
  HC(hipStreamWaitEvent(s3, e[4], 0));
  HC(hipEventRecord(e[14], s3));
  if (n_g2)
    k_g2lines<<<blocks_for(n_g2, SX_JOBS_PER_WAVE), 64, 0, s3>>>(b->g2.p, b->pr.p, n_g2, scal, c->g2tab.p, b->g2out.p, b->pts.p,
                                                   b->lines2.p);
  HC(hipEventRecord(e[15], s3));
  // main stream: pairing chain
  HC(hipEventRecord(e[16], s));
  if (n_g1p) {
    k_g1_part<<<blocks_for(4 * n_g1p, 128), 128, 0, s>>>(b->g1p.p, n_g1p, b->vt.p, b->pts.p, scal, c->g1tab.p,
                                                         b->part1p.p, b->vtab1p.p);
    k_g1_combine<<<blocks_for(n_g1p, 256), 256, 0, s>>>(b->g1p.p, n_g1p, b->part1p.p, b->g1out.p, b->arena.p);
  }
  HC(hipEventRecord(e[5], s));
  // stream2: pairing-independent G1 jobs, started after the jobs the pairing
  // chain waits for (FTZ_G1_AFTER: 0 with them, 1 after the pairing G1 jobs,
  // 2 after the G2 jobs and lines)
  const char* ga = getenv("FTZ_G1_AFTER");
  const int g1_after = ga ? atoi(ga) : 0;
  HC(hipStreamWaitEvent(s2, g1_after == 1 ? e[5] : (g1_after == 2 ? e[15] : e[4]), 0));
  HC(hipEventRecord(e[11], s2));
  if (n_g1) {
    k_g1_part<<<blocks_for(4 * n_g1, 128), 128, 0, s2>>>(b->g1.p, n_g1, b->vt.p, b->pts.p, scal, c->g1tab.p,
                                                         b->part1.p, b->vtab1.p);
    k_g1_combine<<<blocks_for(n_g1, 256), 256, 0, s2>>>(b->g1.p, n_g1, b->part1.p, b->g1out.p, b->arena.p);
  }
  HC(hipEventRecord(e[12], s2));
  HC(hipStreamWaitEvent(s, e[15], 0));
  HC(hipEventRecord(e[6], s));
  if (n_pr)
    k_miller<<<blocks_for(n_pr, SX_JOBS_PER_WAVE), 64, 0, s>>>(b->pr.p, n_pr, c->qlines.p, b->lines2.p, b->g1out.p,
                                                               b->fbuf.p);
  HC(hipEventRecord(e[7], s));
  if (n_pr) k_fexp<<<blocks_for(n_pr, SX_JOBS_PER_WAVE), 64, 0, s>>>(b->pr.p, n_pr, b->fbuf.p, b->arena.p);
  HC(hipEventRecord(e[8], s));
  HC(hipStreamWaitEvent(s, e[12], 0));
  HC(hipEventRecord(e[9], s));
  if (n_hm)
    k_hash<<<blocks_for(n_hm, 128), 128, 0, s>>>(b->hmain.p, n_hm, b->seg.p, b->arena.p, scal, b->canon.p,
                                                 b->hash_ok.p);
  HC(hipEventRecord(e[10], s));
  if (n_tx)
    k_verdict<<<blocks_for(n_tx, 256), 256, 0, s>>>(b->tx.p, n_tx, b->ck.p, b->pt_ok.p, b->hash_ok.p, b->codes.p,
                                                    b->bitmap.p);
  HC(hipEventRecord(e[13], s));
  HC(hipGetLastError());
  b->pending = true;
  return FTZ_SUCCESS;
}

// Wait for the batch's last submission and collect its per-kernel timings.
extern "C" int ftz_batch_wait(ftz_batch* b) {
  if (!b) return set_err(FTZ_E_INVALID, "null batch");
  if (!b->pending) return FTZ_SUCCESS;
  HC(hipSetDevice(b->ctx->device));
  HC(hipStreamSynchronize(b->st[0]));
  b->pending = false;
  hipEvent_t* e = b->ev;
  // stats order: decode zr hash_pre scalar g1p g2+lines miller fexp g1(side) hash verdict total
  const int from[FTZ_NKERNELS] = {0, 1, 2, 3, 16, 14, 6, 7, 11, 9, 10, 0};
  const int to[FTZ_NKERNELS] = {1, 2, 3, 4, 5, 15, 7, 8, 12, 10, 13, 13};
  for (int k = 0; k < FTZ_NKERNELS; k++) {
    float ms = 0;
    HC(hipEventElapsedTime(&ms, e[from[k]], e[to[k]]));
    b->stats.ms[k] = ms;
    b->stats.jobs[k] = b->jobs_last[k];
  }
  return FTZ_SUCCESS;
}

extern "C" int ftz_batch_run(ftz_batch* b) {
  int rc = ftz_batch_submit(b);
  return rc == FTZ_SUCCESS ? ftz_batch_wait(b) : rc;
}

extern "C" int ftz_batch_codes(ftz_batch* b, int32_t* codes) {
  if (!b || (b->n && !codes)) return set_err(FTZ_E_INVALID, "null argument");
  if (b->pending) {
    int rc = ftz_batch_wait(b);
    if (rc != FTZ_SUCCESS) return rc;
  }
  HC(hipSetDevice(b->ctx->device));
  if (b->n) HC(hipMemcpy(codes, b->codes.p, b->n * sizeof(int32_t), hipMemcpyDeviceToHost));
  return FTZ_SUCCESS;
}

extern "C" int ftz_batch_bitmap(ftz_batch* b, uint8_t* bits) {
  if (!b || (b->n && !bits)) return set_err(FTZ_E_INVALID, "null argument");
  if (b->pending) {
    int rc = ftz_batch_wait(b);
    if (rc != FTZ_SUCCESS) return rc;
  }
  HC(hipSetDevice(b->ctx->device));
  std::vector<uint32_t> w((b->n + 31) / 32);
  if (!w.empty()) HC(hipMemcpy(w.data(), b->bitmap.p, w.size() * 4, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < (b->n + 7) / 8; i++) bits[i] = (uint8_t)(w[i / 4] >> (8 * (i % 4)));
  return FTZ_SUCCESS;
}

extern "C" int ftz_batch_stats(const ftz_batch* b, ftz_stats* out) {
  if (!b || !out) return set_err(FTZ_E_INVALID, "null argument");
  *out = b->stats;
  return FTZ_SUCCESS;
}

extern "C" size_t ftz_batch_size(const ftz_batch* b) { return b ? b->n : 0; }

extern "C" void ftz_batch_destroy(ftz_batch* b) {
  if (!b) return;
  (void)hipSetDevice(b->ctx->device);
  for (int k = 0; k < 3; k++)
    if (b->st[k]) (void)hipStreamSynchronize(b->st[k]);
  if (b->ev_init)
    for (int k = 0; k < 20; k++) (void)hipEventDestroy(b->ev[k]);
  for (int k = 0; k < 3; k++)
    if (b->st[k]) (void)hipStreamDestroy(b->st[k]);
  delete b;
}

extern "C" int ftz_verify_transfers(ftz_ctx* c, size_t n, const ftz_transfer* tx, int32_t* codes) {
  if (n == 0) return FTZ_SUCCESS;
  ftz_batch* b = nullptr;
  int rc = ftz_batch_load_transfers(c, n, tx, &b);
  if (rc == FTZ_SUCCESS) rc = ftz_batch_run(b);
  if (rc == FTZ_SUCCESS) rc = ftz_batch_codes(b, codes);
  ftz_batch_destroy(b);
  return rc;
}

extern "C" int ftz_verify_issues(ftz_ctx* c, size_t n, const ftz_issue* is, int32_t* codes) {
  if (n == 0) return FTZ_SUCCESS;
  ftz_batch* b = nullptr;
  int rc = ftz_batch_load_issues(c, n, is, &b);
  if (rc == FTZ_SUCCESS) rc = ftz_batch_run(b);
  if (rc == FTZ_SUCCESS) rc = ftz_batch_codes(b, codes);
  ftz_batch_destroy(b);
  return rc;
}

// ------------------------------------------------------------------ prover
// Plans from host/planner_prove.cpp; the pipeline of ftz_batch_run with the
// prover's extra stages: randomness before the group work, responses, JSON
// hole filling and base64 of the inner documents after the transcript hashes.
struct ftz_prover : ftz_batch {};

template <class W, class In, class Plan_fn>
static int prover_load(ftz_ctx* c, size_t n, const W* w, ftz_prover** out, Plan_fn plan) {
  if (!c || !out || (n && !w)) return set_err(FTZ_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(c->mu);
  HC(hipSetDevice(c->device));
  ftz_prover* b = new ftz_prover();
  b->ctx = c;
  b->n = n;
  std::string e = plan(b->plan);
  if (!e.empty()) {
    delete b;
    return set_err(FTZ_E_INVALID, e);
  }
  int rc = batch_upload(b);
  if (rc != FTZ_SUCCESS) {
    delete b;
    return rc;
  }
  *out = b;
  return FTZ_SUCCESS;
}

static bool seeds_ok(const uint8_t* seed) { return seed != nullptr; }

extern "C" int ftz_prover_load_transfers(ftz_ctx* c, size_t n, const ftz_transfer_witness* w, ftz_prover** out) {
  for (size_t i = 0; i < n && w; i++)
    if ((w[i].n_in && (!w[i].inputs || !w[i].in_values || !w[i].in_bfs)) ||
        (w[i].n_out && (!w[i].outputs || !w[i].out_values || !w[i].out_bfs)) || !seeds_ok(w[i].seed) ||
        (w[i].type_len && !w[i].type))
      return set_err(FTZ_E_INVALID, "null buffer in witness " + std::to_string(i));
  return prover_load<ftz_transfer_witness, TransferWit>(c, n, w, out, [&](Plan& p) {
    std::vector<TransferWit> t(n);
    for (size_t i = 0; i < n; i++)
      t[i] = {w[i].inputs, w[i].n_in, w[i].outputs, w[i].n_out, w[i].in_values, w[i].in_bfs,
              w[i].out_values, w[i].out_bfs, w[i].type, w[i].type_len, w[i].seed};
    return plan_prove_transfers(c->pp, n, t.data(), p, c->threads);
  });
}

extern "C" int ftz_prover_load_issues(ftz_ctx* c, size_t n, const ftz_issue_witness* w, ftz_prover** out) {
  for (size_t i = 0; i < n && w; i++)
    if ((w[i].n_out && (!w[i].outputs || !w[i].values || !w[i].bfs)) || !seeds_ok(w[i].seed) ||
        (w[i].type_len && !w[i].type))
      return set_err(FTZ_E_INVALID, "null buffer in witness " + std::to_string(i));
  return prover_load<ftz_issue_witness, IssueWit>(c, n, w, out, [&](Plan& p) {
    std::vector<IssueWit> t(n);
    for (size_t i = 0; i < n; i++)
      t[i] = {w[i].outputs, w[i].n_out, w[i].values, w[i].bfs, w[i].type, w[i].type_len, w[i].anonymous, w[i].seed};
    return plan_prove_issues(c->pp, n, t.data(), p, c->threads);
  });
}

extern "C" int ftz_prover_submit(ftz_prover* b) {
  if (!b) return set_err(FTZ_E_INVALID, "null prover");
  ftz_ctx* c = b->ctx;
  std::lock_guard<std::mutex> lk(c->mu);
  HC(hipSetDevice(c->device));
  Plan& p = b->plan;
  hipStream_t s = b->st[0], s2 = b->st[1], s3 = b->st[2];
  const bool serial = getenv("FTZ_SERIAL") && getenv("FTZ_SERIAL")[0] == '1';  // read per run (bench toggles it)
  if (serial) s2 = s3 = s;
  uint32_t (*scal)[8] = reinterpret_cast<uint32_t (*)[8]>(b->scal.p);
  uint32_t n_dec = (uint32_t)p.dec.size(), n_zr = (uint32_t)p.zr.size(), n_sc = (uint32_t)p.sc.size();
  uint32_t n_rnd = (uint32_t)p.rnd.size(), n_sp = (uint32_t)p.sc_post.size(), n_em = (uint32_t)p.emit.size();
  uint32_t n_b64 = (uint32_t)p.b64.size();
  uint32_t n_g1 = (uint32_t)p.g1.size(), n_g1p = (uint32_t)p.g1p.size(), n_g2 = (uint32_t)p.g2.size();
  uint32_t n_pr = (uint32_t)p.pr.size();
  uint32_t n_hp = (uint32_t)p.hpre.size(), n_hm = (uint32_t)p.hmain.size(), n_tx = (uint32_t)p.tx.size();
  uint64_t jobs[FTZ_NKERNELS] = {n_dec, n_zr, (uint64_t)n_rnd + n_hp, n_sc, n_g1p, n_g2, n_pr, n_pr, n_g1,
                                 (uint64_t)n_hm + n_sp, (uint64_t)n_em + n_b64, n_tx};
  hipEvent_t* e = b->ev;
  HC(hipMemsetAsync(b->bitmap.p, 0, b->bitmap.n * sizeof(uint32_t), s));
  HC(hipEventRecord(e[0], s));
  if (n_dec) k_decode<<<blocks_for(n_dec, 256), 256, 0, s>>>(b->dec.p, n_dec, b->wire.p, b->pts.p, b->pt_ok.p, b->arena.p);
  HC(hipEventRecord(e[1], s));
  if (n_zr) k_zr<<<blocks_for(n_zr, 256), 256, 0, s>>>(b->zr.p, n_zr, b->wire.p, scal, b->canon.p);
  HC(hipEventRecord(e[2], s));
  if (n_rnd) k_rand<<<blocks_for(n_rnd, 128), 128, 0, s>>>(b->rnd.p, n_rnd, b->arena.p, scal);
  if (n_hp)
    k_hash<<<blocks_for(n_hp, 128), 128, 0, s>>>(b->hpre.p, n_hp, b->seg.p, b->arena.p, scal, b->canon.p,
                                                 b->hash_ok_pre.p);
  HC(hipEventRecord(e[3], s));
  if (n_sc) k_scalar<<<blocks_for(n_sc, 256), 256, 0, s>>>(b->sc.p, n_sc, scal, b->sclist.p);
  uint32_t n_sc1 = (uint32_t)p.sc1.size();
  if (n_sc1) k_scalar<<<blocks_for(n_sc1, 256), 256, 0, s>>>(b->sc1.p, n_sc1, scal, b->sclist.p);
  HC(hipEventRecord(e[4], s));
  // stream2: G1 jobs no pairing depends on
  HC(hipStreamWaitEvent(s2, e[4], 0));
  HC(hipEventRecord(e[11], s2));
  if (n_g1) {
    k_g1_part<<<blocks_for(4 * n_g1, 128), 128, 0, s2>>>(b->g1.p, n_g1, b->vt.p, b->pts.p, scal, c->g1tab.p,
                                                         b->part1.p, b->vtab1.p);
    k_g1_combine<<<blocks_for(n_g1, 256), 256, 0, s2>>>(b->g1.p, n_g1, b->part1.p, b->g1out.p, b->arena.p);
  }
  HC(hipEventRecord(e[12], s2));
  // main: R' = rr R and rsbf P (the pairing inputs)
  HC(hipEventRecord(e[16], s));
  if (n_g1p) {
    k_g1_part<<<blocks_for(4 * n_g1p, 128), 128, 0, s>>>(b->g1p.p, n_g1p, b->vt.p, b->pts.p, scal, c->g1tab.p,
                                                         b->part1p.p, b->vtab1p.p);
    k_g1_combine<<<blocks_for(n_g1p, 256), 256, 0, s>>>(b->g1p.p, n_g1p, b->part1p.p, b->g1out.p, b->arena.p);
  }
  HC(hipEventRecord(e[5], s));
  // stream3: t = rv PK1 + rh PK2 and its lines evaluated at R' (pair 2 reads g1out)
  HC(hipStreamWaitEvent(s3, e[5], 0));
  HC(hipEventRecord(e[14], s3));
  if (n_g2)
    k_g2lines<<<blocks_for(n_g2, SX_JOBS_PER_WAVE), 64, 0, s3>>>(b->g2.p, b->pr.p, n_g2, scal, c->g2tab.p,
                                                                 b->g2out.p, b->g1out.p, b->lines2.p);
  HC(hipEventRecord(e[15], s3));
  HC(hipStreamWaitEvent(s, e[15], 0));
  HC(hipEventRecord(e[6], s));
  if (n_pr)
    k_miller<<<blocks_for(n_pr, SX_JOBS_PER_WAVE), 64, 0, s>>>(b->pr.p, n_pr, c->qlines.p, b->lines2.p, b->g1out.p,
                                                               b->fbuf.p);
  HC(hipEventRecord(e[7], s));
  if (n_pr) k_fexp<<<blocks_for(n_pr, SX_JOBS_PER_WAVE), 64, 0, s>>>(b->pr.p, n_pr, b->fbuf.p, b->arena.p);
  HC(hipEventRecord(e[8], s));
  HC(hipStreamWaitEvent(s, e[12], 0));
  HC(hipEventRecord(e[9], s));
  if (n_hm)
    k_hash<<<blocks_for(n_hm, 128), 128, 0, s>>>(b->hmain.p, n_hm, b->seg.p, b->arena.p, scal, b->canon.p,
                                                 b->hash_ok.p);
  if (n_sp) k_scalar<<<blocks_for(n_sp, 256), 256, 0, s>>>(b->sc_post.p, n_sp, scal, b->sclist.p);
  HC(hipEventRecord(e[10], s));
  if (n_em) k_emit<<<blocks_for(n_em, 256), 256, 0, s>>>(b->emit.p, n_em, scal, b->arena.p);
  if (n_b64) k_b64<<<n_b64, 256, 0, s>>>(b->b64.p, n_b64, b->arena.p, b->out.p);
  HC(hipEventRecord(e[13], s));
  if (n_tx)
    k_verdict<<<blocks_for(n_tx, 256), 256, 0, s>>>(b->tx.p, n_tx, b->ck.p, b->pt_ok.p, b->hash_ok.p, b->codes.p,
                                                    b->bitmap.p);
  HC(hipGetLastError());
  for (int k = 0; k < FTZ_NKERNELS; k++) b->jobs_last[k] = jobs[k];
  b->pending = true;
  return FTZ_SUCCESS;
}

extern "C" int ftz_prover_wait(ftz_prover* b) {
  if (!b) return set_err(FTZ_E_INVALID, "null prover");
  if (!b->pending) return FTZ_SUCCESS;
  HC(hipSetDevice(b->ctx->device));
  HC(hipStreamSynchronize(b->st[0]));
  b->pending = false;
  hipEvent_t* e = b->ev;
  // stats order: decode zr rand+hash_pre scalar g1p g2+lines miller fexp g1(side) hash+responses emit+b64 total
  const int from[FTZ_NKERNELS] = {0, 1, 2, 3, 16, 14, 6, 7, 11, 9, 10, 0};
  const int to[FTZ_NKERNELS] = {1, 2, 3, 4, 5, 15, 7, 8, 12, 10, 13, 13};
  for (int k = 0; k < FTZ_NKERNELS; k++) {
    float ms = 0;
    HC(hipEventElapsedTime(&ms, e[from[k]], e[to[k]]));
    b->stats.ms[k] = ms;
    b->stats.jobs[k] = b->jobs_last[k];
  }
  return FTZ_SUCCESS;
}

extern "C" int ftz_prover_run(ftz_prover* b) {
  int rc = ftz_prover_submit(b);
  return rc == FTZ_SUCCESS ? ftz_prover_wait(b) : rc;
}

extern "C" size_t ftz_prover_bytes(const ftz_prover* b) { return b ? b->plan.out.size() : 0; }

extern "C" int ftz_prover_proofs(ftz_prover* b, uint8_t* buf, size_t cap, size_t* offsets, int32_t* codes) {
  if (!b) return set_err(FTZ_E_INVALID, "null prover");
  const Plan& p = b->plan;
  if (cap < p.out.size() || (p.out.size() && !buf)) return set_err(FTZ_E_INVALID, "proof buffer too small");
  if (b->pending) {
    int rc = ftz_prover_wait(b);
    if (rc != FTZ_SUCCESS) return rc;
  }
  HC(hipSetDevice(b->ctx->device));
  hipStream_t s = b->st[0];
  if (p.out.size()) HC(hipMemcpyAsync(buf, b->out.p, p.out.size(), hipMemcpyDeviceToHost, s));
  if (codes && b->n) HC(hipMemcpyAsync(codes, b->codes.p, b->n * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HC(hipStreamSynchronize(s));
  if (offsets) {
    for (size_t i = 0; i < b->n; i++) offsets[i] = p.out_off[i];
    offsets[b->n] = p.out.size();
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
  if (b->ev_init)
    for (int k = 0; k < 20; k++) (void)hipEventDestroy(b->ev[k]);
  delete b;
}

template <class W, class Load>
static int prove_once(ftz_ctx* c, size_t n, const W* w, uint8_t* buf, size_t cap, size_t* offsets, int32_t* codes,
                      Load load) {
  ftz_prover* p = nullptr;
  int rc = load(c, n, w, &p);
  if (rc != FTZ_SUCCESS) return rc;
  rc = ftz_prover_run(p);
  if (rc == FTZ_SUCCESS) rc = ftz_prover_proofs(p, buf, cap, offsets, codes);
  ftz_prover_destroy(p);
  return rc;
}

extern "C" int ftz_prove_transfers(ftz_ctx* c, size_t n, const ftz_transfer_witness* w, uint8_t* buf, size_t cap,
                                   size_t* offsets, int32_t* codes) {
  return prove_once(c, n, w, buf, cap, offsets, codes, ftz_prover_load_transfers);
}

extern "C" int ftz_prove_issues(ftz_ctx* c, size_t n, const ftz_issue_witness* w, uint8_t* buf, size_t cap,
                                size_t* offsets, int32_t* codes) {
  return prove_once(c, n, w, buf, cap, offsets, codes, ftz_prover_load_issues);
}

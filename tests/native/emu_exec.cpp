// TEST-ONLY: runs the product's planner (host/planner.cpp) and the device job
// functions (dev/jobs.h) on the CPU, in the same order as the HIP kernels in
// runtime.hip, so the CPU test tier can check the complete verification
// pipeline against the Python oracle without a GPU.  The product library
// (libftsamd.so) contains no CPU execution path; this file is never part of it.
#include <string.h>

#include <algorithm>
#include <chrono>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../fabric-token-sdk_amd/csrc/dev/jobs.h"
#include "../../fabric-token-sdk_amd/csrc/host/planner.h"
#include "../../fabric-token-sdk_amd/csrc/host/request.h"
#include "../../include/ftsamd.h"

using namespace fts;
using namespace ftsh;

#ifdef FTS_COUNT_OPS
thread_local unsigned long long fts_mont_count = 0;
#endif

struct EmuCtx {
  PPInfo pp;
  std::vector<uint8_t> const_bytes;
  std::vector<G1Dev> g1tab;  // + the prover's signature-point bases once built (G1B_SIG0 ..)
  std::mutex sig_mu;
  bool sig_ready = false;
  std::vector<G2Dev> g2tab;
  std::vector<LineCoef> pklines;  // PK1 then PK2 (the prover's fixed-pair Miller loops)
  std::vector<LineCoef> qlines;
  int fexp = 0;  // 0: exact (FTZ_FEXP_EXACT), 1: Fuentes
};

static unsigned g_threads = 0;  // 0: all hardware threads

template <class F>
static void par_for(uint32_t n, F f) {
  unsigned t = g_threads ? g_threads : std::max(1u, std::thread::hardware_concurrency());
  std::vector<std::thread> th;
  for (unsigned k = 0; k < t; k++)
    th.emplace_back([&, k]() {
      for (uint32_t i = k; i < n; i += t) f(i);
    });
  for (auto& x : th) x.join();
}

extern "C" {

void* emu_ctx_create(const uint8_t* pp, size_t len, char* err, size_t errlen) {
  EmuCtx* c = new EmuCtx();
  std::string e = parse_pp(pp, len, "zkatdlog", c->pp);
  if (!e.empty()) {
    snprintf(err, errlen, "%s", e.c_str());
    delete c;
    return nullptr;
  }
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
  std::vector<G1Dev> g1(5);
  std::vector<G2Dev> g2(4);
  std::vector<uint8_t> g1b(64 * 5), g2b(128 * 4);
  for (int i = 0; i < 5; i++) {
    DecodeJob j{g1off[i], 64, (uint32_t)i, NONE, NONE};
    if (!job_decode(j, raw.data(), g1.data(), nullptr)) {
      snprintf(err, errlen, "bad G1 in PP");
      delete c;
      return nullptr;
    }
    g1_to_bytes(&g1b[64 * i], g1_load(g1[i]));
  }
  for (int k = 0; k < 4; k++)
    if (!decode_g2(&raw[g2off[k]], 128, g2[k], &g2b[128 * k])) {
      snprintf(err, errlen, "bad G2 in PP");
      delete c;
      return nullptr;
    }
  c->const_bytes.assign(C_SIZE, 0);
  memcpy(&c->const_bytes[C_PEDGEN], &g1b[0], 64);
  memcpy(&c->const_bytes[C_PED0], &g1b[64], 192);
  memcpy(&c->const_bytes[C_Q_PK], &g2b[384], 128);
  memcpy(&c->const_bytes[C_Q_PK + 128], &g2b[0], 384);
  memcpy(&c->const_bytes[C_PK_Q + 384], &g2b[384], 128);
  std::vector<G1Dev> hb(5);
  hb[G1B_PED0] = g1[1];
  hb[G1B_PED1] = g1[2];
  hb[G1B_PED2] = g1[3];
  hb[G1B_PEDGEN] = g1[0];
  hb[G1B_GEN] = g1[4];
  uint32_t n1 = G1B_COUNT * G1TAB_WINDOWS * G1TAB_DIGITS, n2 = G2B_COUNT * G2TAB_WINDOWS * G2TAB_DIGITS;
  c->g1tab.resize(n1);
  c->g2tab.resize(n2);
  par_for(n1, [&](uint32_t i) { job_tab_g1(i, hb.data(), c->g1tab.data()); });
  par_for(n2, [&](uint32_t i) { job_tab_g2(i, g2.data(), c->g2tab.data()); });
  c->qlines.resize(MILLER_LINES);
  precompute_lines(c->qlines.data(), g2_load(g2[3]));
  c->pklines.resize(2 * MILLER_LINES);
  precompute_lines(c->pklines.data(), g2_load(g2[G2B_PK1]));
  precompute_lines(c->pklines.data() + MILLER_LINES, g2_load(g2[G2B_PK2]));
  return c;
}

void emu_ctx_destroy(void* c) { delete (EmuCtx*)c; }

// The prover's fixed-base tables of the PP signature points (runtime.hip
// ensure_prover_tables): the same entries |d| 2^(C w) B, built per (base,
// window) by successive additions and one batch inversion (the per-entry
// scalar multiplication of job_tab_g1 is too slow for 2 b bases on the host)
static void emu_ensure_sig_tables(EmuCtx* c) {
  std::lock_guard<std::mutex> lk(c->sig_mu);
  if (c->sig_ready || !pp_sig_tables(c->pp)) return;
  const uint32_t nsig = 2 * c->pp.base;
  const size_t per = (size_t)G1TAB_WINDOWS * G1TAB_DIGITS, old = (size_t)G1B_COUNT * per;
  std::vector<G1Dev> sig(nsig);
  for (uint32_t k = 0; k < nsig; k++) {
    std::vector<uint8_t> raw = (k & 1) ? c->pp.sig_s[k / 2] : c->pp.sig_r[k / 2];
    raw.resize(std::max<size_t>(raw.size(), 64) + 64, 0);
    DecodeJob j{0, 64, k, NONE, NONE};
    (void)job_decode(j, raw.data(), sig.data(), nullptr);
  }
  c->g1tab.resize(old + nsig * per);
  par_for(nsig * G1TAB_WINDOWS, [&](uint32_t t) {
    const uint32_t b = t / G1TAB_WINDOWS, w = t % G1TAB_WINDOWS;
    g1j acc = jac_from_aff(g1_load(sig[b]));
    for (uint32_t q = 0; q < (uint32_t)G1TAB_C * w; q++) acc = jac_dbl(acc);
    const g1a Bw = jac_to_aff(acc);
    std::vector<g1j> e(G1TAB_DIGITS);
    std::vector<fp> pre(G1TAB_DIGITS);
    e[0] = jac_from_aff(Bw);
    for (int d = 1; d < G1TAB_DIGITS; d++) e[d] = jac_add_aff(e[d - 1], Bw);
    pre[0] = e[0].z;
    for (int d = 1; d < G1TAB_DIGITS; d++) pre[d] = pre[d - 1] * e[d].z;
    fp inv = fp_inv(pre[G1TAB_DIGITS - 1]);
    for (int d = G1TAB_DIGITS - 1; d >= 0; d--) {
      fp zi = d ? inv * pre[d - 1] : inv;
      if (d) inv = inv * e[d].z;
      fp zi2 = sqr(zi);
      g1a a;
      a.x = e[d].x * zi2;
      a.y = e[d].y * zi2 * zi;
      a.inf = false;
      G1Dev o;
      g1_store(o, a);
      c->g1tab[old + (size_t)b * per + (size_t)w * G1TAB_DIGITS + d] = o;
    }
  });
  c->sig_ready = true;
}
void emu_ctx_set_fexp(void* c, int variant) { ((EmuCtx*)c)->fexp = variant; }
void emu_set_threads(int t) { g_threads = t > 0 ? (unsigned)t : 0; }

static void run_plan(EmuCtx* c, Plan& p, size_t n, int32_t* codes, std::vector<uint32_t>* scal_out = nullptr) {
  memcpy(p.arena.data(), c->const_bytes.data(), C_SIZE);
  std::vector<uint8_t> wire = p.wire;
  wire.resize(wire.size() + 64, 0);
  std::vector<G1Dev> pts(std::max<uint32_t>(p.n_pts, 1));
  std::vector<uint8_t> pt_ok(std::max<uint32_t>(p.n_pts, 1), 1);
  std::vector<uint32_t> scalv(8 * (size_t)std::max<uint32_t>(p.n_scal, 1));
  uint32_t(*scal)[8] = reinterpret_cast<uint32_t(*)[8]>(scalv.data());
  std::vector<uint8_t> canon(std::max<uint32_t>(p.n_scal, 1));
  std::vector<G1Dev> g1out(std::max<uint32_t>(p.n_g1out, 1));
  std::vector<G2Dev> g2out(std::max<uint32_t>(p.n_g2out, 1));
  std::vector<F12Dev> fbuf(std::max<size_t>(p.pr.size(), 1));
  std::vector<uint8_t> hok(std::max<size_t>(p.hmain.size(), 1)), hpok(std::max<size_t>(p.hpre.size(), 1));
  // same order as ftz_batch_run
  par_for((uint32_t)p.dec.size(), [&](uint32_t i) { pt_ok[p.dec[i].out] = job_decode(p.dec[i], wire.data(), pts.data(), p.arena.data()); });
  par_for((uint32_t)p.zr.size(), [&](uint32_t i) { job_zr(p.zr[i], wire.data(), scal, canon.data()); });
  par_for((uint32_t)p.hpre.size(), [&](uint32_t i) { hpok[i] = job_hash(p.hpre[i], p.seg.data(), p.arena.data(), scal, canon.data()); });
  par_for((uint32_t)p.sc.size(), [&](uint32_t i) { job_scalar(p.sc[i], scal, p.sclist.data()); });
  // side G1 jobs through the device's split path (parts + combine), pairing G1 jobs whole (job_g1)
  {
    uint32_t n1 = (uint32_t)p.g1.size();
    std::vector<G1JDev> part(4 * (size_t)std::max<uint32_t>(n1, 1));
    std::vector<G1Dev> vtab(16 * (size_t)std::max<uint32_t>(n1, 1));  // the device's strided table layout
    par_for(4 * n1, [&](uint32_t i) {
      job_g1_part(p.g1.data(), n1, i, p.vt.data(), pts.data(), scal, c->g1tab.data(), part.data(), vtab.data());
    });
    par_for(n1, [&](uint32_t i) { job_g1_combine(p.g1[i], i, n1, part.data(), g1out.data(), p.arena.data()); });
  }
  par_for((uint32_t)p.g1p.size(), [&](uint32_t i) {
    job_g1(p.g1p[i], p.vt.data(), pts.data(), scal, c->g1tab.data(), g1out.data(), p.arena.data());
  });
  par_for((uint32_t)p.g2.size(), [&](uint32_t i) { job_g2(p.g2[i], scal, c->g2tab.data(), g2out.data()); });
  par_for((uint32_t)p.pr.size(), [&](uint32_t i) {
    job_miller(p.pr[i], c->qlines.data(), g1out.data(), pts.data(), g2out.data(), fbuf.data(), i);
  });
  par_for((uint32_t)p.pr.size(), [&](uint32_t i) { job_fexp(p.pr[i], fbuf.data(), i, p.arena.data(), c->fexp); });
  par_for((uint32_t)p.hmain.size(), [&](uint32_t i) { hok[i] = job_hash(p.hmain[i], p.seg.data(), p.arena.data(), scal, canon.data()); });
  for (size_t i = 0; i < n; i++) codes[i] = job_verdict(p.tx[i], p.ck.data(), pt_ok.data(), hok.data());
  if (scal_out) scal_out->swap(scalv);
}

#ifdef FTS_COUNT_OPS
// Montgomery products per pipeline stage (decode, zr, hash_pre, scalar, g1,
// g2, miller, fexp, hash, verdict) for a batch, single-threaded.
int emu_opcount_transfers(void* ctx, size_t n, const ftz_transfer* tx, unsigned long long* per_stage,
                          unsigned long long* jobs) {
  EmuCtx* c = (EmuCtx*)ctx;
  std::vector<TransferIn> t(n);
  for (size_t i = 0; i < n; i++)
    t[i] = {tx[i].inputs, tx[i].n_in, tx[i].outputs, tx[i].n_out, tx[i].proof, tx[i].proof_len};
  Plan p;
  plan_transfers(c->pp, n, t.data(), p, 1);
  memcpy(p.arena.data(), c->const_bytes.data(), C_SIZE);
  std::vector<uint8_t> wire = p.wire;
  wire.resize(wire.size() + 64, 0);
  std::vector<G1Dev> pts(std::max<uint32_t>(p.n_pts, 1));
  std::vector<uint8_t> pt_ok(std::max<uint32_t>(p.n_pts, 1), 1);
  std::vector<uint32_t> scalv(8 * (size_t)std::max<uint32_t>(p.n_scal, 1));
  uint32_t(*scal)[8] = reinterpret_cast<uint32_t(*)[8]>(scalv.data());
  std::vector<uint8_t> canon(std::max<uint32_t>(p.n_scal, 1));
  std::vector<G1Dev> g1out(std::max<uint32_t>(p.n_g1out, 1));
  std::vector<G2Dev> g2out(std::max<uint32_t>(p.n_g2out, 1));
  std::vector<F12Dev> fbuf(std::max<size_t>(p.pr.size(), 1));
  std::vector<uint8_t> hok(std::max<size_t>(p.hmain.size(), 1));
  auto stage = [&](int k, size_t nj, auto fn) {
    unsigned long long c0 = fts_mont_count;
    for (size_t i = 0; i < nj; i++) fn(i);
    per_stage[k] = fts_mont_count - c0;
    jobs[k] = nj;
  };
  stage(0, p.dec.size(), [&](size_t i) { pt_ok[p.dec[i].out] = job_decode(p.dec[i], wire.data(), pts.data(), p.arena.data()); });
  stage(1, p.zr.size(), [&](size_t i) { job_zr(p.zr[i], wire.data(), scal, canon.data()); });
  stage(2, p.hpre.size(), [&](size_t i) { job_hash(p.hpre[i], p.seg.data(), p.arena.data(), scal, canon.data()); });
  stage(3, p.sc.size(), [&](size_t i) { job_scalar(p.sc[i], scal, p.sclist.data()); });
  std::vector<G1Job> all = p.g1;
  all.insert(all.end(), p.g1p.begin(), p.g1p.end());
  stage(4, all.size(), [&](size_t i) { job_g1(all[i], p.vt.data(), pts.data(), scal, c->g1tab.data(), g1out.data(), p.arena.data()); });
  stage(5, p.g2.size(), [&](size_t i) { job_g2(p.g2[i], scal, c->g2tab.data(), g2out.data()); });
  stage(6, p.pr.size(), [&](size_t i) { job_miller(p.pr[i], c->qlines.data(), g1out.data(), pts.data(), g2out.data(), fbuf.data(), (uint32_t)i); });
  stage(7, p.pr.size(), [&](size_t i) { job_fexp(p.pr[i], fbuf.data(), (uint32_t)i, p.arena.data(), c->fexp); });
  stage(8, p.hmain.size(), [&](size_t i) { hok[i] = job_hash(p.hmain[i], p.seg.data(), p.arena.data(), scal, canon.data()); });
  per_stage[9] = 0;
  jobs[9] = n;
  // stage 10: the device's k_g2lines split (t' by fixed-base tables + the 88
  // pair-2 Miller lines evaluated at R), g2[i] paired with pr[i] as the kernel does
  std::vector<G2Dev> g2o2(std::max<uint32_t>(p.n_g2out, 1));
  std::vector<EvLineDev> lines(88 * std::max<size_t>(p.g2.size(), 1));
  stage(10, p.g2.size(), [&](size_t i) {
    job_g2lines(p.g2[i], p.pr[i], scal, c->g2tab.data(), g2o2.data(), pts.data(), lines.data(), (uint32_t)i,
                (uint32_t)p.g2.size());
  });
  return 0;
}
#endif

// prover plan (host/planner_prove.cpp) in the order of ftz_prover_run
static long run_prove_plan(EmuCtx* c, Plan& p, size_t n, uint8_t* buf, size_t cap, size_t* offsets,
                           int32_t* codes) {
  memcpy(p.arena.data(), c->const_bytes.data(), C_SIZE);
  std::vector<uint8_t> wire = p.wire;
  wire.resize(wire.size() + 64, 0);
  // device-initialised pools (k_copy): shape images, then the witness bytes
  for (const auto* cps : {&p.cp, &p.cp2})
    for (const CopyJob& j : *cps)
      for (uint32_t b = 0; b < j.len; b++) job_copy_byte(j, b, wire.data(), p.arena.data(), p.out.data());
  std::vector<G1Dev> pts(std::max<uint32_t>(p.n_pts, 1));
  std::vector<uint8_t> pt_ok(std::max<uint32_t>(p.n_pts, 1), 1);
  std::vector<uint32_t> scalv(8 * (size_t)std::max<uint32_t>(p.n_scal, 1));
  uint32_t(*scal)[8] = reinterpret_cast<uint32_t(*)[8]>(scalv.data());
  std::vector<uint8_t> canon(std::max<uint32_t>(p.n_scal, 1));
  std::vector<G1Dev> g1out(std::max<uint32_t>(p.n_g1out, 1));
  std::vector<G2Dev> g2out(std::max<uint32_t>(p.n_g2out, 1));
  std::vector<F12Dev> fbuf(std::max<size_t>(p.pr.size(), 1));
  std::vector<uint8_t> hok(std::max<size_t>(p.hmain.size(), 1));
  par_for((uint32_t)p.dec.size(), [&](uint32_t i) { pt_ok[p.dec[i].out] = job_decode(p.dec[i], wire.data(), pts.data(), p.arena.data()); });
  par_for((uint32_t)p.zr.size(), [&](uint32_t i) { job_zr(p.zr[i], wire.data(), scal, canon.data()); });
  par_for((uint32_t)p.rnd.size(), [&](uint32_t i) { job_rand(p.rnd[i], p.arena.data(), scal); });
  par_for((uint32_t)p.hpre.size(), [&](uint32_t i) { job_hash(p.hpre[i], p.seg.data(), p.arena.data(), scal, canon.data()); });
  // one parallel pass per level, as the device runs them
  par_for((uint32_t)p.sc.size(), [&](uint32_t i) { job_scalar(p.sc[i], scal, p.sclist.data()); });
  par_for((uint32_t)p.sc1.size(), [&](uint32_t i) { job_scalar(p.sc1[i], scal, p.sclist.data()); });
  par_for((uint32_t)p.g1p.size(), [&](uint32_t i) {
    job_g1(p.g1p[i], p.vt.data(), pts.data(), scal, c->g1tab.data(), g1out.data(), p.arena.data());
  });
  {
    uint32_t n1 = (uint32_t)p.g1.size();
    std::vector<G1JDev> part(4 * (size_t)std::max<uint32_t>(n1, 1));
    par_for(4 * n1, [&](uint32_t i) {
      job_g1_part(p.g1.data(), n1, i, p.vt.data(), pts.data(), scal, c->g1tab.data(), part.data(), nullptr);
    });
    par_for(n1, [&](uint32_t i) { job_g1_combine(p.g1[i], i, n1, part.data(), g1out.data(), p.arena.data()); });
  }
  par_for((uint32_t)p.g2.size(), [&](uint32_t i) { job_g2(p.g2[i], scal, c->g2tab.data(), g2out.data()); });
  // pair 2 of a prover pairing job is R' = rr R (a G1 job output)
  par_for((uint32_t)p.pr.size(), [&](uint32_t i) {
    if (p.pr[i].p3 != NONE)  // fixed pairs (k_miller_f3 on the device)
      job_miller3(p.pr[i], c->qlines.data(), c->pklines.data(), c->pklines.data() + MILLER_LINES, g1out.data(),
                  fbuf.data(), i);
    else
      job_miller(p.pr[i], c->qlines.data(), g1out.data(), g1out.data(), g2out.data(), fbuf.data(), i);
  });
  par_for((uint32_t)p.pr.size(), [&](uint32_t i) { job_fexp(p.pr[i], fbuf.data(), i, p.arena.data(), c->fexp); });
  par_for((uint32_t)p.hmain.size(), [&](uint32_t i) { hok[i] = job_hash(p.hmain[i], p.seg.data(), p.arena.data(), scal, canon.data()); });
  par_for((uint32_t)p.sc_post.size(), [&](uint32_t i) { job_scalar(p.sc_post[i], scal, p.sclist.data()); });
  par_for((uint32_t)p.emit.size(), [&](uint32_t i) { job_emit(p.emit[i], scal, p.arena.data()); });
  std::vector<uint8_t> out = p.out;
  for (const B64Job& j : p.b64) b64_encode(out.data() + j.dst, p.arena.data() + j.src, j.len);
  for (size_t i = 0; i < n; i++) codes[i] = job_verdict(p.tx[i], p.ck.data(), pt_ok.data(), hok.data());
  if (out.size() > cap) return -(long)out.size();
  memcpy(buf, out.data(), out.size());
  for (size_t i = 0; i < n; i++) offsets[i] = p.out_off[i];
  offsets[n] = out.size();
  return (long)out.size();
}

long emu_prove_transfers(void* ctx, size_t n, const ftz_transfer_witness* w, uint8_t* buf, size_t cap,
                         size_t* offsets, int32_t* codes, char* err, size_t errlen) {
  EmuCtx* c = (EmuCtx*)ctx;
  emu_ensure_sig_tables(c);
  std::vector<TransferWit> t(n);
  for (size_t i = 0; i < n; i++)
    t[i] = {w[i].inputs, w[i].n_in, w[i].outputs, w[i].n_out, w[i].in_values, w[i].in_bfs,
            w[i].out_values, w[i].out_bfs, w[i].type, w[i].type_len, w[i].seed};
  Plan p;
  std::string e = plan_prove_transfers(c->pp, n, t.data(), p, 4);
  if (!e.empty()) {
    snprintf(err, errlen, "%s", e.c_str());
    return -1;
  }
  return run_prove_plan(c, p, n, buf, cap, offsets, codes);
}

// TEST-ONLY diagnostic: host time of one prover pass's planning as the device
// path runs it (plan_prove_items_transfers on a pool of `threads`, then the
// flattening into one blob), median of `reps`: out_ms[0] items, [1] layout +
// write, [2] blob bytes, [3] bytes uploaded (fp.upload), [4 + s] elements of
// section s (PlanSec order).
int emu_plan_prove_ms(void* ctx, size_t n, const ftz_transfer_witness* w, int threads, int reps, double* out_ms) {
  EmuCtx* c = (EmuCtx*)ctx;
  std::vector<TransferWit> t(n);
  for (size_t i = 0; i < n; i++)
    t[i] = {w[i].inputs, w[i].n_in, w[i].outputs, w[i].n_out, w[i].in_values, w[i].in_bfs,
            w[i].out_values, w[i].out_bfs, w[i].type, w[i].type_len, w[i].seed};
  WorkPool pool(threads);
  PlanWork work;
  FlatPlan fp;
  std::vector<uint8_t> blob;
  std::vector<double> a, b;
  using Clk = std::chrono::steady_clock;
  for (int r = 0; r < reps; r++) {
    auto t0 = Clk::now();
    std::string e = plan_prove_items_transfers(c->pp, n, t.data(), work, pool);
    if (!e.empty()) return -1;
    auto t1 = Clk::now();
    e = flat_layout(work, true, fp);
    if (!e.empty()) return -2;
    if (blob.size() < fp.bytes) blob.resize(fp.bytes);
    flat_write(work, fp, blob.data(), c->const_bytes.data(), pool);
    auto t2 = Clk::now();
    a.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
    b.push_back(std::chrono::duration<double, std::milli>(t2 - t1).count());
  }
  std::sort(a.begin(), a.end());
  std::sort(b.begin(), b.end());
  out_ms[0] = a[a.size() / 2];
  out_ms[1] = b[b.size() / 2];
  out_ms[2] = (double)fp.bytes;
  out_ms[3] = (double)fp.upload;
  for (int k = 0; k < PS_COUNT; k++) out_ms[4 + k] = (double)fp.cnt[k];
  return 0;
}

// TEST-ONLY diagnostic: host time of one verifier pass's planning as the
// engine runs it (plan_items on a pool of `threads`, then flat_layout +
// flat_write into one blob), median of `reps`: out_ms[0] items, [1] layout +
// write, [2] blob bytes, [3] bytes uploaded, [4 + s] bytes of section s.
int emu_plan_verify_ms(void* ctx, size_t n, const ftz_transfer* tx, int threads, int reps, double* out_ms) {
  EmuCtx* c = (EmuCtx*)ctx;
  std::vector<PlanItem> items(n);
  for (size_t i = 0; i < n; i++) {
    memset(&items[i], 0, sizeof(PlanItem));
    items[i].kind = 0;
    items[i].t = {tx[i].inputs, tx[i].n_in, tx[i].outputs, tx[i].n_out, tx[i].proof, tx[i].proof_len};
  }
  WorkPool pool(threads);
  PlanWork work;
  FlatPlan fp;
  std::vector<uint8_t> blob;
  std::vector<double> a, b;
  using Clk = std::chrono::steady_clock;
  for (int r = 0; r < reps; r++) {
    auto t0 = Clk::now();
    plan_items(c->pp, n, items.data(), work, pool);
    auto t1 = Clk::now();
    std::string e = flat_layout(work, false, fp);
    if (!e.empty()) return -2;
    if (blob.size() < fp.bytes) blob.resize(fp.bytes);
    flat_write(work, fp, blob.data(), c->const_bytes.data(), pool);
    auto t2 = Clk::now();
    a.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
    b.push_back(std::chrono::duration<double, std::milli>(t2 - t1).count());
  }
  std::sort(a.begin(), a.end());
  std::sort(b.begin(), b.end());
  out_ms[0] = a[a.size() / 2];
  out_ms[1] = b[b.size() / 2];
  out_ms[2] = (double)fp.bytes;
  out_ms[3] = (double)fp.upload;
  for (int k = 0; k < PS_COUNT; k++)
    out_ms[4 + k] = (double)((k + 1 < PS_COUNT ? fp.off[k + 1] : fp.bytes) - fp.off[k]);
  return 0;
}

long emu_prove_issues(void* ctx, size_t n, const ftz_issue_witness* w, uint8_t* buf, size_t cap, size_t* offsets,
                      int32_t* codes, char* err, size_t errlen) {
  EmuCtx* c = (EmuCtx*)ctx;
  emu_ensure_sig_tables(c);
  std::vector<IssueWit> t(n);
  for (size_t i = 0; i < n; i++)
    t[i] = {w[i].outputs, w[i].n_out, w[i].values, w[i].bfs, w[i].type, w[i].type_len, w[i].anonymous, w[i].seed};
  Plan p;
  std::string e = plan_prove_issues(c->pp, n, t.data(), p, 4);
  if (!e.empty()) {
    snprintf(err, errlen, "%s", e.c_str());
    return -1;
  }
  return run_prove_plan(c, p, n, buf, cap, offsets, codes);
}

// token commitments / auditor opening checks (ftz_commit_tokens / ftz_audit_openings)
int emu_openings(void* ctx, size_t n, const ftz_token_opening* t, const uint8_t* coms, uint8_t* out,
                 int32_t* codes) {
  EmuCtx* c = (EmuCtx*)ctx;
  std::vector<PlanItem> items(n);
  for (size_t i = 0; i < n; i++) {
    memset(&items[i], 0, sizeof(PlanItem));
    items[i].kind = 2;
    items[i].o = {t[i].type, t[i].type_len, t[i].value, t[i].bf, coms ? coms + 64 * i : nullptr};
  }
  Plan p;
  plan_items_merged(c->pp, n, items.data(), p, g_threads ? (int)g_threads : 4);
  std::vector<int32_t> vc(std::max<size_t>(n, 1));
  run_plan(c, p, n, vc.data());
  for (size_t i = 0; i < n; i++) {
    const uint8_t* r = p.arena.data() + p.item_off[i];
    if (out) memcpy(out + 64 * i, r, 64);
    if (codes) codes[i] = vc[i] != E_OK ? vc[i] : (!coms || memcmp(r, r + 64, 64) == 0 ? 0 : 7);
  }
  return 0;
}

int emu_verify_transfers(void* ctx, size_t n, const ftz_transfer* tx, int32_t* codes) {
  EmuCtx* c = (EmuCtx*)ctx;
  std::vector<TransferIn> t(n);
  for (size_t i = 0; i < n; i++)
    t[i] = {tx[i].inputs, tx[i].n_in, tx[i].outputs, tx[i].n_out, tx[i].proof, tx[i].proof_len};
  Plan p;
  plan_transfers(c->pp, n, t.data(), p, g_threads ? (int)g_threads : 4);
  run_plan(c, p, n, codes);
  return 0;
}

// The recomputed challenges of every proof (ftz_batch_challenges on the host):
// transfers (kind 0) or issues (kind 1) planned with debug_challenges; proof i's
// at kinds / values + 32 * (i * cap), counts[i] of them.
int emu_challenges(void* ctx, int kind, size_t n, const void* items, int32_t* codes, int32_t* kinds,
                   uint8_t* values, size_t cap, size_t* counts) {
  EmuCtx* c = (EmuCtx*)ctx;
  PPInfo pp = c->pp;
  pp.debug_challenges = true;
  Plan p;
  if (kind == 0) {
    const ftz_transfer* tx = static_cast<const ftz_transfer*>(items);
    std::vector<TransferIn> t(n);
    for (size_t i = 0; i < n; i++)
      t[i] = {tx[i].inputs, tx[i].n_in, tx[i].outputs, tx[i].n_out, tx[i].proof, tx[i].proof_len};
    plan_transfers(pp, n, t.data(), p, g_threads ? (int)g_threads : 4);
  } else {
    const ftz_issue* is = static_cast<const ftz_issue*>(items);
    std::vector<IssueIn> t(n);
    for (size_t i = 0; i < n; i++) t[i] = {is[i].outputs, is[i].n_out, is[i].proof, is[i].proof_len, is[i].anonymous};
    plan_issues(pp, n, t.data(), p, g_threads ? (int)g_threads : 4);
  }
  std::vector<uint32_t> scal;
  run_plan(c, p, n, codes, &scal);
  std::vector<uint32_t> slot(cap);
  for (size_t i = 0; i < n; i++) {
    counts[i] = proof_challenge_slots(p.tx[i], p.ck.data(), p.hmain.data(), kinds + i * cap, slot.data(), cap);
    for (size_t k = 0; k < std::min(counts[i], cap); k++) limbs_to_be32(values + 32 * (i * cap + k), &scal[8 * (size_t)slot[k]]);
  }
  return 0;
}

int emu_verify_issues(void* ctx, size_t n, const ftz_issue* is, int32_t* codes) {
  EmuCtx* c = (EmuCtx*)ctx;
  std::vector<IssueIn> t(n);
  for (size_t i = 0; i < n; i++) t[i] = {is[i].outputs, is[i].n_out, is[i].proof, is[i].proof_len, is[i].anonymous};
  Plan p;
  plan_issues(c->pp, n, t.data(), p, g_threads ? (int)g_threads : 4);
  run_plan(c, p, n, codes);
  return 0;
}

// host run of the raw token-request path (host/request.cpp) with the same
// orchestration as ftz_verify_token_requests
int emu_verify_token_requests(void* ctx, size_t n, const ftz_bytes* reqs, ftz_get_state_fn get_state, void* user,
                              int32_t* codes, int32_t* failed) {
  ftsh::RequestHooks h;
  h.check = [](size_t m, const uint8_t* slots, uint8_t* ok) {
    for (size_t i = 0; i < m; i++) {
      g1a a;
      ok[i] = g1_setbytes(slots + 64 * i, 64, a) ? 1 : 0;
    }
    return 0;
  };
  h.verify_transfers = [ctx](size_t m, const ftz_transfer* tx, int32_t* c) { return emu_verify_transfers(ctx, m, tx, c); };
  h.verify_issues = [ctx](size_t m, const ftz_issue* is, int32_t* c) { return emu_verify_issues(ctx, m, is, c); };
  h.get_state = get_state;
  h.user = user;
  std::string err;
  return ftsh::verify_token_requests(n, reqs, h, codes, failed, err);
}

// host-side throughput of the request pipeline alone (tools, not a test of
// verdicts): element checks and ZK verification answered "ok" at once, the
// decoding / lookup / token / build stages real.  stats[6] = RequestStats (ms).
int emu_request_host_bench(size_t n, const ftz_bytes* reqs, ftz_get_states_fn get_states, void* user, size_t chunk,
                           int par_threads, int32_t* codes, double* stats) {
  ftsh::RequestHooks h;
  h.check = [](size_t m, const uint8_t*, uint8_t* ok) {
    memset(ok, 1, m);
    return 0;
  };
  h.verify_transfers = [](size_t m, const ftz_transfer*, int32_t* c) {
    memset(c, 0, m * sizeof(int32_t));
    return 0;
  };
  h.verify_issues = [](size_t m, const ftz_issue*, int32_t* c) {
    memset(c, 0, m * sizeof(int32_t));
    return 0;
  };
  h.get_states = get_states;
  h.user = user;
  h.chunk = chunk;
  std::unique_ptr<WorkPool> pool;
  if (par_threads > 0) {
    pool.reset(new WorkPool(par_threads));
    WorkPool* pp = pool.get();
    h.par = [pp](size_t k, const std::function<void(size_t)>& f) { pp->run(k, f); };
  }
  ftsh::RequestStats st;
  h.stats = &st;
  std::string err;
  int rc = ftsh::verify_token_requests(n, reqs, h, codes, nullptr, err);
  double v[6] = {st.decode, st.check, st.lookup, st.tokens, st.build, st.drain};
  memcpy(stats, v, sizeof v);
  return rc;
}

// the same with the pipeline's knobs: batched lookups, chunk size, chunks in
// flight, and `par_threads` decoding threads (0: serial)
int emu_verify_token_requests_ex(void* ctx, size_t n, const ftz_bytes* reqs, ftz_get_state_fn get_state,
                                 ftz_get_states_fn get_states, void* user, size_t chunk, size_t inflight,
                                 int par_threads, int32_t* codes, int32_t* failed) {
  ftsh::RequestHooks h;
  h.check = [](size_t m, const uint8_t* slots, uint8_t* ok) {
    for (size_t i = 0; i < m; i++) {
      g1a a;
      ok[i] = g1_setbytes(slots + 64 * i, 64, a) ? 1 : 0;
    }
    return 0;
  };
  h.verify_transfers = [ctx](size_t m, const ftz_transfer* tx, int32_t* c) { return emu_verify_transfers(ctx, m, tx, c); };
  h.verify_issues = [ctx](size_t m, const ftz_issue* is, int32_t* c) { return emu_verify_issues(ctx, m, is, c); };
  h.get_state = get_state;
  h.get_states = get_states;
  h.user = user;
  h.chunk = chunk;
  h.inflight = inflight;
  std::unique_ptr<WorkPool> pool;
  if (par_threads > 0) {
    pool.reset(new WorkPool(par_threads));
    WorkPool* pp = pool.get();
    h.par = [pp](size_t k, const std::function<void(size_t)>& f) { pp->run(k, f); };
  }
  std::string err;
  return ftsh::verify_token_requests(n, reqs, h, codes, failed, err);
}
}

// ------------------------------------------------------------------ fp29 check
// dev/fp29.h (carry-free 29-bit limbs) against the fp.h arithmetic: field
// products / sums at the bounds the G1 formulas use, and long double-and-add
// chains of j29_dbl / j29_madd against jac_dbl / jac_add_aff including the
// exceptional additions (from infinity, P + P, P + (-P)).  Returns the number
// of mismatches.
namespace {
struct Rng64 {
  uint64_t s;
  uint64_t next() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  }
};
fp rand_fp(Rng64& r) {
  uint32_t v[8];
  for (int i = 0; i < 8; i++) v[i] = (uint32_t)r.next();
  v[7] &= 0x1fffffffu;  // < 2^253 < p
  return fe_from_int<ModP>(v);
}
bool aff_same(const g1a& a, const g1a& b) {
  if (a.inf || b.inf) return a.inf == b.inf;
  return fe_eq(a.x, b.x) && fe_eq(a.y, b.y);
}
}  // namespace

extern "C" int emu_f29_check(uint64_t seed, int iters) {
  Rng64 r{seed | 1};
  int bad = 0;
  fp pm1 = fe_zero<ModP>() - fe_one<ModP>();
  for (int it = 0; it < iters; it++) {
    fp a = it == 0 ? pm1 : rand_fp(r), b = it < 2 ? pm1 : rand_fp(r);
    f29 A = f29_from_fp(a), B = f29_from_fp(b);
    if (!fe_eq(f29_to_fp(A), a)) bad++;
    f29 Ar = f29_reduce(A), Br = f29_reduce(B);
    if (!fe_eq(f29_to_fp(f29_mul(Ar, Br)), a * b)) bad++;
    if (!fe_eq(f29_to_fp(f29_sqr(Ar)), fe_sqr(a))) bad++;
    // unreduced entry form (B 32) times a product (B 2), and a 4-term sum
    f29 Pab = f29_mul(Ar, Br);
    if (!fe_eq(f29_to_fp(f29_mul(A, Pab)), a * (a * b))) bad++;
    f29 s = f29_norm(f29_sub(f29_add(f29_add(Pab, Pab), Ar), Br));
    fp sf = a * b + a * b + a - b;
    if (!fe_eq(f29_to_fp(s), sf)) bad++;
    if (!fe_eq(f29_to_fp(f29_neg(Ar)), fe_neg(a))) bad++;
  }
  // point chains: a few random affine base points
  g1a gen = {fe_one<ModP>(), fe_one<ModP>() + fe_one<ModP>(), false};
  std::vector<g1a> pts;
  for (int k = 0; k < 8; k++) {
    uint32_t sc[8];
    for (int i = 0; i < 8; i++) sc[i] = (uint32_t)r.next();
    sc[7] &= 0x0fffffffu;
    pts.push_back(jac_to_aff(aff_mul(gen, sc)));
  }
  for (int chain = 0; chain < iters / 8 + 1; chain++) {
    g1j acc = jac_inf<fp>();
    j29 a29 = j29_from(acc);
    for (int step = 0; step < 40; step++) {
      int kind = (int)(r.next() % 8);
      if (step > 0 && kind < 3) {
        int nd = 1 + (int)(r.next() % 4);
        for (int d = 0; d < nd; d++) {
          acc = jac_dbl(acc);
          a29 = j29_dbl(a29);
        }
      }
      g1a q = pts[r.next() % pts.size()];
      int e = (int)(r.next() % 16);
      if (e == 0) q = jac_to_aff(acc);                   // P + P
      if (e == 1) q = aff_neg(jac_to_aff(acc));          // P + (-P)
      if (q.inf) continue;
      bool neg = r.next() & 1;
      f29 Y = f29_from_fp(q.y);
      a29 = j29_madd(a29, f29_from_fp(q.x), neg ? f29_neg(Y) : Y);
      acc = jac_add_aff(acc, neg ? aff_neg(q) : q);
      if (!aff_same(jac_to_aff(j29_to(a29)), jac_to_aff(acc))) {
        bad++;
        a29 = j29_from(acc);  // resynchronise
      }
    }
    // round trip through the fp form mid-chain
    if (!aff_same(jac_to_aff(j29_to(j29_from(acc))), jac_to_aff(acc))) bad++;
  }
  // full Jacobian additions (j29_add vs jac_add): random sums, P + P, P + (-P),
  // either side infinity, and chained sums of sums
  for (int it = 0; it < iters / 4 + 4; it++) {
    uint32_t s1[8], s2[8];
    for (int i = 0; i < 8; i++) s1[i] = (uint32_t)r.next(), s2[i] = (uint32_t)r.next();
    s1[7] &= 0x0fffffffu;
    s2[7] &= 0x0fffffffu;
    g1j P = aff_mul(pts[it % pts.size()], s1), Q = aff_mul(pts[(it + 3) % pts.size()], s2);
    int e = it % 6;
    if (e == 1) Q = jac_dbl(jac_add(P, jac_inf<fp>()));            // Q = 2P (other Z)
    if (e == 2) Q = P;                                             // P + P, same Z
    if (e == 3) Q = {P.x, fe_neg(P.y), P.z};                       // P + (-P)
    if (e == 4) P = jac_inf<fp>();
    if (e == 5) Q = jac_inf<fp>();
    j29 A = j29_from(P), B = j29_from(Q);
    j29 S = j29_add(A, B);
    g1j want = jac_add(P, Q);
    if (!aff_same(jac_to_aff(j29_to(S)), jac_to_aff(want))) bad++;
    // a sum of sums (outputs feed inputs: the B <= 2 bound) and a doubling of a sum
    j29 S2 = j29_add(S, j29_add(B, S));
    g1j want2 = jac_add(want, jac_add(Q, want));
    if (!aff_same(jac_to_aff(j29_to(S2)), jac_to_aff(want2))) bad++;
    if (!aff_same(jac_to_aff(j29_to(j29_add(S2, S2))), jac_to_aff(jac_dbl(want2)))) bad++;
  }
  return bad;
}

// Range-proof digit weights and the prover's digits as the product computes
// them (host/planner.cpp digit_weight / prover_digits), for the weight parity
// tests (tests/test_weights.py)
extern "C" int64_t emu_digit_weight(uint32_t base, int64_t i) { return ftsh::digit_weight(base, i); }
extern "C" int emu_prover_digits(const uint8_t* pp_json, size_t pp_len, const uint8_t* be32, uint32_t* digits,
                                 int64_t* weights) {
  ftsh::PPInfo pp;
  if (!ftsh::parse_pp(pp_json, pp_len, "zkatdlog", pp).empty()) return -1;
  for (size_t i = 0; i < pp.pow.size(); i++) weights[i] = (int64_t)pp.pow[i];
  weights[pp.pow.size()] = pp.pow_top;
  return ftsh::prover_digits(pp, be32, digits);
}

// TEST-ONLY host run of the MSM pipeline (dev/msm.h) with the same stage order
// as msm_rt.hip: sort keys -> stable sort -> bucket ranges -> bucket sums -> segment sums ->
// window sums -> Horner.  Small window sizes exercise many windows and the
// signed-digit carries; tests/test_msm.py compares with the Python oracle.
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../fabric-token-sdk_amd/csrc/dev/msm.h"

using namespace fts;

extern "C" int emu_msm_ex(size_t n, const uint8_t* points, const uint8_t* scalars, uint32_t c, uint32_t slot_cap,
                          uint32_t seg_len, uint32_t glv, uint32_t pre, uint8_t out[64]) {
  MsmPlan p = msm_make_plan(n, c, slot_cap, seg_len, glv != 0, pre != 0);
  std::vector<G1Dev> pts(p.pts);
  memset(pts.data(), 0, pts.size() * sizeof(G1Dev));
  std::vector<uint32_t> scal(8 * n);
  uint32_t(*sc)[8] = reinterpret_cast<uint32_t(*)[8]>(scal.data());
  for (size_t i = 0; i < n; i++) {
    uint32_t x[8], y[8], k[8];
    be32_to_limbs(x, points + 64 * i);
    be32_to_limbs(y, points + 64 * i + 32);
    g1a a;
    a.x = fe_from_int<ModP>(x);
    a.y = fe_from_int<ModP>(y);
    a.inf = is_zero(a.x) && is_zero(a.y);
    if (!g1_on_curve(a)) return -1;
    g1_store(pts[i], a);
    be32_to_limbs(k, scalars + 32 * i);
    fe_to_int(sc[i], fe_from_int<ModR>(k));
  }
  if (p.glv)
    for (uint32_t i = 0; i < n; i++) msm_job_phi(p, i, pts.data());
  if (p.pre)
    for (uint32_t v = 0; v < p.nv; v++) msm_job_precompute(p, v, pts.data());
  size_t wb = (size_t)p.rw * p.buckets, wn = (size_t)p.windows * p.nv;
  std::vector<uint32_t> key(wn), val(wn), skey(wn), perm(wn), count(wb), start(wb, 0), end(wb, 0);
  for (uint32_t i = 0; i < n; i++) msm_job_keys(p, i, sc, key.data(), val.data());
  // the device's stable radix sort over msm_key_bits(p) bits
  uint32_t kb = msm_key_bits(p);
  uint32_t kmask = kb >= 32 ? 0xFFFFFFFFu : (1u << kb) - 1;
  std::vector<uint32_t> idx(wn);
  for (size_t t = 0; t < wn; t++) idx[t] = (uint32_t)t;
  std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return (key[a] & kmask) < (key[b] & kmask); });
  for (size_t t = 0; t < wn; t++) skey[t] = key[idx[t]], perm[t] = val[idx[t]];
  for (uint64_t t = 0; t < wn; t++) msm_job_bounds(p, t, wn, skey.data(), perm.data(), start.data(), end.data());
  for (size_t g = 0; g < wb; g++) count[g] = end[g] - start[g];
  std::vector<uint32_t> soff(wb), owner((size_t)p.rw * p.max_slots, 0xFFFFFFFFu), wlo(p.rw), whi(p.rw);
  uint32_t run = 0;
  for (size_t b = 0; b < wb; b++) soff[b] = run, run += msm_bucket_slots(p, count[b]);
  if (run > (size_t)p.rw * p.max_slots) return -2;
  for (uint32_t g = 0; g < wb; g++) msm_job_owner(p, g, count.data(), soff.data(), owner.data(), wlo.data(), whi.data());
  if (whi[p.rw - 1] != run) return -3;
  std::vector<G1JDev> slot_sum(run);
  for (uint32_t j = 0; j < run; j++)
    g1j_store(slot_sum[j], msm_job_slot(p, j, owner.data(), soff.data(), start.data(), count.data(), perm.data(),
                                        pts.data()));
  g1j acc = jac_inf<fp>();
  for (int w = (int)p.rw - 1; w >= 0; w--) {
    for (uint32_t q = 0; q < p.c; q++) acc = jac_dbl(acc);
    g1j ws = jac_inf<fp>();
    for (uint32_t s = 0; s < p.segs; s++)
      ws = jac_add(ws, msm_job_segment(p, (uint32_t)w, s, wlo.data(), whi.data(), owner.data(), slot_sum.data()));
    acc = jac_add(acc, ws);
  }
  g1_to_bytes(out, jac_to_aff(acc));
  return 0;
}

extern "C" int emu_msm(size_t n, const uint8_t* points, const uint8_t* scalars, uint32_t c, uint32_t slot_cap,
                       uint32_t seg_len, uint32_t glv, uint8_t out[64]) {
  return emu_msm_ex(n, points, scalars, c, slot_cap, seg_len, glv, 0, out);
}

// host run of the multi-GPU MSM's final add (dev/msm.h g1_sum_raw)
extern "C" int emu_g1_sum(size_t n, const uint8_t* points, uint8_t out[64]) {
  return g1_sum_raw((uint32_t)n, points, out) == n ? 0 : -1;
}

// ---------------------------------------------------------------- CPU baseline
// bench.py's cpu_msm leg (BASELINE configs[2] on the host): a plain bucket
// Pippenger with the same GLV split and signed c-bit digits as the device plan,
// on `threads` host threads -- one contiguous chunk of points per thread, every
// chunk summed window by window (mixed additions into Jacobian buckets, the
// running-sum reduction, Horner over the windows), the partials added at the
// end.  Built with FTS_HOST64 (4 x 64-bit Montgomery) in oracle/cpu.
#include <thread>

namespace {

g1j msm_chunk(const G1Dev* pts, const G1Dev* phi, const uint32_t (*sc)[8], size_t a, size_t b, uint32_t c) {
  const uint32_t W = (129 + c - 1) / c, B = 1u << (c - 1);
  const size_t m = b - a;
  std::vector<int32_t> dig((size_t)2 * W * m);
  for (size_t i = 0; i < m; i++) {
    uint32_t k1[4], k2[4];
    bool n1, n2;
    glv_split(sc[a + i], k1, n1, k2, n2);
    uint32_t x[8] = {k1[0], k1[1], k1[2], k1[3], 0, 0, 0, 0}, y[8] = {k2[0], k2[1], k2[2], k2[3], 0, 0, 0, 0};
    uint32_t cx = 0, cy = 0;
    for (uint32_t w = 0; w < W; w++) {
      int32_t d1 = msm_digit(x, c, w, cx), d2 = msm_digit(y, c, w, cy);
      dig[(size_t)w * 2 * m + 2 * i] = n1 ? -d1 : d1;
      dig[(size_t)w * 2 * m + 2 * i + 1] = n2 ? -d2 : d2;
    }
  }
  std::vector<g1j> bucket(B);
  g1j acc = jac_inf<fp>();
  for (int w = (int)W - 1; w >= 0; w--) {
    for (uint32_t q = 0; q < c; q++) acc = jac_dbl(acc);
    for (auto& x : bucket) x = jac_inf<fp>();
    const int32_t* d = &dig[(size_t)w * 2 * m];
    for (size_t i = 0; i < m; i++)
      for (int h = 0; h < 2; h++) {
        int32_t v = d[2 * i + h];
        if (!v) continue;
        g1a P = g1_load(h ? phi[a + i] : pts[a + i]);
        uint32_t u = (uint32_t)(v < 0 ? -v : v);
        bucket[u - 1] = jac_add_aff(bucket[u - 1], v < 0 ? aff_neg(P) : P);
      }
    g1j run = jac_inf<fp>(), sum = jac_inf<fp>();
    for (int k = (int)B - 1; k >= 0; k--) {
      run = jac_add(run, bucket[k]);
      sum = jac_add(sum, run);
    }
    acc = jac_add(acc, sum);
  }
  return acc;
}

}  // namespace

// points: n x 64-byte RawBytes, scalars n x 32 bytes big-endian; c = 0: the
// device planner's window for the chunk size
extern "C" int emu_msm_cpu(size_t n, const uint8_t* points, const uint8_t* scalars, int threads, uint32_t c,
                           uint8_t out[64]) {
  if (threads < 1) threads = 1;
  std::vector<G1Dev> pts(n), phi(n);
  std::vector<uint32_t> scal(8 * n);
  uint32_t(*sc)[8] = reinterpret_cast<uint32_t(*)[8]>(scal.data());
  auto par = [&](auto&& body) {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) th.emplace_back([&, t]() { body((size_t)t); });
    for (auto& x : th) x.join();
  };
  std::vector<int> bad((size_t)threads, 0);
  par([&](size_t t) {
    for (size_t i = n * t / threads; i < n * (t + 1) / threads; i++) {
      uint32_t x[8], y[8], k[8];
      be32_to_limbs(x, points + 64 * i);
      be32_to_limbs(y, points + 64 * i + 32);
      g1a P;
      P.x = fe_from_int<ModP>(x);
      P.y = fe_from_int<ModP>(y);
      P.inf = is_zero(P.x) && is_zero(P.y);
      if (!g1_on_curve(P)) bad[t] = 1;
      g1_store(pts[i], P);
      if (!P.inf) P.x = P.x * fe_const<ModP>(GLV_BETA);
      g1_store(phi[i], P);
      be32_to_limbs(k, scalars + 32 * i);
      fe_to_int(sc[i], fe_from_int<ModR>(k));
    }
  });
  for (int b : bad)
    if (b) return -1;
  size_t chunk = (n + threads - 1) / threads;
  if (!c) c = msm_window_bits(2 * (uint64_t)chunk);
  std::vector<g1j> part((size_t)threads, jac_inf<fp>());
  par([&](size_t t) {
    size_t a = std::min(n, t * chunk), b = std::min(n, a + chunk);
    if (b > a) part[t] = msm_chunk(pts.data(), phi.data(), sc, a, b, c);
  });
  g1j acc = jac_inf<fp>();
  for (auto& p : part) acc = jac_add(acc, p);
  g1_to_bytes(out, jac_to_aff(acc));
  return 0;
}

// P_i = (offset + i) G for i < n as RawBytes (the bench's known-log points,
// as ftz_msm_load_gen makes them on the device), on `threads` host threads
extern "C" int emu_gen_points(size_t n, uint64_t offset, int threads, uint8_t* out) {
  if (threads < 1) threads = 1;
  std::vector<std::thread> th;
  for (int t = 0; t < threads; t++)
    th.emplace_back([&, t]() {
      size_t a = n * t / threads, b = n * (t + 1) / threads;
      if (b <= a) return;
      g1a G;
      G.x = fe_one<ModP>();
      uint32_t two[8] = {2, 0, 0, 0, 0, 0, 0, 0};
      G.y = fe_from_int<ModP>(two);
      G.inf = false;
      g1j cur = aff_mul_u64(G, offset + a);
      for (size_t i = a; i < b; i++) {
        g1_to_bytes(out + 64 * i, jac_to_aff(cur));
        cur = jac_add_aff(cur, G);
      }
    });
  for (auto& x : th) x.join();
  return 0;
}

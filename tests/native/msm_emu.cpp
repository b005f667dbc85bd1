// TEST-ONLY host run of the MSM pipeline (dev/msm.h) with the same stage order
// as msm_rt.hip: sort keys -> stable sort -> bucket ranges -> bucket sums -> segment sums ->
// window sums -> Horner.  Small window sizes exercise many windows and the
// signed-digit carries; tests/test_msm.py compares with the Python oracle.
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../fabric-token-sdk_amd/csrc/dev/msm.h"

using namespace fts;

extern "C" int emu_msm(size_t n, const uint8_t* points, const uint8_t* scalars, uint32_t c, uint32_t slot_cap,
                       uint32_t seg_len, uint32_t glv, uint8_t out[64]) {
  MsmPlan p = msm_make_plan(n, c, slot_cap, seg_len, glv != 0);
  std::vector<G1Dev> pts(p.nv);
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
  size_t wb = (size_t)p.windows * p.buckets, wn = (size_t)p.windows * p.nv;
  std::vector<uint32_t> key(wn), val(wn), skey(wn), perm(wn), count(wb), start(wb, 0), end(wb, 0);
  for (uint32_t i = 0; i < n; i++) msm_job_keys(p, i, sc, key.data(), val.data());
  // the device's stable radix sort over msm_key_bits(p) bits
  uint32_t kb = msm_key_bits(p);
  uint32_t kmask = kb >= 32 ? 0xFFFFFFFFu : (1u << kb) - 1;
  std::vector<uint32_t> idx(wn);
  for (size_t t = 0; t < wn; t++) idx[t] = (uint32_t)t;
  std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return (key[a] & kmask) < (key[b] & kmask); });
  for (size_t t = 0; t < wn; t++) skey[t] = key[idx[t]], perm[t] = val[idx[t]];
  for (uint64_t t = 0; t < wn; t++) msm_job_bounds(t, wn, skey.data(), start.data(), end.data());
  for (size_t g = 0; g < wb; g++) count[g] = end[g] - start[g];
  std::vector<uint32_t> soff(wb), owner((size_t)p.windows * p.max_slots, 0xFFFFFFFFu), wlo(p.windows), whi(p.windows);
  uint32_t run = 0;
  for (size_t b = 0; b < wb; b++) soff[b] = run, run += msm_bucket_slots(p, count[b]);
  if (run > (size_t)p.windows * p.max_slots) return -2;
  for (uint32_t g = 0; g < wb; g++) msm_job_owner(p, g, count.data(), soff.data(), owner.data(), wlo.data(), whi.data());
  if (whi[p.windows - 1] != run) return -3;
  std::vector<G1JDev> slot_sum(run);
  for (uint32_t j = 0; j < run; j++)
    g1j_store(slot_sum[j], msm_job_slot(p, j, owner.data(), soff.data(), start.data(), count.data(), perm.data(),
                                        pts.data()));
  g1j acc = jac_inf<fp>();
  for (int w = (int)p.windows - 1; w >= 0; w--) {
    for (uint32_t q = 0; q < p.c; q++) acc = jac_dbl(acc);
    g1j ws = jac_inf<fp>();
    for (uint32_t s = 0; s < p.segs; s++)
      ws = jac_add(ws, msm_job_segment(p, (uint32_t)w, s, wlo.data(), whi.data(), owner.data(), slot_sum.data()));
    acc = jac_add(acc, ws);
  }
  g1_to_bytes(out, jac_to_aff(acc));
  return 0;
}

// host run of the multi-GPU MSM's final add (dev/msm.h g1_sum_raw)
extern "C" int emu_g1_sum(size_t n, const uint8_t* points, uint8_t out[64]) {
  return g1_sum_raw((uint32_t)n, points, out) == n ? 0 : -1;
}

// TEST-ONLY host emulation of the sextet pairing code (dev/sextet.h): the six
// lanes of a sextet run as six host threads sharing a slot array, with a
// pthread barrier standing in for the wave's __syncthreads.  Each routine is
// compared with the one-lane tower/pairing code (dev/tower.h, dev/pairing.h),
// which tests/test_emu.py checks against the Python oracle.
#include <pthread.h>
#include <string.h>

#include <functional>
#include <thread>
#include <vector>

#include "../../fabric-token-sdk_amd/csrc/dev/jobs.h"
#include "../../fabric-token-sdk_amd/csrc/dev/sx29.h"
#include "g2l29.h"
#include "../../fabric-token-sdk_amd/csrc/dev/g2lines29.h"

using namespace fts;

namespace {

struct SyncHost {
  pthread_barrier_t* b;
  void operator()() const { pthread_barrier_wait(b); }
};
typedef Sx<SyncHost> SxH;

// run body(x) on six threads (lanes 0..5) sharing one slot region
void run6(const std::function<void(const SxH&)>& body) {
  std::vector<F2Slot> slots(SX_SLOTS_MILLER > SX_SLOTS_FEXP ? SX_SLOTS_MILLER : SX_SLOTS_FEXP);
  memset(slots.data(), 0xA5, slots.size() * sizeof(F2Slot));  // garbage: nothing may read unwritten slots
  pthread_barrier_t b;
  pthread_barrier_init(&b, nullptr, 6);
  std::vector<std::thread> th;
  for (int k = 0; k < 6; k++)
    th.emplace_back([&, k] {
      SxH x{k, slots.data(), true, {&b}};
      body(x);
    });
  for (auto& t : th) t.join();
  pthread_barrier_destroy(&b);
}

typedef Sq<SyncHost> SqH;
void run6q(const std::function<void(const SqH&)>& body) {
  std::vector<Q2Slot> slots(SX_SLOTS_FEXP);
  memset(slots.data(), 0xA5, slots.size() * sizeof(Q2Slot));
  pthread_barrier_t b;
  pthread_barrier_init(&b, nullptr, 6);
  std::vector<std::thread> th;
  for (int k = 0; k < 6; k++)
    th.emplace_back([&, k] {
      SqH x{k, slots.data(), true, {&b}};
      body(x);
    });
  for (auto& t : th) t.join();
  pthread_barrier_destroy(&b);
}

uint32_t xs(uint32_t& s) {
  s ^= s << 13;
  s ^= s >> 17;
  s ^= s << 5;
  return s;
}
fp rnd_fp(uint32_t& s) {
  uint32_t t[8];
  for (int i = 0; i < 8; i++) t[i] = xs(s);
  t[7] &= 0x1FFFFFFF;
  return fe_from_int<ModP>(t);
}
fp12 rnd_f12(uint32_t& s) {
  fp12 f;
  fp* p = &f.c0.c0.c0;
  for (int i = 0; i < 12; i++) p[i] = rnd_fp(s);
  return f;
}
fp12 from_coefs(const fp2 c[6]) {
  fp12 f;
  f.c0.c0 = c[0];
  f.c1.c0 = c[1];
  f.c0.c1 = c[2];
  f.c1.c1 = c[3];
  f.c0.c2 = c[4];
  f.c1.c2 = c[5];
  return f;
}

fp ld_fp(const uint8_t* b) {
  uint32_t t[8];
  be32_to_limbs(t, b);
  return fe_from_int<ModP>(t);
}
g1a ld_g1(const uint8_t* b) {
  g1a a;
  a.x = ld_fp(b);
  a.y = ld_fp(b + 32);
  a.inf = is_zero(a.x) && is_zero(a.y);
  return a;
}
g2a ld_g2(const uint8_t* b) {
  g2a a;
  a.x.c1 = ld_fp(b);
  a.x.c0 = ld_fp(b + 32);
  a.y.c1 = ld_fp(b + 64);
  a.y.c0 = ld_fp(b + 96);
  a.inf = f2_is_zero(a.x) && f2_is_zero(a.y);
  return a;
}

}  // namespace

extern "C" {

// Returns a bitmask of mismatching operations (0 = all sextet ops equal the
// one-lane tower ops) over `iters` random inputs:
// 1 mul, 2 sqr, 4 line, 8 cyc, 16 frob1, 32 frob2, 64 frob3, 128 inv, 256 conj, 512 expt
int sxe_ops(uint32_t seed, int iters) {
  int bad = 0;
  uint32_t s = seed | 1;
  for (int it = 0; it < iters; it++) {
    fp12 a = rnd_f12(s), b = rnd_f12(s);
    fp2 l0 = {rnd_fp(s), rnd_fp(s)}, l1 = {rnd_fp(s), rnd_fp(s)}, l3 = {rnd_fp(s), rnd_fp(s)};
    // a cyclotomic element for cyc / expt: easy part of the final exponentiation
    fp12 c = f12_conj(a) * f12_inv(a);
    c = f12_frob2(c) * c;
    fp2 r[10][6];
    run6([&](const SxH& x) {
      int k = x.k;
      fp2 ak = f12_coef(a, k), bk = f12_coef(b, k), ck = f12_coef(c, k);
      r[0][k] = sx_mulv(x, ak, bk);
      r[1][k] = sx_sqr(x, ak);
      if (k == 0) {
        x.put(SX_L + 0, l0);
        x.put(SX_L + 1, l1);
        x.put(SX_L + 2, l3);
      }
      x.sync();
      r[2][k] = sx_mul_line(x, ak, SX_L);
      r[3][k] = sx_cyc_sqr(x, ck);
      r[4][k] = sx_frob1(k, ak);
      r[5][k] = sx_frob2(k, ak);
      r[6][k] = sx_frob3(k, ak);
      r[7][k] = sx_inv(x, ak);
      r[8][k] = sx_conj(k, ak);
      r[9][k] = it == 0 ? sx_expt(x, ck) : ck;
    });
    fp12 want[10] = {a * b,        f12_sqr(a),   f12_mul_034(a, l0, l1, l3), f12_cyclo_sqr(c), f12_frob(a),
                     f12_frob2(a), f12_frob3(a), f12_inv(a),                 f12_conj(a),      it == 0 ? f12_expt(c) : c};
    for (int o = 0; o < 10; o++)
      if (!f12_eq(from_coefs(r[o]), want[o])) bad |= 1 << o;
  }
  return bad;
}

// dev/g2x29.h's scanned products against sx29.h's column products: the same
// columns and digits, so the same words.  Operands: random balanced values,
// differences of two (limbs within 2^29), and all-extreme limbs; returns the
// number of mismatches (1 mul, 2 sqr per failing case, summed)
int sxe_q2_scan(uint32_t seed, int iters) {
  uint32_t s = seed | 1;
  auto bal = [&]() { return q2_from_fp2(fp2{rnd_fp(s), rnd_fp(s)}); };
  auto edge = [&](int32_t v) {
    q2 a;
    for (int i = 0; i < 9; i++) a.c0.l[i] = a.c1.l[i] = (i < 8) ? v : (v < 0 ? -1 : 1);
    return a;
  };
  int bad = 0;
  for (int it = 0; it < iters; it++) {
    q2 a = bal(), b = bal();
    if (it % 3 == 1) a = q2_subr(a, bal());
    if (it % 3 == 2) b = q2_subr(bal(), b);
    if (it == 0) a = edge(1 << 29), b = edge(-(1 << 28));
    if (it == 1) a = edge(-(1 << 29)), b = edge(-(1 << 28));
    q2 x = q2_mulb(a, b), y = w29_prod1(a, b);
    if (memcmp(&x, &y, sizeof(q2))) bad += 1;
    q2 c = bal();
    if (it == 2) c = edge(1 << 28);
    if (it == 3) c = edge(-(1 << 28));
    x = q2_sqrb(c);
    y = w29_prod1(c, c);
    if (memcmp(&x, &y, sizeof(q2))) bad += 2;
  }
  return bad;
}

// final exponentiation of a random Fp12: sextet vs one-lane (GT bytes);
// variant 0 = exact (k_fexp_exact), 1 = Fuentes (k_fexp)
int sxe_fexp(uint32_t seed, int variant, uint8_t* out_sx, uint8_t* out_ref) {
  uint32_t s = seed | 1;
  fp12 f = rnd_f12(s);
  f12_to_bytes(out_ref, final_exp(f, variant));
  run6([&](const SxH& x) {
    fp2 g = variant == 1 ? sx_final_exp(x, f12_coef(f, x.k)) : sx_final_exp_exact(x, f12_coef(f, x.k));
    sx_gt_bytes(out_sx, x.k, g);
  });
  return memcmp(out_sx, out_ref, 384) != 0;
}

// the same with the carry-free sextet final exponentiation (dev/sx29.h)
// the device's easy part in three phases (sq_fexp_easy_a, the batched
// inversion -- here fp_inv_var of the parked n, as k_fexp_binv computes it --
// and sq_fexp_easy_b) against sq_fexp_easy in one piece: the same m words.
// zero_norm forces the n = 0 branch (n^-1 = 0 in both).
int sxe_fexp_easy_split(uint32_t seed) {
  uint32_t s = seed | 1;
  int bad = 0;
  for (int it = 0; it < 4; it++) {
    fp12 f = rnd_f12(s);
    std::vector<int32_t> park(6 * FEXP_PARK_SLOTS * 18, 0);
    q2 one[6], split[6];
    run6q([&](const SqH& x) { one[x.k] = sq_fexp_easy(x, f12_coef(f, x.k)); });
    run6q([&](const SqH& x) {
      Park pk{park.data(), (uint32_t)x.k, 6, true};
      sq_fexp_easy_a(x, f12_coef(f, x.k), pk, 0u);
    });
    {
      Park pk{park.data(), 0, 6, true};
      pk.put_fp(FEXP_EASY_N, 0, fp_inv_var(pk.get_fp(FEXP_EASY_N, 0)));
    }
    run6q([&](const SqH& x) {
      Park pk{park.data(), (uint32_t)x.k, 6, true};
      split[x.k] = sq_fexp_easy_b(x, f12_coef(f, x.k), pk, 0u);
    });
    for (int k = 0; k < 6; k++)
      if (memcmp(&one[k], &split[k], sizeof(q2))) bad++;
  }
  return bad;
}

int sxe_fexp29(uint32_t seed, int variant, uint8_t* out_sx, uint8_t* out_ref) {
  uint32_t s = seed | 1;
  fp12 f = rnd_f12(s);
  f12_to_bytes(out_ref, final_exp(f, variant));
  std::vector<int32_t> park(6 * FEXP_PARK_SLOTS * 18, (int32_t)0xA5A5A5A5);  // lane planes, stride 6
  run6q([&](const SqH& x) {
    Park pk{park.data(), (uint32_t)x.k, 6, true};
    fp2 g = variant == 1 ? sq_final_exp(x, f12_coef(f, x.k), pk) : sq_final_exp_exact(x, f12_coef(f, x.k), pk);
    sx_gt_bytes(out_sx, x.k, g);
  });
  return memcmp(out_sx, out_ref, 384) != 0;
}

// 2-pair Miller loop: sextet vs one-lane, raw Fp12 (same formulas => equal).
// p1, p2: G1 RawBytes (64); q2, qfix: G2 RawBytes (128, X.A1|X.A0|Y.A1|Y.A0).
int sxe_miller(const uint8_t* p1, const uint8_t* p2, const uint8_t* q2, const uint8_t* qfix, uint8_t* out_sx,
               uint8_t* out_ref) {
  std::vector<LineCoef> ql(MILLER_LINES);
  precompute_lines(ql.data(), ld_g2(qfix));
  g1a P1 = ld_g1(p1), P2 = ld_g1(p2);
  g2a Q2 = ld_g2(q2);
  fp12 want = miller_2(ql.data(), P1, P2, Q2);
  fp2 got[6];
  run6([&](const SxH& x) { got[x.k] = sx_miller_2(x, ql.data(), P1, P2, Q2); });
  // the production path: pair-2 lines precomputed (g2lines_emit), f-chain only
  std::vector<EvLineDev> l2(MILLER_LINES);
  g2lines_emit(Q2, P2, l2.data(), 0, 1);
  fp2 got2[6];
  run6([&](const SxH& x) { got2[x.k] = sx_miller_f(x, ql.data(), P1, l2.data(), 0, 1); });
  if (!f12_eq(from_coefs(got2), want)) return 2;
  f12_to_bytes(out_ref, want);
  f12_to_bytes(out_sx, from_coefs(got));
  return memcmp(out_sx, out_ref, 384) != 0;
}

// carry-free Miller f-chain (dev/sx29.h sq_miller_f, the device path) vs the
// one-lane miller_2: 0 = equal
int sxe_miller29(const uint8_t* p1, const uint8_t* p2, const uint8_t* q2b, const uint8_t* qfix) {
  std::vector<LineCoef> ql(MILLER_LINES);
  precompute_lines(ql.data(), ld_g2(qfix));
  std::vector<LineCoef29> ql29(MILLER_LINES);
  for (int i = 0; i < MILLER_LINES; i++) ql29[i] = linecoef29(ql[i]);
  g1a P1 = ld_g1(p1), P2 = ld_g1(p2);
  g2a Q2 = ld_g2(q2b);
  fp12 want = miller_2(ql.data(), P1, P2, Q2);
  std::vector<EvLineDev> l2(MILLER_LINES);
  g2lines_emit(Q2, P2, l2.data(), 0, 1);
  fp2 got[6];
  run6q([&](const SqH& x) { got[x.k] = q2_to_fp2(sq_miller_f(x, ql29.data(), P1, l2.data(), 0, 1)); });
  if (!f12_eq(from_coefs(got), want)) return 1;
  // normalised fixed lines (k_qlines out29n, k_miller_n): the evaluation point
  // (x/y, 1/y) from g1_pnorm on a Jacobian representative with Z != 1 (as the
  // G1 combine sees it); equal to miller_2 after the final exponentiation
  std::vector<LineCoef29> qn(MILLER_LINES);
  for (int i = 0; i < MILLER_LINES; i++) {
    fp2 ri = f2_inv(ql[i].r0);
    qn[i] = linecoef29(LineCoef{f2_one(), ql[i].r1 * ri, ql[i].r2 * ri});
  }
  G1Dev pn;
  memset(&pn, 0, sizeof(pn));
  if (!P1.inf) {
    fp lam = fe_from_int<ModP>(std::vector<uint32_t>{7, 11, 13, 17, 19, 23, 29, 31}.data());
    fp l2_ = sqr(lam);
    g1j J = {P1.x * l2_, P1.y * l2_ * lam, lam};
    g1_pnorm(J, fp_inv(J.z * J.y), pn);
    fp xq, yi;
    g1dev_get(pn, xq, yi);
    if (!fe_eq(yi * P1.y, fe_one<ModP>()) || !fe_eq(xq * P1.y, P1.x)) return 3;
  }
  fp2 gotn[6];
  run6q([&](const SqH& x) { gotn[x.k] = q2_to_fp2(sq_miller_fn(x, qn.data(), P1, pn, l2.data(), 0, 1)); });
  uint8_t a[384], b[384];
  f12_to_bytes(a, final_exp(from_coefs(gotn), 0));
  f12_to_bytes(b, final_exp(want, 0));
  return memcmp(a, b, 384) ? 2 : 0;
}

// G2 job + pair-2 lines: sextet (sx_job_g2lines) vs one lane (job_g2lines).
// bases: 3 G2 RawBytes (PK0..2), p2: G1 RawBytes (R), scalars: 3 x 32 bytes BE.
// Only the table entries the scalars touch are built.
int sxe_g2lines(const uint8_t* bases, const uint8_t* p2, const uint8_t* scalars) {
  std::vector<G2Dev> b(4);
  for (int i = 0; i < 3; i++) g2_store(b[i], ld_g2(bases + 128 * i));
  std::vector<uint32_t> sc(8 * 3);
  for (int i = 0; i < 3; i++) be32_to_limbs(&sc[8 * i], scalars + 32 * i);
  std::vector<G2Dev> tab((size_t)G2B_COUNT * G2TAB_WINDOWS * G2TAB_DIGITS);
  for (int f = 0; f < 3; f++)
    for (int w = 0; w < G2TAB_WINDOWS; w++) {
      int32_t d = sdigit_at(&sc[8 * f], G2TAB_C, w);
      if (d)
        job_tab_g2((uint32_t)((f * G2TAB_WINDOWS + w) * G2TAB_DIGITS + (d < 0 ? -d : d) - 1), b.data(), tab.data());
    }
  G2Job g;
  memset(&g, 0, sizeof(g));
  g.nfix = 3;
  for (int f = 0; f < 3; f++) {
    g.fbase[f] = (uint8_t)f;
    g.fscal[f] = (uint32_t)f;
  }
  g.out = 0;
  G1Dev pt;
  g1_store(pt, ld_g1(p2));
  PairJob j = {0, 0, 0, 0};
  const uint32_t(*scal)[8] = reinterpret_cast<const uint32_t(*)[8]>(sc.data());
  std::vector<G2Dev> o1(1), o2(1);
  std::vector<EvLineDev> l1(MILLER_LINES), l2(MILLER_LINES);
  job_g2lines(g, j, scal, tab.data(), o1.data(), &pt, l1.data(), 0, 1);
  run6([&](const SxH& x) { sx_job_g2lines(x, g, j, scal, tab.data(), o2.data(), &pt, l2.data(), 0, 1, true); });
  if (memcmp(o1.data(), o2.data(), sizeof(G2Dev))) return 1;
  for (int s = 0; s < MILLER_LINES; s++)
    if (memcmp(&l1[s], &l2[s], sizeof(EvLineDev))) return 2 + s;
  // the split one-lane device path (k_g2_part + k_g2lines1)
  std::vector<G2PartDev> part(4);
  for (int q = 0; q < 4; q++) job_g2_part(g, q, scal, tab.data(), part[q]);
  for (int q = 0; q < 4; q++) {  // the carry-free part kernel writes the same words
    G2PartDev p29;
    job_g2_part29(g, q, scal, tab.data(), p29);
    if (memcmp(&p29, &part[q], sizeof(G2PartDev))) return 200 + q;
  }
  std::vector<G2Dev> o3(1);
  std::vector<EvLineDev> l3(MILLER_LINES);
  job_g2lines_parts(g, j, part.data(), o3.data(), &pt, l3.data(), 0, 1);
  if (memcmp(o1.data(), o3.data(), sizeof(G2Dev))) return 100;
  for (int s = 0; s < MILLER_LINES; s++)
    if (memcmp(&l1[s], &l3[s], sizeof(EvLineDev))) return 101 + s;
  // the XYZZ carry-free part kernel (dev/g2x29.h, the device default): other
  // Jacobian representatives, the same t' and lines
  for (int q = 0; q < 4; q++) job_g2_part_x29(g, q, scal, tab.data(), part[q]);
  std::vector<G2Dev> o4(1);
  std::vector<EvLineDev> l4(MILLER_LINES);
  job_g2lines_parts(g, j, part.data(), o4.data(), &pt, l4.data(), 0, 1);
  if (memcmp(o1.data(), o4.data(), sizeof(G2Dev))) return 300;
  for (int s = 0; s < MILLER_LINES; s++)
    if (memcmp(&l1[s], &l4[s], sizeof(EvLineDev))) return 301 + s;
  return 0;
}

// the literal constants of tests/native/g2l29.h against their conversions: 0 = equal
int sxe_g2l29_consts() {
  const q2 b3 = q2_scale(q2_from_fp2(f2_const(TWIST_B)), 3);
  const q2 fx = q2_from_fp2(f2_const(TW_FROB_X)), fy = q2_from_fp2(f2_const(TW_FROB_Y));
  const f29 want[9] = {b3.c0, b3.c1, fx.c0, fx.c1, fy.c0, fy.c1, f29_breduce(f29_from_fp(fe_const<ModP>(TW_FROB2_X))),
                       f29_breduce(f29_from_fp(fe_const<ModP>(TW_FROB2_Y))), f29_breduce(f29_from_fp(fe_one<ModP>()))};
  for (int i = 0; i < 9; i++)
    for (int k = 0; k < 9; k++)
      if (want[i].l[k] != G2L29_CONST[i][k]) return 1 + i;
  return 0;
}

// G2 job + pair-2 lines, one lane on the carry-free form (tests/native/g2l29.h
// job_g2lines29) vs the 32-bit one lane (job_g2lines): the same affine t', and
// lines equal up to Fp factors, so the carry-free Miller f-chain with either
// set of lines (fixed pair: qfix at p1) gives the same final exponentiation.
// Returns 0 = equal, 1 = t' differs, 2 = GT differs.
int sxe_g2lines29(const uint8_t* bases, const uint8_t* p2, const uint8_t* scalars, const uint8_t* p1,
                  const uint8_t* qfix, uint8_t* gt) {
  std::vector<G2Dev> b(4);
  for (int i = 0; i < 3; i++) g2_store(b[i], ld_g2(bases + 128 * i));
  std::vector<uint32_t> sc(8 * 3);
  for (int i = 0; i < 3; i++) be32_to_limbs(&sc[8 * i], scalars + 32 * i);
  std::vector<G2Dev> tab((size_t)G2B_COUNT * G2TAB_WINDOWS * G2TAB_DIGITS);
  for (int f = 0; f < 3; f++)
    for (int w = 0; w < G2TAB_WINDOWS; w++) {
      int32_t d = sdigit_at(&sc[8 * f], G2TAB_C, w);
      if (d)
        job_tab_g2((uint32_t)((f * G2TAB_WINDOWS + w) * G2TAB_DIGITS + (d < 0 ? -d : d) - 1), b.data(), tab.data());
    }
  G2Job g;
  memset(&g, 0, sizeof(g));
  g.nfix = 3;
  for (int f = 0; f < 3; f++) {
    g.fbase[f] = (uint8_t)f;
    g.fscal[f] = (uint32_t)f;
  }
  G1Dev pt;
  g1_store(pt, ld_g1(p2));
  PairJob j = {0, 0, 0, 0};
  const uint32_t(*scal)[8] = reinterpret_cast<const uint32_t(*)[8]>(sc.data());
  std::vector<G2Dev> o1(1), o2(1);
  std::vector<EvLineDev> l1(MILLER_LINES), l2(MILLER_LINES);
  job_g2lines(g, j, scal, tab.data(), o1.data(), &pt, l1.data(), 0, 1);
  job_g2lines29<0>(g, j, scal, tab.data(), o2.data(), &pt, l2.data(), 0, 1);
  if (memcmp(o1.data(), o2.data(), sizeof(G2Dev))) return 1;
  // the device's k_g2_part + k_g2lines1 (dev/g2x29.h, dev/g2lines29.h)
  std::vector<G2PartDev> part(4);
  for (int q = 0; q < 4; q++) job_g2_part_x29(g, q, scal, tab.data(), part[q]);
  std::vector<G2Dev> o3(1);
  std::vector<EvLineDev> l3(MILLER_LINES);
  job_g2lines_parts_x29(g, j, part.data(), o3.data(), &pt, l3.data(), 0, 1);
  if (memcmp(o1.data(), o3.data(), sizeof(G2Dev))) return 3;
  // the device default: k_g2_sum, the batched inversion of N(Z) (one job
  // here: its inverse), k_g2lines1 from the sum -- the same bytes
  {
    std::vector<G2PartDev> ps(part);
    job_g2_sum(ps.data(), 0, 1);
    fp nz;
    for (int i = 0; i < 8; i++) nz.v[i] = ps[1].w[i];
    nz = fe_is_zero(nz) ? fe_zero<ModP>() : fp_inv_var(nz);
    for (int i = 0; i < 8; i++) ps[1].w[i] = nz.v[i];
    std::vector<G2Dev> o5(1);
    std::vector<EvLineDev> l5(MILLER_LINES);
    job_g2lines_summed_x29(g, j, ps.data(), o5.data(), &pt, l5.data(), 0, 1);
    if (memcmp(o3.data(), o5.data(), sizeof(G2Dev))) return 5;
    for (int s = 0; s < MILLER_LINES; s++)
      if (memcmp(&l3[s], &l5[s], sizeof(EvLineDev))) return 6;
  }
  std::vector<LineCoef> ql(MILLER_LINES);
  precompute_lines(ql.data(), ld_g2(qfix));
  std::vector<LineCoef29> ql29(MILLER_LINES);
  for (int i = 0; i < MILLER_LINES; i++) ql29[i] = linecoef29(ql[i]);
  g1a P1 = ld_g1(p1);
  uint8_t out[3][384];
  for (int v = 0; v < 3; v++) {
    const EvLineDev* l = v == 2 ? l3.data() : (v ? l2.data() : l1.data());
    fp2 got[6];
    run6q([&](const SqH& x) { got[x.k] = q2_to_fp2(sq_miller_f(x, ql29.data(), P1, l, 0, 1)); });
    f12_to_bytes(out[v], final_exp(from_coefs(got), 0));
  }
  memcpy(gt, out[1], 384);
  if (memcmp(out[0], out[2], 384)) return 4;
  return memcmp(out[0], out[1], 384) ? 2 : 0;
}

}  // extern "C"

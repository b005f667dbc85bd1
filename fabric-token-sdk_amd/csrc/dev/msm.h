// BN254 G1 multi-scalar multiplication  sum_i k_i P_i  (Pippenger, signed
// c-bit windows), the standalone MSM of BASELINE.json configs[2].  The
// reference path has no MSM; the operation is what
// mathlib exposes from gnark-crypto v0.6.0 as G1Jac.MultiExp [EXT]: the result
// is the unique group element, so any correct bucket order gives the same bytes.
//
// Pipeline (k_msm.hip; every stage one lane per item):
//   keys      k_i -> W signed digits d in [-2^(c-1), 2^(c-1)]; sort key = the
//             bucket |d| - 1 within the window (c - 1 bits), value = the
//             entry index t = w nv + v | sign (| ZERO for a zero digit)
//   sort      stable LSD radix sort of the (key, value) pairs (rocPRIM); the
//             entries are generated window-major, so stability keeps each
//             bucket's entries grouped by window
//   bounds    (window, bucket) ranges [start, end) read off the sorted keys and
//             the windows of the sorted values
//   slots     bucket b gets m_b = max(1, ceil(count_b / T)) slots of at most T
//             points (scan of m_b -> slot offsets, slot -> bucket owner map), so
//             that heavy buckets (the top window's few buckets, skewed scalars)
//             are spread over several lanes
//   bucket    one lane per slot: Jacobian sum of its <= T points
//   segment   one lane per run of S consecutive slots of one window: running
//             sums give sum (b+1) S_b restricted to the run
//   window    tree sum of the segments through LDS (quad-cooperative
//             additions) down to one part per window
//   final     the window sums read back; Horner over the windows, affine and
//             gnark RawBytes on the host (msm_rt.hip msm_horner_host)
//
// Resident-point mode (MsmPlan.pre, ftz_options.msm_precompute): the points of
// an ftz_msm handle stay on the device across runs (ftz_msm_set_scalars swaps
// the scalars), so ftz_msm_load also stores 2^(c w) P_v for every window w
// (msm_job_precompute).  Window w's digits then select buckets of ONE shared
// bucket set over those points -- sum_w 2^(c w) sum_b (b+1) S_(w,b) becomes
// sum_b (b+1) sum_w S'_(w,b) -- so the bucket reduction runs over B buckets
// instead of W B and the Horner chain of c (W-1) serial doublings disappears;
// zero digits go to bucket 0 with the identity point (a skipped load), so the
// sort keys are c - 1 bits.  Memory: W nv 64 bytes of points (1 GiB at 2^20).
#pragma once
#include "jobs.h"

namespace fts {

struct MsmPlan {
  uint32_t n;          // points
  uint32_t glv;        // 1: scalars split k = k1 + k2 lambda (|k_i| < 2^128) over P_i and phi(P_i)
  uint32_t nv;         // virtual points: 2n with GLV (index n + i is phi(P_i) = (beta x_i, y_i)), else n
  uint32_t c;          // window bits
  uint32_t windows;    // W = ceil(bits / c), bits = 129 (GLV halves) or 255
  uint32_t buckets;    // B = 2^(c-1) per window
  uint32_t slot_cap;   // T: points per bucket slot
  uint32_t seg_len;    // S: slots per segment
  uint32_t max_slots;  // per window: B + ceil(n / T) bounds sum_b m_b
  uint32_t segs;       // segments per window: ceil(max_slots / S)
  uint32_t pre;        // 1: resident-point mode (points 2^(c w) P_v precomputed, one bucket set)
  uint32_t rw;         // reduction windows: W, or 1 with pre
  uint32_t per;        // sort entries per reduction window: nv, or W nv with pre
  uint32_t pts;        // resident points: nv + 1, or W nv + 1 with pre (last = the identity)
  uint64_t nv_magic;   // floor(2^32 / nv) + 1: the window of an entry t without a division
};

// k_msm_tree: parts per block (quad-cooperative additions: 128, one lane each: 256)
#ifndef FTS_MSM_QUAD_TREE
#define FTS_MSM_QUAD_TREE 1
#endif
static constexpr uint32_t MSM_TREE_CHUNK = FTS_MSM_QUAD_TREE ? 128u : 256u;
// k_msm_segment: one quad per segment (64 per 256-lane block) or one lane each
// (default: the quads measured slower, 2^16 segment stage 264 against 188 us,
// 2^20 523 against 282, profiles/r06/msm_tail.txt)
#ifndef FTS_MSM_QUAD_SEG
#define FTS_MSM_QUAD_SEG 0
#endif
static constexpr uint32_t MSM_SEG_THREADS = FTS_MSM_QUAD_SEG ? 256u : 128u;
static constexpr uint32_t MSM_SEG_PER_BLOCK = FTS_MSM_QUAD_SEG ? 64u : 128u;

// the window combination (Horner) on the host from the read-back window sums
// (msm_rt.hip msm_horner_host); 0: on one wave of the device (k_msm_horner)
#ifndef FTS_MSM_HOST_HORNER
#define FTS_MSM_HOST_HORNER 1
#endif

// window bits for n (virtual) points: floor(log2 n / 2) + 7 clamped to [8, 20]
// (measured on MI355X with GLV: 2^17 -> 15, 2^21 -> 17, 2^25 -> 19; the
// latency-bound reduction favours fewer windows than the usual log2 n - 4)
FTS_HD uint32_t msm_window_bits(uint64_t n) {
  uint32_t lg = 0;
  while ((1ull << (lg + 1)) <= n) lg++;
  uint32_t c = lg / 2 + 7;
  if (c < 8) c = 8;
  if (c > 20) c = 20;
  return c;
}

// variable base with the host window combination (round 6; msmtune sweeps in
// profiles/r06/msm_plan.txt, 2^14 .. 2^24 points): up to 2^19 virtual points
// 13-bit windows with slots of <= 16 points and 4-slot segments (2^17 points:
// 0.77 ms against 1.11 at c = 16; 2^18: 1.17 against 1.37); above, the
// round-5 rule except where it picks c = 18, whose top window of the 129-bit
// halves keeps 3 bits (2^21 points: 4.21 ms at 17 against 5.37 at 18; 2^22:
// 7.67 at 19 against 9.13).
static constexpr uint32_t MSM_SMALL_LG = 19;
FTS_HD uint32_t msm_lg(uint64_t n) {
  uint32_t lg = 0;
  while ((1ull << (lg + 1)) <= n) lg++;
  return lg;
}
FTS_HD uint32_t msm_window_bits_var(uint64_t nv) {
  const uint32_t lg = msm_lg(nv);
  if (lg <= MSM_SMALL_LG) return 13;
  if (lg == 22) return 17;
  if (lg == 23) return 19;
  return msm_window_bits(nv);
}

// resident-point mode: the bucket reduction runs once (not per window), and
// the sort keys are c - 1 bits.  Up to 2^22 virtual points the variable-base
// width (<= 17: keys of <= 16 bits, two radix passes); above, the bucket
// additions dominate and c = 22 (6 windows instead of 7-8) pays for the third
// pass.  Measured: 2^20 points 2.71 ms at 17 against 2.89 at 19; 2^24 26.6 ms
// at 22 against 28.4 at 19.
FTS_HD uint32_t msm_window_bits_pre(uint64_t nv, bool glv) {
  (void)glv;
  return nv <= (1ull << 22) ? msm_window_bits(nv) : 22u;
}

// plan for n points with c-bit windows (0: msm_window_bits of the virtual point
// count), slot cap T (0: twice the mean bucket load, at least 4) and S slots per
// segment (0: sized for >= 64k segment lanes, in [4, 64]).  GLV halves the
// scalar length, so the Horner chain of c (W-1) doublings and the bucket
// reduction shrink by half for the same number of bucket additions.
inline MsmPlan msm_make_plan(uint64_t n, uint32_t c = 0, uint32_t slot_cap = 0, uint32_t seg_len = 0,
                             bool glv = true, bool pre = false) {
  MsmPlan p;
  p.n = (uint32_t)n;
  p.glv = glv ? 1 : 0;
  p.nv = glv ? 2 * p.n : p.n;
  p.c = c ? c : (pre ? msm_window_bits_pre(p.nv, glv) : msm_window_bits_var(p.nv));
  const bool small = !pre && msm_lg(p.nv) <= MSM_SMALL_LG;
  uint32_t bits = glv ? 129 : 255;  // magnitude bits + 1 for the signed-digit carry
  p.windows = (bits + p.c - 1) / p.c;
  p.buckets = 1u << (p.c - 1);
  p.pre = pre ? 1 : 0;
  p.rw = pre ? 1 : p.windows;
  p.per = pre ? p.windows * p.nv : p.nv;
  p.pts = pre ? p.windows * p.nv + 1 : p.nv + 1;
  p.nv_magic = (1ull << 32) / p.nv + 1;
  // the default cap keeps the per-window mean (about as many bucket lanes per
  // point as without pre)
  if (!slot_cap && small) slot_cap = 16;
  if (!slot_cap) {
    uint64_t mean = (p.nv + p.buckets - 1) / p.buckets;
    slot_cap = (uint32_t)(2 * mean < 4 ? 4 : 2 * mean);
  }
  if (slot_cap > 1023) slot_cap = 1023;  // length bins of the slot ordering (k_msm.hip)
  p.slot_cap = slot_cap;
  p.max_slots = p.buckets + (uint32_t)((p.per + slot_cap - 1) / slot_cap);
  if (!seg_len && pre) {
    // at most ~24k segment lanes, S in [4, 64]: measured best at 2^16 (90k
    // slots, S = 4: 0.63-0.65 ms against 0.84 with 16), 2^20 (328k slots,
    // S = 16: 2.54 ms against 3.54 with 64 and 2.85 with 32) and 2^24 (8.4M
    // slots, S = 64: 26.0 ms against 26.7 with 16)
    seg_len = 4;
    while (seg_len < 64 && p.max_slots / seg_len > 24576) seg_len *= 2;
  }
  if (!seg_len && small) seg_len = 4;
  if (!seg_len) {
    uint64_t tot = (uint64_t)p.rw * p.max_slots;
    seg_len = 4;
    while (seg_len < 64 && tot / (2 * seg_len) >= 65536) seg_len *= 2;
  }
  p.seg_len = seg_len;
  p.segs = (p.max_slots + seg_len - 1) / seg_len;
  return p;
}

// Signed digits of k (8 limbs, k < 2^255) for window w: raw c-bit chunk plus the
// carry of the window below.  Returns d in [-2^(c-1), 2^(c-1)].
FTS_HD int32_t msm_digit(const uint32_t k[8], uint32_t c, uint32_t w, uint32_t& carry) {
  uint32_t bit = c * w, limb = bit >> 5, sh = bit & 31;
  uint64_t lo = limb < 8 ? k[limb] : 0, hi = limb + 1 < 8 ? k[limb + 1] : 0;
  uint32_t raw = (uint32_t)(((lo | (hi << 32)) >> sh) & ((1ull << c) - 1)) + carry;
  if (raw > (1u << (c - 1))) {
    carry = 1;
    return (int32_t)raw - (int32_t)(1u << c);
  }
  carry = 0;
  return (int32_t)raw;
}

// Sort keys of point i (both GLV halves): window w's entry t = w nv + vi gets
// key[t] = |d| - 1, the bucket within the window, and val[t] = t | sign << 31.
// A zero digit goes to bucket 0 with the identity: val = t | MSM_ZERO (the
// bucket pass loads the identity point for it and skips it; pre: the value is
// the index of the identity point).  Keys are c - 1 bits -- one radix pass
// fewer than keys w B + b with a sort-last bit for zero digits (2^20: 16
// bits, two passes instead of three) -- and the stable sort keeps each
// bucket's entries in window order, so msm_job_bounds reads the (window,
// bucket) ranges off (key, window of the value): no atomics, coalesced writes.
// Non-pre values hold t in 30 bits: W nv < 2^30 (msm_rt.hip checks it).
static constexpr uint32_t MSM_ZERO = 0x40000000u;
static constexpr uint32_t MSM_T_MASK = 0x3FFFFFFFu;

// key bits the sort must look at: the bucket within a window (c - 1 bits)
FTS_HD uint32_t msm_key_bits(const MsmPlan& p) { return p.c > 1 ? p.c - 1 : 1; }

FTS_HD void msm_put_key(const MsmPlan& p, uint32_t w, uint32_t vi, int32_t d, bool neg, uint32_t* key,
                        uint32_t* val) {
  size_t t = (size_t)w * p.nv + vi;
  if (d == 0) {
    key[t] = 0;
    val[t] = p.pre ? p.pts - 1 : (uint32_t)t | MSM_ZERO;
    return;
  }
  key[t] = (uint32_t)(d < 0 ? -d : d) - 1;
  val[t] = (uint32_t)t | (((d < 0) != neg) ? 0x80000000u : 0u);
}

FTS_HD void msm_job_keys(const MsmPlan& p, uint32_t i, const uint32_t (*scal)[8], uint32_t* key, uint32_t* val) {
  if (p.glv) {
    uint32_t k1[4], k2[4];
    bool n1, n2;
    glv_split(scal[i], k1, n1, k2, n2);
    uint32_t a[8] = {k1[0], k1[1], k1[2], k1[3], 0, 0, 0, 0}, b[8] = {k2[0], k2[1], k2[2], k2[3], 0, 0, 0, 0};
    uint32_t ca = 0, cb = 0;
    for (uint32_t w = 0; w < p.windows; w++) {
      msm_put_key(p, w, i, msm_digit(a, p.c, w, ca), n1, key, val);
      msm_put_key(p, w, p.n + i, msm_digit(b, p.c, w, cb), n2, key, val);
    }
  } else {
    uint32_t carry = 0;
    for (uint32_t w = 0; w < p.windows; w++) msm_put_key(p, w, i, msm_digit(scal[i], p.c, w, carry), false, key, val);
  }
}

// the window of entry index x = w nv + v (x < 2^30): x nv_magic / 2^32 is
// floor(x / nv) or one more (x / 2^32 < 1/4 of slack), one compare fixes it
FTS_HD uint32_t msm_window_of(const MsmPlan& p, uint32_t x) {
  uint32_t w = (uint32_t)(((uint64_t)x * p.nv_magic) >> 32);
  return (uint64_t)w * p.nv > x ? w - 1 : w;
}

// global bucket of sorted entry t: w B + key (pre: one bucket set, g = key)
FTS_HD uint32_t msm_entry_bucket(const MsmPlan& p, uint64_t t, const uint32_t* skey, const uint32_t* sval) {
  if (p.pre) return skey[t];
  return msm_window_of(p, sval[t] & MSM_T_MASK) * p.buckets + skey[t];
}

// sorted entry t and its successor: where the (window, bucket) changes, the
// one ends (end[g] = t + 1) and the next starts (start[g'] = t + 1); start /
// end zeroed beforehand, so an empty bucket reads 0, 0
FTS_HD void msm_job_bounds(const MsmPlan& p, uint64_t t, uint64_t total, const uint32_t* skey, const uint32_t* sval,
                           uint32_t* start, uint32_t* end) {
  uint32_t g = msm_entry_bucket(p, t, skey, sval);
  if (t == 0) start[g] = 0;
  if (t + 1 == total) {
    end[g] = (uint32_t)total;
    return;
  }
  uint32_t g1 = msm_entry_bucket(p, t + 1, skey, sval);
  if (g1 != g) {
    end[g] = (uint32_t)(t + 1);
    start[g1] = (uint32_t)(t + 1);
  }
}

// virtual point v of the resident array: P_v for v < n, phi(P_(v-n)) =
// (beta x, y) for n <= v < 2n (GLV; filled once at load, msm_job_phi)
FTS_HD void msm_job_phi(const MsmPlan& p, uint32_t i, G1Dev* pts) {
  g1a P = g1_load(pts[i]);
  if (!P.inf) P.x = P.x * fe_const<ModP>(GLV_BETA);
  G1Dev d;
  g1_store(d, P);
  pts[p.n + i] = d;
}

// pre: resident point w nv + v = 2^(c w) P_v for w = 1..W-1 (affine), from
// P_v (window 0, already holding phi(P) for v >= n); the identity stays zero
FTS_HD void msm_job_precompute(const MsmPlan& p, uint32_t v, G1Dev* pts) {
  g1a P = g1_load(pts[v]);
  g1j acc = {P.x, P.y, fe_one<ModP>()};
  for (uint32_t w = 1; w < p.windows; w++) {
    g1a r;
    r.inf = P.inf;
    if (!P.inf) {
      for (uint32_t q = 0; q < p.c; q++) acc = jac_dbl(acc);
      // P has order r, so 2^k P is never the identity
      fp zi = fp_inv_var(acc.z), zi2 = sqr(zi);
      r.x = acc.x * zi2;
      r.y = acc.y * zi2 * zi;
    }
    G1Dev d;
    g1_store(d, r);
    pts[(size_t)w * p.nv + v] = d;
  }
}

// bucket g = w B + b: its slot count and, once the counts are scanned into
// soff, the slot -> bucket owner map and the window slot ranges [wlo, whi)
FTS_HD uint32_t msm_bucket_slots(const MsmPlan& p, uint32_t count) {
  uint32_t m = (count + p.slot_cap - 1) / p.slot_cap;
  return m ? m : 1;
}

FTS_HD void msm_job_owner(const MsmPlan& p, uint32_t g, const uint32_t* count, const uint32_t* soff,
                          uint32_t* owner, uint32_t* wlo, uint32_t* whi) {
  uint32_t m = msm_bucket_slots(p, count[g]), o = soff[g];
  for (uint32_t s = 0; s < m; s++) owner[o + s] = g;
  uint32_t w = g / p.buckets, b = g - w * p.buckets;
  if (b == 0) wlo[w] = o;
  if (b == p.buckets - 1) whi[w] = o + m;
}

// number of points in slot j (1..T, 0 for the slot of an empty bucket)
FTS_HD uint32_t msm_slot_len(const MsmPlan& p, uint32_t j, const uint32_t* owner, const uint32_t* soff,
                             const uint32_t* count) {
  uint32_t g = owner[j], s = j - soff[g], lo = s * p.slot_cap, hi = lo + p.slot_cap;
  if (hi > count[g]) hi = count[g];
  return hi > lo ? hi - lo : 0;
}

// Jacobian sum of slot j: points [s T, s T + T) of its bucket's sorted list
// (negated where bit 31 of the entry is set)
FTS_HD g1j msm_job_slot(const MsmPlan& p, uint32_t j, const uint32_t* owner, const uint32_t* soff,
                        const uint32_t* start, const uint32_t* count, const uint32_t* perm, const G1Dev* pts) {
  uint32_t g = owner[j], s = j - soff[g];
  uint32_t lo = s * p.slot_cap, hi = lo + p.slot_cap;
  if (hi > count[g]) hi = count[g];
  const uint32_t* e = perm + start[g];
  g1j acc = jac_inf<fp>();
  if (lo >= hi) return acc;
  // entry -> resident point: pre values are point indices; otherwise t - w nv,
  // and a zero digit loads the identity (the last point)
  const uint32_t base = p.pre ? 0u : (g / p.buckets) * p.nv, ident = p.pts - 1;
  auto point_of = [&](uint32_t v) -> uint32_t {
    return p.pre ? (v & 0x7FFFFFFFu) : ((v & MSM_ZERO) ? ident : (v & MSM_T_MASK) - base);
  };
  uint32_t v = e[lo];
  G1Dev nxt = pts[point_of(v)];
#if FTS_G1_F29
  // the additions in the carry-free XYZZ form (dev/fp29.h), one conversion per slot
  x29 a{};
  a.inf = true;
#endif
  for (uint32_t q = lo; q < hi; q++) {
    // the next point's load is issued before this point's addition
    G1Dev cur = nxt;
    uint32_t sign = v >> 31;
    if (q + 1 < hi) {
      v = e[q + 1];
      nxt = pts[point_of(v)];
    }
    g1a P = g1_load(cur);
#if FTS_G1_F29
    if (!P.inf) {
      f29 Y = f29_from_fp(P.y);
      a = x29_madd(a, f29_from_fp(P.x), sign ? f29_neg(Y) : Y);
    }
#else
    if (sign) P = aff_neg(P);
    acc = jac_add_aff(acc, P);
#endif
  }
#if FTS_G1_F29
  acc = j29_to(x29_to_j29(a));
#endif
  return acc;
}

// The reduction stages (segment, tree, Horner) are latency-bound chains of
// full additions in few lanes; they run in the carry-free form (dev/fp29.h),
// whose products accumulate columns without carry chains (shorter dependent
// chains than the 32-bit CIOS product).  Slot and segment sums are stored in
// the 32-bit Montgomery Jacobian form (G1JDev).
FTS_HD j29 j29_inf() {
  j29 o{};
  o.inf = true;
  return o;
}
FTS_HD j29 j29_ld(const G1JDev& d) { return j29_from(g1j_load(d)); }

// small-scalar multiple (k < 2^32) by 2-bit windows from the top one: P, 2P, 3P
// in registers (selects, no indexed array), two doublings and at most one
// addition per window.  The lanes of a wave take different k, so a per-bit
// conditional addition ran in every bit position for the wave (16 doublings +
// 16 additions for 16-bit k); windows halve the additions
FTS_HD j29 j29_mul_small(const j29& p, uint32_t k) {
  if (!k) return j29_inf();
  const j29 p2 = j29_dbl(p), p3 = j29_add(p2, p);
  const int top = 31 - __builtin_clz(k), w = top >> 1;
  uint32_t d = (k >> (2 * w)) & 3u;
  j29 acc = d == 1 ? p : (d == 2 ? p2 : p3);
  for (int i = w - 1; i >= 0; i--) {
    acc = j29_dbl(j29_dbl(acc));
    d = (k >> (2 * i)) & 3u;
    if (d) acc = j29_add(acc, d == 1 ? p : (d == 2 ? p2 : p3));
  }
  return acc;
}

// Segment s of window w: slots [lo, hi) of the window's slot range, covering
// consecutive buckets bl..bh (every bucket owns >= 1 slot).  Returns
//   sum_slots (b + 1) P_slot = sum (b - bl + 1) P + bl sum P,
// the first term by the running-sum trick from the top slot down.
FTS_HD g1j msm_job_segment(const MsmPlan& p, uint32_t w, uint32_t s, const uint32_t* wlo, const uint32_t* whi,
                           const uint32_t* owner, const G1JDev* slot_sum) {
  uint32_t lo = wlo[w] + s * p.seg_len, hi = lo + p.seg_len;
  if (hi > whi[w]) hi = whi[w];
  if (lo >= hi) return jac_inf<fp>();
  j29 run = j29_inf(), acc = j29_inf();
  for (uint32_t j = hi; j > lo; j--) {
    run = j29_add(run, j29_ld(slot_sum[j - 1]));
    if (j - 1 == lo || owner[j - 2] != owner[j - 1]) acc = j29_add(acc, run);
  }
  uint32_t bl = owner[lo] - w * p.buckets;
  return j29_to(j29_add(acc, j29_mul_small(run, bl)));
}

// Decode one 64-byte gnark RawBytes G1 point (uncompressed, big-endian; the
// identity is 64 zero bytes) with the load rules of k_msm_load_pts: false when
// it is not canonical (flag bits, coordinates >= p) or not on the curve.
FTS_HD bool g1_from_raw(const uint8_t* b, g1a& a) {
  uint32_t x[8], y[8], t[8], mm[8];
  be32_to_limbs(x, b);
  be32_to_limbs(y, b + 32);
  for (int q = 0; q < 8; q++) mm[q] = P_MOD[q];
  bool canon = ((b[0] & 0xC0) == 0) && sub8(t, x, mm) && sub8(t, y, mm);
  a.x = fe_from_int<ModP>(x);
  a.y = fe_from_int<ModP>(y);
  a.inf = is_zero(a.x) && is_zero(a.y);
  return canon && g1_on_curve(a);
}

// Jacobian -> affine -> gnark RawBytes (infinity: 64 zero bytes)
FTS_HD void g1j_to_raw(const g1j& acc, uint8_t out[64]) {
  g1a r;
  r.inf = is_zero(acc.z);
  fp zi = r.inf ? fe_one<ModP>() : fp_inv_var(acc.z), zi2 = sqr(zi);
  r.x = r.inf ? fe_zero<ModP>() : acc.x * zi2;
  r.y = r.inf ? fe_zero<ModP>() : acc.y * zi2 * zi;
  g1_to_bytes(out, r);
}

// Sum of n RawBytes points into out (RawBytes): the final addition of a
// point-split multi-GPU MSM, where each rank contributes the MSM of its slice
// of the points ("each GPU returns one partial sum; one gather
// and a final add").  Returns n, or the index of the first point that does not
// decode (out untouched).  Exceptional cases (identity, P + P, P - P) go
// through jac_add_aff.
FTS_HDN uint32_t g1_sum_raw(uint32_t n, const uint8_t* raw, uint8_t out[64]) {
  g1j acc = jac_inf<fp>();
  for (uint32_t i = 0; i < n; i++) {
    g1a a;
    if (!g1_from_raw(raw + 64 * (size_t)i, a)) return i;
    acc = jac_add_aff(acc, a);
  }
  g1j_to_raw(acc, out);
  return n;
}

}  // namespace fts

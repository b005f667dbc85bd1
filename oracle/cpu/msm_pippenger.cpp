// BASELINE INFRASTRUCTURE ONLY -- a CPU-tuned Pippenger for the BN254 G1 MSM
// leg's CPU baseline (bench.py cpu_msm; BASELINE configs[2]).  Nothing in the
// product loads it (it lives in oracle/cpu/libftscpu.so).
//
// The CPU algorithm gnark-crypto's G1Jac.MultiExp uses (the library mathlib
// wraps, go.mod:53 [EXT, not vendored]), restated for 4 x 64-bit Montgomery
// products (FTS_HOST64, 128-bit multiplies):
//   * scalars GLV-split k = k1 + k2 lambda (|k_i| < 2^128, dev/glv.h) over the
//     points P and phi(P) = (beta x, y), so 2n points with 129-bit scalars;
//   * signed c-bit window digits (|d| <= 2^(c-1), buckets 1 .. 2^(c-1)), c from
//     the usual cost model n W + W 2^c over the points each task sees;
//   * buckets in extended Jacobian "XYZZ" coordinates (x = X/ZZ, y = Y/ZZZ):
//     mixed additions 8M + 2S (add-2008-s / madd-2008-s), the running-sum
//     reduction in general XYZZ additions;
//   * tasks = (window, slice of the points), at least two per thread, each with
//     its own bucket array, run on `threads` std::threads; the slices of a
//     window are summed, then the windows by Horner doublings.
// The result is checked against the GPU's bit for bit by the bench (and against
// the known discrete log by tests/test_msm.py).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "../../fabric-token-sdk_amd/csrc/dev/glv.h"

using namespace fts;

namespace {

struct XYZZ {
  fp X, Y, ZZ, ZZZ;  // ZZ = 0: the point at infinity
};

inline XYZZ xyzz_inf() { return {fe_one<ModP>(), fe_one<ModP>(), fe_zero<ModP>(), fe_zero<ModP>()}; }
inline bool xyzz_is_inf(const XYZZ& p) { return is_zero(p.ZZ); }

// dbl-2008-s-1 (a = 0)
inline XYZZ xyzz_dbl(const XYZZ& p) {
  if (xyzz_is_inf(p)) return p;
  fp U = p.Y + p.Y, V = sqr(U), W = U * V, S = p.X * V, X2 = sqr(p.X), M = X2 + X2 + X2;
  XYZZ r;
  r.X = sqr(M) - S - S;
  r.Y = M * (S - r.X) - W * p.Y;
  r.ZZ = V * p.ZZ;
  r.ZZZ = W * p.ZZZ;
  return r;
}

// p + (x, y) affine: madd-2008-s with the exceptional cases
inline void xyzz_madd(XYZZ& p, const fp& x, const fp& y) {
  if (xyzz_is_inf(p)) {
    p = {x, y, fe_one<ModP>(), fe_one<ModP>()};
    return;
  }
  fp U2 = x * p.ZZ, S2 = y * p.ZZZ, P = U2 - p.X, R = S2 - p.Y;
  if (is_zero(P)) {
    if (is_zero(R)) {  // p == (x, y): mdbl-2008-s-1
      fp U = y + y, V = sqr(U), W = U * V, S = x * V, X2 = sqr(x), M = X2 + X2 + X2;
      p.X = sqr(M) - S - S;
      p.Y = M * (S - p.X) - W * y;
      p.ZZ = V;
      p.ZZZ = W;
    } else {
      p = xyzz_inf();
    }
    return;
  }
  fp PP = sqr(P), PPP = P * PP, Q = p.X * PP;
  fp X3 = sqr(R) - PPP - Q - Q;
  p.Y = R * (Q - X3) - p.Y * PPP;
  p.X = X3;
  p.ZZ = p.ZZ * PP;
  p.ZZZ = p.ZZZ * PPP;
}

// p + q: add-2008-s with the exceptional cases
inline XYZZ xyzz_add(const XYZZ& p, const XYZZ& q) {
  if (xyzz_is_inf(p)) return q;
  if (xyzz_is_inf(q)) return p;
  fp U1 = p.X * q.ZZ, U2 = q.X * p.ZZ, S1 = p.Y * q.ZZZ, S2 = q.Y * p.ZZZ, P = U2 - U1, R = S2 - S1;
  if (is_zero(P)) return is_zero(R) ? xyzz_dbl(p) : xyzz_inf();
  fp PP = sqr(P), PPP = P * PP, Q = U1 * PP;
  XYZZ r;
  r.X = sqr(R) - PPP - Q - Q;
  r.Y = R * (Q - r.X) - S1 * PPP;
  r.ZZ = p.ZZ * q.ZZ * PP;
  r.ZZZ = p.ZZZ * q.ZZZ * PPP;
  return r;
}

// signed c-bit digit w of a little-endian 128-bit magnitude (carry in / out)
inline int32_t digit(const uint32_t k[4], uint32_t c, uint32_t w, uint32_t& carry) {
  uint32_t bit = w * c;
  uint32_t v = 0;
  for (uint32_t b = 0; b < c; b++) {
    uint32_t pos = bit + b;
    if (pos < 128) v |= ((k[pos >> 5] >> (pos & 31)) & 1u) << b;
  }
  int64_t d = (int64_t)v + carry;
  carry = 0;
  if (d > (int64_t)(1u << (c - 1))) {
    d -= (int64_t)1 << c;
    carry = 1;
  }
  return (int32_t)d;
}

uint32_t pick_c(uint64_t m) {  // points a task sees (2 per input point)
  uint32_t best = 4;
  double bc = 1e300;
  for (uint32_t c = 4; c <= 20; c++) {
    double W = (129.0 + c - 1) / c + 1;
    double cost = W * ((double)m + 2.0 * (double)(1u << (c - 1)) * 1.4);  // bucket adds + running sums
    if (cost < bc) bc = cost, best = c;
  }
  return best;
}

}  // namespace

// points: n x 64-byte RawBytes (canonical, on the curve); scalars: n x 32
// bytes big-endian (reduced mod r here).  out: the 64-byte RawBytes sum.  Returns 0,
// or -1 on a point that does not decode.
extern "C" int cpu_msm_pippenger(size_t n, const uint8_t* points, const uint8_t* scalars, int threads, uint32_t c,
                                 uint8_t out[64]) {
  if (threads < 1) threads = 1;
  std::vector<fp> px(n), py(n), bx(n);  // x, y, beta x (Montgomery)
  std::vector<int32_t> dig;
  std::vector<uint8_t> inf(n);
  std::atomic<int> bad{0};
  auto par = [&](size_t tasks, auto&& body) {
    std::atomic<size_t> next{0};
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++)
      th.emplace_back([&]() {
        for (size_t i; (i = next.fetch_add(1)) < tasks;) body(i);
      });
    for (auto& x : th) x.join();
  };
  // the task split: slices of the points so that windows x slices >= 2 x threads
  const uint32_t cc = c ? c : pick_c(2 * (uint64_t)n);
  const uint32_t W = (129 + cc - 1) / cc + 1;
  const size_t S = std::max<size_t>(1, std::min<size_t>(n, (2 * (size_t)threads + W - 1) / W));
  const uint32_t cfin = c ? c : pick_c(2 * (uint64_t)((n + S - 1) / S));
  const uint32_t Wf = (129 + cfin - 1) / cfin + 1;
  dig.assign((size_t)Wf * 2 * n, 0);
  const size_t PIECE = 4096;
  par((n + PIECE - 1) / PIECE, [&](size_t p) {
    for (size_t i = p * PIECE; i < n && i < (p + 1) * PIECE; i++) {
      uint32_t x[8], y[8], k[8];
      be32_to_limbs(x, points + 64 * i);
      be32_to_limbs(y, points + 64 * i + 32);
      g1a P;
      P.x = fe_from_int<ModP>(x);
      P.y = fe_from_int<ModP>(y);
      P.inf = is_zero(P.x) && is_zero(P.y);
      if (!g1_on_curve(P)) bad.store(1);
      inf[i] = P.inf;
      px[i] = P.x;
      py[i] = P.y;
      bx[i] = P.x * fe_const<ModP>(GLV_BETA);
      be32_to_limbs(k, scalars + 32 * i);
      fe_to_int(k, fe_from_int<ModR>(k));  // any 256-bit value, reduced mod r
      uint32_t k1[4], k2[4];
      bool n1, n2;
      glv_split(k, k1, n1, k2, n2);
      uint32_t c1 = 0, c2 = 0;
      for (uint32_t w = 0; w < Wf; w++) {
        int32_t d1 = digit(k1, cfin, w, c1), d2 = digit(k2, cfin, w, c2);
        dig[((size_t)w * n + i) * 2] = n1 ? -d1 : d1;
        dig[((size_t)w * n + i) * 2 + 1] = n2 ? -d2 : d2;
      }
    }
  });
  if (bad.load()) return -1;
  const size_t NB = (size_t)1 << (cfin - 1);
  std::vector<XYZZ> part((size_t)Wf * S, xyzz_inf());
  par((size_t)Wf * S, [&](size_t task) {
    const uint32_t w = (uint32_t)(task / S);
    const size_t s = task % S, a = n * s / S, b = n * (s + 1) / S;
    std::vector<XYZZ> bucket(NB, xyzz_inf());
    const int32_t* d = &dig[(size_t)w * 2 * n];
    for (size_t i = a; i < b; i++) {
      if (inf[i]) continue;
      for (int h = 0; h < 2; h++) {
        int32_t v = d[2 * i + h];
        if (!v) continue;
        const fp& x = h ? bx[i] : px[i];
        fp y = v < 0 ? fe_neg(py[i]) : py[i];
        xyzz_madd(bucket[(size_t)(v < 0 ? -v : v) - 1], x, y);
      }
    }
    XYZZ run = xyzz_inf(), sum = xyzz_inf();
    for (size_t k = NB; k-- > 0;) {
      run = xyzz_add(run, bucket[k]);
      sum = xyzz_add(sum, run);
    }
    part[task] = sum;
  });
  XYZZ acc = xyzz_inf();
  for (uint32_t w = Wf; w-- > 0;) {
    for (uint32_t q = 0; q < cfin; q++) acc = xyzz_dbl(acc);
    for (size_t s = 0; s < S; s++) acc = xyzz_add(acc, part[(size_t)w * S + s]);
  }
  g1a r;
  if (xyzz_is_inf(acc)) {
    r.inf = true;
  } else {
    fp zi = inv(acc.ZZ * acc.ZZZ);  // 1/(ZZ ZZZ): x = X ZZZ zi, y = Y ZZ zi
    r.x = acc.X * acc.ZZZ * zi;
    r.y = acc.Y * acc.ZZ * zi;
    r.inf = false;
  }
  g1_to_bytes(out, r);
  return 0;
}

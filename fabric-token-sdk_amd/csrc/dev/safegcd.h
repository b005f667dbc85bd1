// Variable-time modular inverse mod the BN254 base field p by Bernstein-Yang
// divsteps ("Fast constant-time gcd computation and modular inversion",
// ePrint 2019/266) in batches of 62, the variable-time variant with
// trailing-zero skipping and the 62-bit-limb signed representation that
// libsecp256k1's modinv64 uses [EXT: the algorithm, restated here; no
// reference file holds an inversion -- the reference's gnark-crypto inverts
// with a binary Euclid, and an inverse is unique, so any correct method gives
// its bytes].  For PUBLIC values only (the running time depends on the input).
//
// Why: the batched inversions (dev/binv.h) and the block inversions of
// k_g1_combine end in ONE inversion run by one lane, on the latency path of
// every pass; the 8 x 32-bit binary Euclid (fp_inv_eea) issues ~40k dependent
// instructions there.  Here ~10 rounds of 62 divsteps on 64-bit words plus a
// 2x2 matrix applied to 5-limb numbers.  tools/fpcheck.hip (ftz_invcheck,
// tests/test_gpu.py) compares it with fp_inv_eea on 262k values on the device;
// tests/test_safegcd.py (tests/native/sg_check.cpp) checks both limb layouts
// against Python on the host.
#pragma once
// (included by fp.h, after its FTS_HD definitions)
#include <stdint.h>

namespace fts {

struct Sg62 {
  int64_t v[5];  // value = sum v[i] 2^(62 i); limbs 0..3 in [0, 2^62) after normalisation
};
struct SgTrans {
  int64_t u, v, q, r;
};

static constexpr uint64_t SG_M62 = ~0ull >> 2;
// p in 62-bit limbs and p^-1 mod 2^62
FTS_HD Sg62 sg_modulus() { return {{0x3c208c16d87cfd47ll, 0x1e05aa45a1c72a34ll, 0x5045b68181585d9ll, 0x19139cb84c680a6ell, 0x30ll}}; }
static constexpr uint64_t SG_P_INV62 = 0x382df87d1b799c77ull;

FTS_HD int sg_ctz64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (int)__builtin_ctzll(x);
#else
  return __builtin_ctzll(x);
#endif
}

// 62 divsteps on the low words of f and g (f odd), variable time: runs of
// zero bits of g are skipped at once and up to 6 (eta < 0 after the swap) or
// 4 bits of g cancelled per step.  Returns the new eta.
FTS_HD int64_t sg_divsteps_62_var(int64_t eta, uint64_t f0, uint64_t g0, SgTrans& t) {
  uint64_t u = 1, v = 0, q = 0, r = 1;
  uint64_t f = f0, g = g0, m;
  uint32_t w;
  int i = 62, limit, zeros;
  for (;;) {
    zeros = sg_ctz64(g | (~0ull << i));  // a sentinel bit: at most i zeros
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    // f and g odd
    if (eta < 0) {
      uint64_t tmp;
      eta = -eta;
      tmp = f;
      f = g;
      g = 0 - tmp;
      tmp = u;
      u = q;
      q = 0 - tmp;
      tmp = v;
      v = r;
      r = 0 - tmp;
      limit = ((int)eta + 1) > i ? i : ((int)eta + 1);
      m = (~0ull >> (64 - limit)) & 63u;
      w = (uint32_t)((f * g * (f * f - 2)) & m);  // g + w f = 0 mod 2^min(limit, 6)
    } else {
      limit = ((int)eta + 1) > i ? i : ((int)eta + 1);
      m = (~0ull >> (64 - limit)) & 15u;
      w = (uint32_t)(f + (((f + 1) & 4) << 1));
      w = (uint32_t)((0 - (uint64_t)w * g) & m);  // g + w f = 0 mod 2^min(limit, 4)
    }
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t.u = (int64_t)u;
  t.v = (int64_t)v;
  t.q = (int64_t)q;
  t.r = (int64_t)r;
  return eta;
}

// [d, e] <- t [d, e] / 2^62 mod p (p multiples added so the low 62 bits vanish)
FTS_HD void sg_update_de(Sg62& d, Sg62& e, const SgTrans& t) {
  typedef __int128 i128;
  const Sg62 P = sg_modulus();
  const int64_t u = t.u, v = t.v, q = t.q, r = t.r;
  const int64_t sd = d.v[4] >> 63, se = e.v[4] >> 63;
  int64_t md = (u & sd) + (v & se), me = (q & sd) + (r & se);
  i128 cd = (i128)u * d.v[0] + (i128)v * e.v[0];
  i128 ce = (i128)q * d.v[0] + (i128)r * e.v[0];
  md -= (int64_t)((SG_P_INV62 * (uint64_t)(int64_t)cd + (uint64_t)md) & SG_M62);
  me -= (int64_t)((SG_P_INV62 * (uint64_t)(int64_t)ce + (uint64_t)me) & SG_M62);
  cd += (i128)P.v[0] * md;
  ce += (i128)P.v[0] * me;
  cd >>= 62;
  ce >>= 62;
#pragma unroll
  for (int k = 1; k < 5; k++) {
    cd += (i128)u * d.v[k] + (i128)v * e.v[k] + (i128)P.v[k] * md;
    ce += (i128)q * d.v[k] + (i128)r * e.v[k] + (i128)P.v[k] * me;
    d.v[k - 1] = (int64_t)((uint64_t)(int64_t)cd & SG_M62);
    e.v[k - 1] = (int64_t)((uint64_t)(int64_t)ce & SG_M62);
    cd >>= 62;
    ce >>= 62;
  }
  d.v[4] = (int64_t)cd;
  e.v[4] = (int64_t)ce;
}

// [f, g] <- t [f, g] / 2^62 over the first len limbs (exact division)
FTS_HD void sg_update_fg(int len, Sg62& f, Sg62& g, const SgTrans& t) {
  typedef __int128 i128;
  const int64_t u = t.u, v = t.v, q = t.q, r = t.r;
  i128 cf = (i128)u * f.v[0] + (i128)v * g.v[0];
  i128 cg = (i128)q * f.v[0] + (i128)r * g.v[0];
  cf >>= 62;
  cg >>= 62;
#pragma unroll
  for (int k = 1; k < 5; k++) {
    if (k < len) {
      cf += (i128)u * f.v[k] + (i128)v * g.v[k];
      cg += (i128)q * f.v[k] + (i128)r * g.v[k];
      f.v[k - 1] = (int64_t)((uint64_t)(int64_t)cf & SG_M62);
      g.v[k - 1] = (int64_t)((uint64_t)(int64_t)cg & SG_M62);
      cf >>= 62;
      cg >>= 62;
    }
  }
#pragma unroll
  for (int k = 1; k <= 5; k++)
    if (k == len) {
      f.v[k - 1] = (int64_t)cf;
      g.v[k - 1] = (int64_t)cg;
    }
}

// r * sign(f) reduced into [0, p): r in (-2p, p)
FTS_HD void sg_normalize(Sg62& r, int64_t sign) {
  const Sg62 P = sg_modulus();
  int64_t c = r.v[4] >> 63;
#pragma unroll
  for (int k = 0; k < 5; k++) r.v[k] += P.v[k] & c;
  const int64_t neg = sign >> 63;
#pragma unroll
  for (int k = 0; k < 5; k++) r.v[k] = (r.v[k] ^ neg) - neg;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    r.v[k + 1] += r.v[k] >> 62;
    r.v[k] &= (int64_t)SG_M62;
  }
  c = r.v[4] >> 63;
#pragma unroll
  for (int k = 0; k < 5; k++) r.v[k] += P.v[k] & c;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    r.v[k + 1] += r.v[k] >> 62;
    r.v[k] &= (int64_t)SG_M62;
  }
}

// x^-1 mod p for a plain integer 0 < x < p in 8 x 32-bit limbs (out likewise)
FTS_HD void sg_inv_int(const uint32_t x[8], uint32_t out[8]) {
  uint64_t w[4];
#pragma unroll
  for (int k = 0; k < 4; k++) w[k] = (uint64_t)x[2 * k] | ((uint64_t)x[2 * k + 1] << 32);
  Sg62 g = {{(int64_t)(w[0] & SG_M62), (int64_t)(((w[0] >> 62) | (w[1] << 2)) & SG_M62),
             (int64_t)(((w[1] >> 60) | (w[2] << 4)) & SG_M62), (int64_t)(((w[2] >> 58) | (w[3] << 6)) & SG_M62),
             (int64_t)(w[3] >> 56)}};
  Sg62 f = sg_modulus(), d = {{0, 0, 0, 0, 0}}, e = {{1, 0, 0, 0, 0}};
  int64_t eta = -1;
  int len = 5;
  for (;;) {
    SgTrans t;
    eta = sg_divsteps_62_var(eta, (uint64_t)f.v[0], (uint64_t)g.v[0], t);
    sg_update_de(d, e, t);
    sg_update_fg(len, f, g, t);
    if (g.v[0] == 0) {
      int64_t cond = 0;
#pragma unroll
      for (int k = 1; k < 5; k++)
        if (k < len) cond |= g.v[k];
      if (cond == 0) break;
    }
    // shorten f and g when both top limbs are 0 or -1
    int64_t fn = 0, gn = 0;
#pragma unroll
    for (int k = 0; k < 5; k++)
      if (k == len - 1) {
        fn = f.v[k];
        gn = g.v[k];
      }
    int64_t cond = ((int64_t)len - 2) >> 63;
    cond |= fn ^ (fn >> 63);
    cond |= gn ^ (gn >> 63);
    if (cond == 0) {
#pragma unroll
      for (int k = 0; k < 5; k++)
        if (k == len - 2) {
          f.v[k] |= (int64_t)((uint64_t)fn << 62);
          g.v[k] |= (int64_t)((uint64_t)gn << 62);
        }
      --len;
    }
  }
  int64_t fs = 0;  // f = +-1: its top limb carries the sign
#pragma unroll
  for (int k = 0; k < 5; k++)
    if (k == len - 1) fs = f.v[k];
  sg_normalize(d, fs);
  const uint64_t o0 = (uint64_t)d.v[0] | ((uint64_t)d.v[1] << 62), o1 = ((uint64_t)d.v[1] >> 2) | ((uint64_t)d.v[2] << 60),
                 o2 = ((uint64_t)d.v[2] >> 4) | ((uint64_t)d.v[3] << 58),
                 o3 = ((uint64_t)d.v[3] >> 6) | ((uint64_t)d.v[4] << 56);
  const uint64_t o[4] = {o0, o1, o2, o3};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    out[2 * k] = (uint32_t)o[k];
    out[2 * k + 1] = (uint32_t)(o[k] >> 32);
  }
}


// ---- the same with 30-bit limbs and 30-divstep batches (libsecp256k1's
// modinv32 layout): every product is 32 x 32 -> 64 bits (v_mad_i64_i32) and the
// divstep loop runs on 32-bit words, where the 62-bit form spends two VALU
// instructions on every 64-bit operation and emulates its 128-bit products.
struct Sg30 {
  int32_t v[9];
};
struct SgTrans30 {
  int32_t u, v, q, r;
};
static constexpr uint32_t SG_M30 = 0x3FFFFFFFu;
FTS_HD Sg30 sg30_modulus() {
  return {{0x187cfd47, 0x3082305b, 0x71ca8d3, 0x205aa45a, 0x1585d97, 0x116da06, 0x1a029b85, 0x139cb84c, 0x3064}};
}
static constexpr uint32_t SG_P_INV30 = 0x1b799c77u;

FTS_HD int32_t sg_divsteps_30_var(int32_t eta, uint32_t f0, uint32_t g0, SgTrans30& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  uint32_t f = f0, g = g0, m, w;
  int i = 30, limit, zeros;
  for (;;) {
    zeros = (int)__builtin_ctz(g | (~0u << i));  // a sentinel bit: at most i zeros
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    if (eta < 0) {
      uint32_t tmp;
      eta = -eta;
      tmp = f;
      f = g;
      g = 0u - tmp;
      tmp = u;
      u = q;
      q = 0u - tmp;
      tmp = v;
      v = r;
      r = 0u - tmp;
      limit = (eta + 1) > i ? i : (eta + 1);
      m = (~0u >> (32 - limit)) & 63u;
      w = (f * g * (f * f - 2)) & m;
    } else {
      limit = (eta + 1) > i ? i : (eta + 1);
      m = (~0u >> (32 - limit)) & 15u;
      w = f + (((f + 1) & 4) << 1);
      w = (0u - w * g) & m;
    }
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t.u = (int32_t)u;
  t.v = (int32_t)v;
  t.q = (int32_t)q;
  t.r = (int32_t)r;
  return eta;
}

FTS_HD void sg30_update_de(Sg30& d, Sg30& e, const SgTrans30& t) {
  const Sg30 P = sg30_modulus();
  const int32_t u = t.u, v = t.v, q = t.q, r = t.r;
  const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
  int32_t md = (u & sd) + (v & se), me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d.v[0] + (int64_t)v * e.v[0];
  int64_t ce = (int64_t)q * d.v[0] + (int64_t)r * e.v[0];
  md -= (int32_t)((SG_P_INV30 * (uint32_t)cd + (uint32_t)md) & SG_M30);
  me -= (int32_t)((SG_P_INV30 * (uint32_t)ce + (uint32_t)me) & SG_M30);
  cd += (int64_t)P.v[0] * md;
  ce += (int64_t)P.v[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int k = 1; k < 9; k++) {
    cd += (int64_t)u * d.v[k] + (int64_t)v * e.v[k] + (int64_t)P.v[k] * md;
    ce += (int64_t)q * d.v[k] + (int64_t)r * e.v[k] + (int64_t)P.v[k] * me;
    d.v[k - 1] = (int32_t)((uint32_t)cd & SG_M30);
    e.v[k - 1] = (int32_t)((uint32_t)ce & SG_M30);
    cd >>= 30;
    ce >>= 30;
  }
  d.v[8] = (int32_t)cd;
  e.v[8] = (int32_t)ce;
}

FTS_HD void sg30_update_fg(int len, Sg30& f, Sg30& g, const SgTrans30& t) {
  const int32_t u = t.u, v = t.v, q = t.q, r = t.r;
  int64_t cf = (int64_t)u * f.v[0] + (int64_t)v * g.v[0];
  int64_t cg = (int64_t)q * f.v[0] + (int64_t)r * g.v[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int k = 1; k < 9; k++) {
    if (k < len) {
      cf += (int64_t)u * f.v[k] + (int64_t)v * g.v[k];
      cg += (int64_t)q * f.v[k] + (int64_t)r * g.v[k];
      f.v[k - 1] = (int32_t)((uint32_t)cf & SG_M30);
      g.v[k - 1] = (int32_t)((uint32_t)cg & SG_M30);
      cf >>= 30;
      cg >>= 30;
    }
  }
#pragma unroll
  for (int k = 1; k <= 9; k++)
    if (k == len) {
      f.v[k - 1] = (int32_t)cf;
      g.v[k - 1] = (int32_t)cg;
    }
}

FTS_HD void sg30_normalize(Sg30& r, int32_t sign) {
  const Sg30 P = sg30_modulus();
  int32_t c = r.v[8] >> 31;
#pragma unroll
  for (int k = 0; k < 9; k++) r.v[k] += P.v[k] & c;
  const int32_t neg = sign >> 31;
#pragma unroll
  for (int k = 0; k < 9; k++) r.v[k] = (r.v[k] ^ neg) - neg;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    r.v[k + 1] += r.v[k] >> 30;
    r.v[k] &= (int32_t)SG_M30;
  }
  c = r.v[8] >> 31;
#pragma unroll
  for (int k = 0; k < 9; k++) r.v[k] += P.v[k] & c;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    r.v[k + 1] += r.v[k] >> 30;
    r.v[k] &= (int32_t)SG_M30;
  }
}

FTS_HD void sg30_inv_int(const uint32_t x[8], uint32_t out[8]) {
  Sg30 g;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const int b = 30 * k, l = b >> 5, o = b & 31;
    uint64_t lo = l < 8 ? x[l] : 0u, hi = l + 1 < 8 ? x[l + 1] : 0u;
    g.v[k] = (int32_t)((uint32_t)(((hi << 32) | lo) >> o) & SG_M30);
  }
  Sg30 f = sg30_modulus(), d = {{0, 0, 0, 0, 0, 0, 0, 0, 0}}, e = {{1, 0, 0, 0, 0, 0, 0, 0, 0}};
  int32_t eta = -1;
  int len = 9;
  for (;;) {
    SgTrans30 t;
    eta = sg_divsteps_30_var(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    sg30_update_de(d, e, t);
    sg30_update_fg(len, f, g, t);
    if (g.v[0] == 0) {
      int32_t cond = 0;
#pragma unroll
      for (int k = 1; k < 9; k++)
        if (k < len) cond |= g.v[k];
      if (cond == 0) break;
    }
    int32_t fn = 0, gn = 0;
#pragma unroll
    for (int k = 0; k < 9; k++)
      if (k == len - 1) {
        fn = f.v[k];
        gn = g.v[k];
      }
    int32_t cond = ((int32_t)len - 2) >> 31;
    cond |= fn ^ (fn >> 31);
    cond |= gn ^ (gn >> 31);
    if (cond == 0) {
#pragma unroll
      for (int k = 0; k < 9; k++)
        if (k == len - 2) {
          f.v[k] |= (int32_t)((uint32_t)fn << 30);
          g.v[k] |= (int32_t)((uint32_t)gn << 30);
        }
      --len;
    }
  }
  int32_t fs = 0;
#pragma unroll
  for (int k = 0; k < 9; k++)
    if (k == len - 1) fs = f.v[k];
  sg30_normalize(d, fs);
  // 9 x 30-bit limbs (the top one < 2^14 for d < p) -> 8 x 32
#pragma unroll
  for (int k = 0; k < 8; k++) out[k] = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const int b = 30 * k, l = b >> 5, o = b & 31;
    const uint64_t w = (uint64_t)(uint32_t)d.v[k] << o;
    out[l] |= (uint32_t)w;
    if (l + 1 < 8) out[l + 1] |= (uint32_t)(w >> 32);
  }
}

}  // namespace fts

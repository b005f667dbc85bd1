// Sextet layout for the pairing kernels: one pairing job per 6 lanes.
//
// Lane k (k = 0..5) of a sextet owns coefficient k of an Fp12 element in the
// w-power basis  f = sum_k f_k w^k,  f_k in Fp2,  w^6 = xi = 9 + u.  With
// gnark's tower (E12 = C0 + C1 w, E6 = B0 + B1 v + B2 v^2, v = w^2):
//   f_0 = C0.B0, f_1 = C1.B0, f_2 = C0.B1, f_3 = C1.B1, f_4 = C0.B2, f_5 = C1.B2.
// A product c = a*b is then  c_k = sum_i a_i b_(k-i)  with xi on the wrapped
// terms (i > k); lane k accumulates its six Fp2 products unreduced (dev/fp_wide.h)
// and Montgomery-reduces once.  Coefficients are exchanged through a small
// LDS region per sextet (Fp2 "slots"); the kernels run one wave per workgroup
// so the exchange barrier is a single-wave __syncthreads.
//
// Why: a 4096-transfer batch has only 16,384 pairing jobs; one job per lane
// leaves 3/4 of the SIMDs empty (256 waves), six lanes per job give 1,536
// waves at about the same total arithmetic (lazy reduction pays for the
// schoolbook product) and a small per-lane register footprint.
//
// Every routine computes exactly the same field values as the one-lane tower
// code (dev/tower.h, dev/pairing.h): same formulas, same line scaling, so the
// results are bit-identical (checked on the host by tests/native/sx_emu.cpp).
#pragma once
#include "fp29.h"
#include "fp_wide.h"
#include "pairing.h"

namespace fts {

#if defined(__HIP_DEVICE_COMPILE__)
#define FTS_LDS __attribute__((address_space(3)))
#else
#define FTS_LDS
#endif

struct alignas(16) F2Slot {
  uint32_t w[16];
};
typedef FTS_LDS F2Slot SlotT;  // slots live in LDS on the device

FTS_HD fp2 f2_sel(bool c, const fp2& a, const fp2& b) {  // c ? a : b
  fp2 r;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r.c0.v[i] = c ? a.c0.v[i] : b.c0.v[i];
    r.c1.v[i] = c ? a.c1.v[i] : b.c1.v[i];
  }
  return r;
}
// value of the lane's role among up to six register candidates
FTS_HD fp2 f2_pick(int k, const fp2& v0, const fp2& v1, const fp2& v2, const fp2& v3, const fp2& v4,
                   const fp2& v5) {
  fp2 r = v0;
  r = f2_sel(k == 1, v1, r);
  r = f2_sel(k == 2, v2, r);
  r = f2_sel(k == 3, v3, r);
  r = f2_sel(k == 4, v4, r);
  r = f2_sel(k == 5, v5, r);
  return r;
}
FTS_HD fp2 f2_of_fp(const fp& a) { return {a, fe_zero<ModP>()}; }

// Slot map of one sextet's LDS region.
enum : int {
  SX_A = 0,    // a_0..a_5   (published operand)
  SX_AX = 6,   // xi * a_0..a_5
  SX_P = 12,   // per-lane products
  SX_A2 = 12,  // 2 a_0..2 a_5 (sx_sqr only; aliases SX_P)
  SX_B = 18,   // b_0..b_5   (second operand of full products; final exponentiation)
  SX_BX = 24,  // xi * b_0..b_5
  SX_SLOTS_FEXP = 30,
  // Miller loop (shares SX_A, SX_AX, SX_P)
  SX_T = 18,   // running point T = (X, Y, Z) of pair 2
  SX_Q = 21,   // affine Q of the current addition step (x, y)
  SX_PC = 23,  // (yP2, xP2), (yP1, xP1) packed as Fp2 slots
  SX_L = 25,   // lines at P: pair 2 (l0, l1, l3), pair 1 (l0, l1, l3)
  SX_SLOTS_MILLER = 31,
  SX_SLOTS_MILLER_F = 18,  // f-chain only Miller loop (pair-2 lines precomputed)
};

// Sextet context, passed by value.  Sync is a callable barrier across the
// sextet (device: the one-wave workgroup's __syncthreads; host emulation: a
// 6-thread barrier).
template <class Sync>
struct Sx {
  int k;      // role 0..5
  SlotT* s;   // this sextet's slots
  bool wr;    // false for the ghost lanes 60..63 of a wave (read only)
  Sync sync;
  FTS_HD void put(int slot, const fp2& a) const {
    if (wr) {
#pragma unroll
      for (int i = 0; i < 8; i++) {
        s[slot].w[i] = a.c0.v[i];
        s[slot].w[8 + i] = a.c1.v[i];
      }
    }
  }
  FTS_HD fp2 get(int slot) const {
    fp2 a;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      a.c0.v[i] = s[slot].w[i];
      a.c1.v[i] = s[slot].w[8 + i];
    }
    return a;
  }
};

// A term of a lane's sum: a_ia * b_ib, optionally a doubled, b negated.
// Packed in 16 bits: ia (6) | ib (6) | dbl (1) | neg (1) | zero (1); a table
// row holds one term for each of the six lanes (4 x 16 bits + 2 x 16 bits).
enum : uint16_t { TM_DBL = 1u << 12, TM_NEG = 1u << 13, TM_ZERO = 1u << 14 };
#define SX_T(ia, ib, fl) (uint16_t)((ia) | ((ib) << 6) | (fl))
struct TermRow {
  uint64_t lo, hi;
};
constexpr TermRow term_row(uint16_t a, uint16_t b, uint16_t c, uint16_t d, uint16_t e, uint16_t f) {
  return {(uint64_t)a | ((uint64_t)b << 16) | ((uint64_t)c << 32) | ((uint64_t)d << 48),
          (uint64_t)e | ((uint64_t)f << 16)};
}
FTS_HD uint32_t term_at(const TermRow& r, int k) {
  return (uint32_t)((k < 4 ? (r.lo >> (16 * k)) : (r.hi >> (16 * (k - 4)))) & 0xFFFF);
}

template <class X>
FTS_HD void sx_term(const X& x, Wide2& w, uint32_t t) {
  fp2 a = x.get(t & 63);
  fp2 b = x.get((t >> 6) & 63);
  a = f2_sel((t & TM_DBL) != 0, f2_dbl(a), a);
  b = f2_sel((t & TM_NEG) != 0, f2_neg(b), b);
  a = f2_sel((t & TM_ZERO) != 0, f2_zero(), a);
  w2_mac(w, a, b);
}

// publish a lane value and its xi-multiple
template <class X>
FTS_HD void sx_pub(const X& x, int base, const fp2& v) {
  x.put(base + x.k, v);
  x.put(base + 6 + x.k, f2_mul_xi(v));
}

// ----------------------------------------------------------------- Fp12 ops
// c = a * b  (schoolbook over w, 6 lazily reduced Fp2 products per lane); b
// must already be published in SX_B / SX_BX (sx_mulv does both).
template <class X>
FTS_HD fp2 sx_mul(X x, fp2 a) {
  x.put(SX_A + x.k, a);
  x.sync();
  Wide2 w;
  w2_init(w);
#pragma nounroll
  for (int i = 0; i < 6; i++) {
    int j = x.k - i;
    int sb = j < 0 ? SX_BX + j + 6 : SX_B + j;
    w2_mac(w, x.get(SX_A + i), x.get(sb));
  }
  x.sync();
  return w2_reduce(w);
}
template <class X>
FTS_HD fp2 sx_mulv(const X& x, const fp2& a, const fp2& b) {
  sx_pub(x, SX_B, b);
  return sx_mul(x, a);
}

// c = a^2.  Term macros shared with the cyclotomic table below.
#define SQ_(i, j, wrap, dbl) SX_T(SX_A + (i), ((wrap) ? SX_AX : SX_A) + (j), (dbl) ? TM_DBL : 0)
#define SQZ SX_T(0, 0, TM_ZERO)

// Symmetric form with the doubled coefficients published (SX_A2): lane k
// sums a_i a_j over i + j = k (mod 6), i <= j, taking 2 a_i from SX_A2 for
// i < j and xi a_j from SX_AX for wrapped terms: 4 products on even lanes, 3
// (+ one zeroed) on odd lanes, no per-term selects but the last.
#define S4_(i, j) SX_T(i, j, 0)
static constexpr TermRow SX_SQR4_TAB[4] = {
    term_row(S4_(SX_A + 0, SX_A + 0), S4_(SX_A2 + 0, SX_A + 1), S4_(SX_A + 1, SX_A + 1), S4_(SX_A2 + 0, SX_A + 3),
             S4_(SX_A + 2, SX_A + 2), S4_(SX_A2 + 0, SX_A + 5)),
    term_row(S4_(SX_A + 3, SX_AX + 3), S4_(SX_A2 + 2, SX_AX + 5), S4_(SX_A2 + 0, SX_A + 2), S4_(SX_A2 + 1, SX_A + 2),
             S4_(SX_A2 + 0, SX_A + 4), S4_(SX_A2 + 1, SX_A + 4)),
    term_row(S4_(SX_A2 + 1, SX_AX + 5), S4_(SX_A2 + 3, SX_AX + 4), S4_(SX_A + 4, SX_AX + 4), S4_(SX_A2 + 4, SX_AX + 5),
             S4_(SX_A2 + 1, SX_A + 3), S4_(SX_A2 + 2, SX_A + 3)),
    term_row(S4_(SX_A2 + 2, SX_AX + 4), SX_T(0, 0, TM_ZERO), S4_(SX_A2 + 3, SX_AX + 5), SX_T(0, 0, TM_ZERO),
             S4_(SX_A + 5, SX_AX + 5), SX_T(0, 0, TM_ZERO)),
};
#undef S4_
template <class X>
FTS_HD fp2 sx_sqr(X x, fp2 a) {
  sx_pub(x, SX_A, a);
  x.put(SX_A2 + x.k, f2_dbl(a));
  x.sync();
  Wide2 w;
  w2_init(w);
#pragma nounroll
  for (int t = 0; t < 4; t++) {
    uint32_t e = term_at(SX_SQR4_TAB[t], x.k);
    fp2 u = x.get(e & 63);
    fp2 v = x.get((e >> 6) & 63);
    w2_mac(w, f2_sel((e & TM_ZERO) != 0, f2_zero(), u), v);
  }
  x.sync();
  return w2_reduce(w);
}

// Granger-Scott cyclotomic squaring (same formula as f12_cyclo_sqr):
//   even lanes k = 2m: z = 3 (a_m^2 + xi a_(m+3)^2) - 2 a_k
//   odd lanes:  z_1 = 3 * 2 a_5 (xi a_2) + 2 a_1, z_3 = 3 * 2 a_3 a_0 + 2 a_3, z_5 = 3 * 2 a_4 a_1 + 2 a_5
static constexpr TermRow SX_CYC_TAB[2] = {
    term_row(SQ_(0, 0, 0, 0), SQ_(5, 2, 1, 1), SQ_(1, 1, 0, 0), SQ_(3, 0, 0, 1), SQ_(2, 2, 0, 0), SQ_(4, 1, 0, 1)),
    term_row(SQ_(3, 3, 1, 0), SQZ, SQ_(4, 4, 1, 0), SQZ, SQ_(5, 5, 1, 0), SQZ),
};
#undef SQ_
#undef SQZ

template <class X>
FTS_HD fp2 sx_cyc_sqr(X x, fp2 a) {
  const int k = x.k, m = k >> 1;
  sx_pub(x, SX_A, a);
  x.sync();
  // even k = 2m: a_m * a_m + a_(m+3) * (xi a_(m+3));  odd: one product
  // k=1: a_5 (xi a_2), k=3: a_3 a_0, k=5: a_4 a_1 (the factor 2 goes into the final 6r)
  bool odd = (k & 1) != 0;
  int i1 = odd ? (k == 1 ? 5 : (k == 3 ? 3 : 4)) : m;
  int j1 = odd ? (k == 1 ? SX_AX + 2 : (k == 3 ? SX_A + 0 : SX_A + 1)) : SX_A + m;
  Wide2 w;
  w2_init(w);
#pragma nounroll
  for (int t = 0; t < 2; t++) {
    fp2 u = x.get(t == 0 ? SX_A + i1 : SX_A + m + 3);
    fp2 v = x.get(t == 0 ? j1 : SX_AX + m + 3);
    w2_mac(w, f2_sel(odd && t == 1, f2_zero(), u), v);
  }
  x.sync();
  fp2 r = w2_reduce(w);
  fp2 r3 = f2_dbl(r) + r;
  fp2 ad = f2_dbl(a);
  return f2_sel(odd, f2_dbl(r3) + ad, r3 - ad);
}

// f * l with l = l0 + l1 w + l3 w^3 (gnark MulBy034 shape), l in slots lb..lb+2
template <class X>
FTS_HD fp2 sx_mul_line(X x, fp2 f, int lb) {
  sx_pub(x, SX_A, f);
  x.sync();
  Wide2 w;
  w2_init(w);
#pragma nounroll
  for (int t = 0; t < 3; t++) {
    int j = x.k - (t == 0 ? 0 : (t == 1 ? 1 : 3));
    int sb = j < 0 ? SX_AX + j + 6 : SX_A + j;
    w2_mac(w, x.get(lb + t), x.get(sb));
  }
  x.sync();
  return w2_reduce(w);
}

FTS_HD fp2 sx_conj(int k, const fp2& a) { return f2_sel((k & 1) != 0, f2_neg(a), a); }

// Frobenius maps: coefficient k scaled by gamma_(n,k) (after conjugation for odd n)
FTS_HD fp2 sx_frob1(int k, const fp2& a) { return f2_conj(a) * f2_const(FROB1[k]); }
FTS_HD fp2 sx_frob2(int k, const fp2& a) { return f2_mul_fp(a, fe_const<ModP>(FROB2[k][0])); }
FTS_HD fp2 sx_frob3(int k, const fp2& a) { return f2_conj(a) * f2_const(FROB3[k]); }

static constexpr TermRow SX_INV_TAB[2] = {
    term_row(SX_T(SX_A + 0, SX_A + 0, 0), SX_T(SX_A + 4, SX_AX + 4, 0), SX_T(SX_A + 2, SX_A + 2, 0),
             SX_T(0, 0, TM_ZERO), SX_T(0, 0, TM_ZERO), SX_T(0, 0, TM_ZERO)),
    term_row(SX_T(SX_A + 2, SX_AX + 4, TM_NEG), SX_T(SX_A + 0, SX_A + 2, TM_NEG), SX_T(SX_A + 0, SX_A + 4, TM_NEG),
             SX_T(0, 0, TM_ZERO), SX_T(0, 0, TM_ZERO), SX_T(0, 0, TM_ZERO)),
};

// f^-1 (same value as f12_inv): den = f conj(f) = c0^2 - v c1^2 in Fp6 (even lanes);
// Fp6 inverse by the f6_inv formula; f^-1 = conj(f) * den^-1.
template <class X>
FTS_HD fp2 sx_inv(X x, fp2 f) {
  fp2 fc = sx_conj(x.k, f);
  fp2 d = sx_mulv(x, fc, f);  // lanes 0, 2, 4: d0, d1, d2 (Fp6 over v); odd lanes 0
  sx_pub(x, SX_A, d);
  x.sync();
  // t0 = d0^2 - xi d1 d2, t1 = xi d2^2 - d0 d1, t2 = d1^2 - d0 d2 (lanes 0..2)
  Wide2 w;
  w2_init(w);
#pragma nounroll
  for (int t = 0; t < 2; t++) sx_term(x, w, term_at(SX_INV_TAB[t], x.k));
  fp2 t = w2_reduce(w);
  x.put(SX_P + x.k, t);
  x.sync();
  // den6 = d0 t0 + xi d2 t1 + xi d1 t2  (every lane)
  Wide2 v;
  w2_init(v);
#pragma nounroll
  for (int t = 0; t < 3; t++) w2_mac(v, x.get(t == 0 ? SX_A + 0 : (t == 1 ? SX_AX + 4 : SX_AX + 2)), x.get(SX_P + t));
  fp2 tk = x.get(SX_P + (x.k >> 1));
  x.sync();
  fp2 di = f2_inv(w2_reduce(v));
  fp2 inv6 = f2_sel((x.k & 1) == 0, tk * di, f2_zero());  // coefficient of v^(k/2) = w^k
  return sx_mulv(x, fc, inv6);
}

// Width-4 NAF of the BN parameter x: digits in {+-1, +-3, +-5, +-7}, 14 non-zero
// over bits 62..0 (the binary NAF used by f12_expt has 24), top digit +1 at bit
// 62.  Masks: any non-zero digit, negative digits, magnitude 3 / 5 / 7.
static constexpr uint64_t BN_X_W4_NZ = 0x4108844442110211ull;
static constexpr uint64_t BN_X_W4_NEG = 0x0008004400010010ull;
static constexpr uint64_t BN_X_W4_M3 = 0x0008800400000000ull;
static constexpr uint64_t BN_X_W4_M5 = 0x0100044002000200ull;
static constexpr uint64_t BN_X_W4_M7 = 0x0000000000110000ull;

// a^x (x = BN parameter), a in the cyclotomic subgroup: the same element as
// f12_expt (any addition chain for x gives it), by the width-4 NAF with a^3,
// a^5, a^7 precomputed -- 13 + 3 multiplications and one extra squaring
// instead of 23 multiplications.  The digit's odd power (a^7 kept in LDS to
// stay within the register budget) is published in
// SX_B / SX_BX when its magnitude changes; a digit -d multiplies by
// conj(a^d) = a^-d through r conj(a^d) = conj(conj(r) a^d).
template <class X>
FTS_HD fp2 sx_expt(X x, fp2 a) {
  fp2 a2 = sx_cyc_sqr(x, a);
  fp2 a3 = sx_mulv(x, a2, a);
  fp2 a5 = sx_mulv(x, a3, a2);  // publishes a^2 for a^7 too
  x.put(SX_P + x.k, sx_mul(x, a5));  // a^7 parked in the lane's own SX_P slot (free during expt)
  int cur = 0;  // magnitude published in SX_B (0: a^2)
  fp2 r = a;
#pragma nounroll
  for (int i = 61; i >= 0; i--) {
    r = sx_cyc_sqr(x, r);
    if ((BN_X_W4_NZ >> i) & 1) {
      int m = ((BN_X_W4_M3 >> i) & 1) ? 3 : (((BN_X_W4_M5 >> i) & 1) ? 5 : (((BN_X_W4_M7 >> i) & 1) ? 7 : 1));
      if (m != cur) {
        sx_pub(x, SX_B, m == 7 ? x.get(SX_P + x.k) : (m == 1 ? a : (m == 3 ? a3 : a5)));
        cur = m;
      }
      bool neg = (BN_X_W4_NEG >> i) & 1;
      fp2 t = neg ? sx_conj(x.k, r) : r;
      t = sx_mul(x, t);
      r = neg ? sx_conj(x.k, t) : t;
    }
  }
  return r;
}

// final exponentiation (same sequence as final_exp).  The three x-powers run
// as one loop so the expt body is emitted once.
template <class X>
FTS_HD fp2 sx_final_exp(const X& x, const fp2& f) {
  const int k = x.k;
  fp2 t = sx_mulv(x, sx_conj(k, f), sx_inv(x, f));
  t = sx_mulv(x, sx_frob2(k, t), t);
  fp2 in = t, a2, a6, b, c;
#pragma nounroll
  for (int e = 0; e < 3; e++) {
    fp2 r = sx_expt(x, in);
    if (e == 0) {  // a = t^x, a2 = a^2, a6 = a2^3
      a2 = sx_cyc_sqr(x, r);
      a6 = sx_mulv(x, sx_cyc_sqr(x, a2), a2);
      in = a6;
    } else if (e == 1) {  // b = a6^x, then c = (b^2)^x
      b = r;
      in = sx_cyc_sqr(x, b);
    } else {
      c = r;
    }
  }
  fp2 A = sx_mulv(x, sx_mulv(x, a6, b), c);
  fp2 B = sx_mulv(x, A, sx_conj(k, a2));
  fp2 res = sx_frob2(k, A);
  res = sx_mulv(x, res, sx_mulv(x, sx_mulv(x, A, b), t));
  res = sx_mulv(x, res, sx_frob1(k, B));
  res = sx_mulv(x, res, sx_frob3(k, sx_mulv(x, B, sx_conj(k, t))));
  return res;
}

// Exact final exponentiation (f^((p^12-1)/r), Scott et al. chain as
// final_exp_exact in pairing.h).  The three x-powers run as one loop; the
// y_i are formed as soon as their inputs exist so at most six Fp12 values
// (one Fp2 per lane each) are live.
template <class X>
FTS_HD fp2 sx_final_exp_exact(const X& x, const fp2& f) {
  const int k = x.k;
  fp2 m = sx_mulv(x, sx_conj(k, f), sx_inv(x, f));
  m = sx_mulv(x, sx_frob2(k, m), m);
  fp2 in = m, mx, mx2, mx3;
#pragma nounroll
  for (int e = 0; e < 3; e++) {
    fp2 r = sx_expt(x, in);
    if (e == 0) {
      mx = r;
    } else if (e == 1) {
      mx2 = r;
    } else {
      mx3 = r;
    }
    in = r;
  }
  fp2 y3 = sx_conj(k, sx_frob1(k, mx));
  fp2 y4 = sx_conj(k, sx_mulv(x, mx, sx_frob1(k, mx2)));
  fp2 y5 = sx_conj(k, mx2);
  fp2 y2 = sx_frob2(k, mx2);
  fp2 y6 = sx_conj(k, sx_mulv(x, mx3, sx_frob1(k, mx3)));
  fp2 t0 = sx_mulv(x, sx_mulv(x, sx_cyc_sqr(x, y6), y4), y5);
  fp2 t1 = sx_mulv(x, sx_mulv(x, y3, y5), t0);
  t0 = sx_mulv(x, t0, y2);
  t1 = sx_cyc_sqr(x, sx_mulv(x, sx_cyc_sqr(x, t1), t0));
  fp2 y0 = sx_mulv(x, sx_mulv(x, sx_frob1(k, m), sx_frob2(k, m)), sx_frob3(k, m));
  t0 = sx_mulv(x, t1, sx_conj(k, m));
  t1 = sx_mulv(x, t1, y0);
  return sx_mulv(x, sx_cyc_sqr(x, t0), t1);
}

// gnark E12.Bytes position (in 64-byte Fp2 units) of coefficient k:
// C1.B2 (f5), C1.B1 (f3), C1.B0 (f1), C0.B2 (f4), C0.B1 (f2), C0.B0 (f0)
FTS_HD int sx_gt_pos(int k) { return (int)((0x031425u >> (4 * k)) & 0xF); }

FTS_HD void sx_gt_bytes(uint8_t* out, int k, const fp2& a) {
  uint32_t t[8];
  uint8_t* o = out + 64 * sx_gt_pos(k);
  fe_to_int(t, a.c1);
  limbs_to_be32(o, t);
  fe_to_int(t, a.c0);
  limbs_to_be32(o + 32, t);
}

// Evaluated lines of pair 2: l = c0 + c3 w + c4 w^3, in the balanced 29-bit
// form of dev/fp29.h (the operand format of the carry-free Miller kernel,
// dev/sx29.h sq_miller_f).  Component planes: component c = 2 m + part (part 0:
// c0 limbs, 1: c1 limbs) of line s of job idx is a 10-word record (9 limbs and
// a zero pad, 8-byte aligned) at ((s * 6 + c) * njobs + idx) * 10, so that the
// ten sextets of a wave, which handle consecutive jobs, write and read each
// plane contiguously.  Writers: evline_store (one lane) and sx_job_g2lines
// (lane k writes component k); same bytes either way.  EvLineDev is the size
// of one (line, job).
static constexpr uint32_t EVL_REC = 10;
struct EvLineDev {
  int32_t w[6 * EVL_REC];
};
FTS_HD size_t evl_off(uint32_t s, int c, uint32_t idx, uint32_t njobs) {
  return (((size_t)s * 6 + c) * njobs + idx) * EVL_REC;
}
FTS_HD void evline_put(EvLineDev* base, uint32_t s, int c, uint32_t idx, uint32_t njobs, const fp& v) {
  f29 b = f29_breduce(f29_from_fp(v));
  int32_t* o = (int32_t*)base + evl_off(s, c, idx, njobs);
#pragma unroll
  for (int i = 0; i < 9; i++) o[i] = b.l[i];
  o[9] = 0;
}
FTS_HD void evline_store(EvLineDev* base, uint32_t s, uint32_t idx, uint32_t njobs, const fp2& c0, const fp2& c3,
                         const fp2& c4) {
  const fp2* v[3] = {&c0, &c3, &c4};
#pragma unroll
  for (int m = 0; m < 3; m++) {
    evline_put(base, s, 2 * m, idx, njobs, v[m]->c0);
    evline_put(base, s, 2 * m + 1, idx, njobs, v[m]->c1);
  }
}
FTS_HD q2 evline_ld29(const EvLineDev* base, uint32_t s, int m, uint32_t idx, uint32_t njobs) {
  const int32_t* a0 = (const int32_t*)base + evl_off(s, 2 * m, idx, njobs);
  const int32_t* a1 = (const int32_t*)base + evl_off(s, 2 * m + 1, idx, njobs);
  q2 a;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    a.c0.l[i] = a0[i];
    a.c1.l[i] = a1[i];
  }
  return a;
}
FTS_HD fp2 evline_ld(const EvLineDev* base, uint32_t s, int m, uint32_t idx, uint32_t njobs) {
  return q2_to_fp2(evline_ld29(base, s, m, idx, njobs));
}

// ----------------------------------------------------------------- Miller loop
// State of pair 2 (T, Q, P2) and the evaluated lines live in LDS slots so the
// step functions take only the context.  A step runs "layers" of one reduced
// Fp2 product per lane (lane-selected operands), published to SX_P.
template <class X>
FTS_HD void sx_prod(const X& x, const fp2& a, const fp2& b) {
  x.put(SX_P + x.k, a * b);
  x.sync();
}

// write the six evaluated lines (lane k writes line slot k); a pair whose flag
// in `use` (bit 0: pair 2, bit 1: pair 1) is clear gets the line 1.
template <class X>
FTS_HD void sx_put_lines(const X& x, int use, const fp2& a0, const fp2& a1, const fp2& a3, const fp2& b0,
                         const fp2& b1, const fp2& b3) {
  const int k = x.k;
  bool on = (k < 3) ? (use & 1) != 0 : (use & 2) != 0;
  fp2 l = f2_pick(k, a0, a1, a3, b0, b1, b3);
  fp2 id = f2_sel(k == 0 || k == 3, f2_one(), f2_zero());
  x.put(SX_L + k, f2_sel(on, l, id));
}

// Doubling step T <- 2T (homogeneous projective, same formulas as dbl_step);
// lines: tangent at T evaluated at P2, fixed line lq evaluated at P1.
template <class X>
FTS_HD void sx_dbl_step(X x, const LineCoef* lq, int use) {
  const int k = x.k;
  fp2 TX = x.get(SX_T + 0), TY = x.get(SX_T + 1), TZ = x.get(SX_T + 2);
  fp2 pc2 = x.get(SX_PC + 0), pc1 = x.get(SX_PC + 1);
  fp2 YZ = TY + TZ;
  // layer 1: XY, Y^2, Z^2, (Y+Z)^2, X^2
  sx_prod(x, f2_pick(k, TX, TY, TZ, YZ, TX, TX), f2_pick(k, TY, TY, TZ, YZ, TX, TX));
  fp2 XY = x.get(SX_P + 0), B = x.get(SX_P + 1), C = x.get(SX_P + 2), YZ2 = x.get(SX_P + 3), J = x.get(SX_P + 4);
  x.sync();
  fp2 A = f2_half(XY);
  fp2 H = YZ2 - (B + C);
  fp2 C3 = C + C + C;
  fp2 J3 = J + J + J;
  LineCoef q = *lq;
  // layer 2: E = 3C b', lines: -H yP2, 3J xP2, r0 yP1, r1 xP1
  sx_prod(x, f2_pick(k, C3, f2_neg(H), J3, q.r0, q.r1, C3),
          f2_pick(k, f2_const(TWIST_B), f2_of_fp(pc2.c0), f2_of_fp(pc2.c1), f2_of_fp(pc1.c0), f2_of_fp(pc1.c1),
                  f2_const(TWIST_B)));
  fp2 E = x.get(SX_P + 0), a0 = x.get(SX_P + 1), a1 = x.get(SX_P + 2), b0 = x.get(SX_P + 3), b1 = x.get(SX_P + 4);
  x.sync();
  fp2 F = E + E + E;
  fp2 G = f2_half(B + F);
  sx_put_lines(x, use, a0, a1, E - B, b0, b1, q.r2);
  // layer 3: X3 = A (B - F), G^2, E^2, Z3 = B H
  sx_prod(x, f2_pick(k, A, G, E, B, A, A), f2_pick(k, B - F, G, E, H, B - F, B - F));
  fp2 X3 = x.get(SX_P + 0), G2 = x.get(SX_P + 1), EE = x.get(SX_P + 2), Z3 = x.get(SX_P + 3);
  x.sync();
  x.put(SX_T + (k < 3 ? k : 0), f2_pick(k, X3, G2 - (EE + EE + EE), Z3, X3, X3, X3));
  x.sync();
}

// Addition step T <- T + Q (Q affine from SX_Q, negated if neg; same formulas
// as add_step); lines: chord evaluated at P2, fixed line lq evaluated at P1.
template <class X>
FTS_HD void sx_add_step(X x, const LineCoef* lq, int use, int neg) {
  const int k = x.k;
  fp2 TX = x.get(SX_T + 0), TY = x.get(SX_T + 1), TZ = x.get(SX_T + 2);
  fp2 Qx = x.get(SX_Q + 0), Qy = x.get(SX_Q + 1);
  fp2 pc2 = x.get(SX_PC + 0), pc1 = x.get(SX_PC + 1);
  Qy = f2_sel(neg != 0, f2_neg(Qy), Qy);
  LineCoef q = *lq;
  // layer 1: Qy Z, Qx Z, pair-1 line r0 yP1, r1 xP1
  sx_prod(x, f2_pick(k, Qy, Qx, q.r0, q.r1, Qy, Qy), f2_pick(k, TZ, TZ, f2_of_fp(pc1.c0), f2_of_fp(pc1.c1), TZ, TZ));
  fp2 O = TY - x.get(SX_P + 0);
  fp2 Lc = TX - x.get(SX_P + 1);
  fp2 b0 = x.get(SX_P + 2), b1 = x.get(SX_P + 3);
  x.sync();
  // layer 2: O^2, L^2, Qx O, L Qy, L yP2, -O xP2
  fp2 On = f2_neg(O);
  sx_prod(x, f2_pick(k, O, Lc, Qx, Lc, Lc, On), f2_pick(k, O, Lc, O, Qy, f2_of_fp(pc2.c0), f2_of_fp(pc2.c1)));
  fp2 Cc = x.get(SX_P + 0), D = x.get(SX_P + 1);
  fp2 a3 = x.get(SX_P + 2) - x.get(SX_P + 3);
  fp2 a0 = x.get(SX_P + 4), a1 = x.get(SX_P + 5);
  x.sync();
  sx_put_lines(x, use, a0, a1, a3, b0, b1, q.r2);
  // layer 3: E = L D, F = Z C, G = X D
  sx_prod(x, f2_pick(k, Lc, TZ, TX, Lc, Lc, Lc), f2_pick(k, D, Cc, D, D, D, D));
  fp2 E = x.get(SX_P + 0), F = x.get(SX_P + 1), G = x.get(SX_P + 2);
  x.sync();
  fp2 H = E + F - (G + G);
  fp2 GH = G - H;
  // layer 4: t1 = Y E, X3 = L H, (G - H) O, Z3 = E Z
  sx_prod(x, f2_pick(k, TY, Lc, GH, E, E, E), f2_pick(k, E, H, O, TZ, TZ, TZ));
  fp2 t1 = x.get(SX_P + 0), X3 = x.get(SX_P + 1), GO = x.get(SX_P + 2), Z3 = x.get(SX_P + 3);
  x.sync();
  x.put(SX_T + (k < 3 ? k : 0), f2_pick(k, X3, GO - t1, Z3, X3, X3, X3));
  x.sync();
}

// 2-pair Miller loop f(P1, Qfix) * f(P2, Q2) (same as miller_2): qlines are the
// precomputed lines of the fixed Q (uniform across lanes).
template <class X>
FTS_HD fp2 sx_miller_2(const X& x, const LineCoef* qlines, const g1a& P1, const g1a& P2, const g2a& Q2) {
  const int k = x.k;
  int use = (!(P2.inf || Q2.inf) ? 1 : 0) | (!P1.inf ? 2 : 0);
  // initial slots: T = (Qx, Qy, 1), Q, P coordinates
  x.put(SX_T + (k < 3 ? k : 0), f2_pick(k, Q2.x, Q2.y, f2_one(), Q2.x, Q2.x, Q2.x));
  x.put(SX_Q + (k & 1), f2_sel((k & 1) == 0, Q2.x, Q2.y));
  x.put(SX_PC + (k & 1), f2_sel((k & 1) == 0, fp2{P2.y, P2.x}, fp2{P1.y, P1.x}));
  x.sync();
  fp2 f = f2_sel(k == 0, f2_one(), f2_zero());
  int n = 0;
#pragma nounroll
  for (int i = 64; i >= 0; i--) {
    if (i != 64) f = sx_sqr(x, f);
    sx_dbl_step(x, qlines + n, use);
    n++;
    f = sx_mul_line(x, f, SX_L + 3);
    f = sx_mul_line(x, f, SX_L + 0);
    int d = naf_digit(i);
    if (d != 0) {
      sx_add_step(x, qlines + n, use, d < 0);
      n++;
      f = sx_mul_line(x, f, SX_L + 3);
      f = sx_mul_line(x, f, SX_L + 0);
    }
  }
  // the two Frobenius lines: Q <- pi(Q2), then -pi^2(Q2)
#pragma nounroll
  for (int e = 0; e < 2; e++) {
    g2a Qf = e == 0 ? tw_frob(Q2) : tw_frob2_neg(Q2);
    x.put(SX_Q + (k & 1), f2_sel((k & 1) == 0, Qf.x, Qf.y));
    x.sync();
    sx_add_step(x, qlines + n + e, use, 0);
    f = sx_mul_line(x, f, SX_L + 3);
    f = sx_mul_line(x, f, SX_L + 0);
  }
  return f;
}

// f * l, l = l0 + l1 w + l3 w^3 held in registers of every lane
template <class X>
FTS_HD fp2 sx_mul_line_r(const X& x, const fp2& f, const fp2& l0, const fp2& l1, const fp2& l3) {
  sx_pub(x, SX_A, f);
  x.sync();
  Wide2 w;
  w2_init(w);
#pragma nounroll
  for (int t = 0; t < 3; t++) {
    int j = x.k - (t == 0 ? 0 : (t == 1 ? 1 : 3));
    int sb = j < 0 ? SX_AX + j + 6 : SX_A + j;
    w2_mac(w, t == 0 ? l0 : (t == 1 ? l1 : l3), x.get(sb));
  }
  x.sync();
  return w2_reduce(w);
}

// f <- f * (line lq of the fixed Q evaluated at P1): lanes 0..3 compute the
// four Fp products r0.c0 yP, r0.c1 yP, r1.c0 xP, r1.c1 xP and exchange them.
// A pair-1 point at infinity contributes 1.
template <class X>
FTS_HD fp2 sx_fixed_line(const X& x, const fp2& f, const LineCoef* lq, const g1a& P1) {
  const int k = x.k;
  const LineCoef& q = *lq;
  fp a = (k == 0) ? q.r0.c0 : (k == 1) ? q.r0.c1 : (k == 2) ? q.r1.c0 : q.r1.c1;
  fp b = (k < 2) ? P1.y : P1.x;
  x.put(SX_P + k, f2_of_fp(a * b));
  x.sync();
  fp2 l0 = {x.get(SX_P + 0).c0, x.get(SX_P + 1).c0};
  fp2 l1 = {x.get(SX_P + 2).c0, x.get(SX_P + 3).c0};
  fp2 l3 = q.r2;
  l0 = f2_sel(P1.inf, f2_one(), l0);
  l1 = f2_sel(P1.inf, f2_zero(), l1);
  l3 = f2_sel(P1.inf, f2_zero(), l3);
  return sx_mul_line_r(x, f, l0, l1, l3);
}

// Which of the MILLER_LINES lines is preceded by a squaring of f: the first
// line of every loop iteration i < 64 (miller_2 order).
struct SqrMask {
  uint64_t lo, hi;
};
constexpr SqrMask miller_sqr_mask() {
  SqrMask m{0, 0};
  int n = 0;
  for (int i = 64; i >= 0; i--) {
    if (i != 64) {
      if (n < 64)
        m.lo |= 1ull << n;
      else
        m.hi |= 1ull << (n - 64);
    }
    n += 1 + ((i < 64 && (((ATE_NAF_POS >> i) & 1) || ((ATE_NAF_NEG >> i) & 1))) ? 1 : 0);
  }
  return m;
}
static constexpr SqrMask MILLER_SQR = miller_sqr_mask();

// 2-pair Miller loop with pair 2's lines precomputed per job (job_g2lines,
// layout [line][job]): same factors, same order as miller_2.
template <class X>
FTS_HD fp2 sx_miller_f(const X& x, const LineCoef* qlines, const g1a& P1, const EvLineDev* l2, uint32_t idx,
                       uint32_t njobs) {
  fp2 f = f2_sel(x.k == 0, f2_one(), f2_zero());
#pragma nounroll
  for (int s = 0; s < MILLER_LINES; s++) {
    bool sq = s < 64 ? ((MILLER_SQR.lo >> s) & 1) : ((MILLER_SQR.hi >> (s - 64)) & 1);
    if (sq) f = sx_sqr(x, f);
    f = sx_fixed_line(x, f, qlines + s, P1);
    f = sx_mul_line_r(x, f, evline_ld(l2, s, 0, idx, njobs), evline_ld(l2, s, 1, idx, njobs),
                      evline_ld(l2, s, 2, idx, njobs));
  }
  return f;
}

// Fp12 <-> sextet coefficient k (w-power basis)
FTS_HD fp2 f12_coef(const fp12& f, int k) {
  return f2_pick(k, f.c0.c0, f.c1.c0, f.c0.c1, f.c1.c1, f.c0.c2, f.c1.c2);
}

}  // namespace fts

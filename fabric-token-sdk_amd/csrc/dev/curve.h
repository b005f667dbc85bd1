// G1 (E: y^2 = x^3 + 3 over Fp) and G2 (twist E': y^2 = x^3 + 3/(9+u) over Fp2)
// group law in Jacobian coordinates, written once over the coordinate field.
// Replaces mathlib G1/G2 Add/Sub/Mul (gnark G1Jac/G2Jac) -- SURVEY Appendix C.2.
#pragma once
#include "tower.h"

namespace fts {

// field-generic helpers ------------------------------------------------------
FTS_HD fp sqr(const fp& a) { return fe_sqr(a); }
FTS_HD fp2 sqr(const fp2& a) { return f2_sqr(a); }
FTS_HD fp neg(const fp& a) { return fe_neg(a); }
FTS_HD fp2 neg(const fp2& a) { return f2_neg(a); }
FTS_HD bool is_zero(const fp& a) { return fe_is_zero(a); }
FTS_HD bool is_zero(const fp2& a) { return f2_is_zero(a); }
FTS_HD bool eqf(const fp& a, const fp& b) { return fe_eq(a, b); }
FTS_HD bool eqf(const fp2& a, const fp2& b) { return f2_eq(a, b); }
FTS_HD fp inv(const fp& a) { return fp_inv_var(a); }  // variable time: public values only
FTS_HD fp2 inv(const fp2& a) { return f2_inv(a); }
template <class F> FTS_HD F zero_of();
template <> FTS_HD fp zero_of<fp>() { return fe_zero<ModP>(); }
template <> FTS_HD fp2 zero_of<fp2>() { return f2_zero(); }
template <class F> FTS_HD F one_of();
template <> FTS_HD fp one_of<fp>() { return fe_one<ModP>(); }
template <> FTS_HD fp2 one_of<fp2>() { return f2_one(); }

template <class F>
struct Aff {
  F x, y;
  bool inf;
};
template <class F>
struct Jac {
  F x, y, z;  // z == 0 <=> point at infinity
};

typedef Aff<fp> g1a;
typedef Jac<fp> g1j;
typedef Aff<fp2> g2a;
typedef Jac<fp2> g2j;

template <class F>
FTS_HD Jac<F> jac_inf() {
  return {one_of<F>(), one_of<F>(), zero_of<F>()};
}

template <class F>
FTS_HD Jac<F> jac_from_aff(const Aff<F>& a) {
  if (a.inf) return jac_inf<F>();
  return {a.x, a.y, one_of<F>()};
}

template <class F>
FTS_HD Aff<F> aff_neg(const Aff<F>& a) {
  return {a.x, neg(a.y), a.inf};
}

template <class F>
FTS_HD Jac<F> jac_neg(const Jac<F>& a) {
  return {a.x, neg(a.y), a.z};
}

// dbl-2009-l (a = 0): 2M + 5S
template <class F>
FTS_HD Jac<F> jac_dbl(const Jac<F>& p) {
  F A = sqr(p.x);
  F B = sqr(p.y);
  F C = sqr(B);
  F t = p.x + B;
  F D = sqr(t) - A - C;
  D = D + D;
  F E = A + A + A;
  F Fq = sqr(E);
  F X3 = Fq - D - D;
  F C8 = C + C;
  C8 = C8 + C8;
  C8 = C8 + C8;
  F Y3 = E * (D - X3) - C8;
  F Z3 = p.y * p.z;
  Z3 = Z3 + Z3;
  return {X3, Y3, Z3};
}

// madd-2007-bl: Jacobian + affine, 7M + 4S, with the exceptional cases
template <class F>
FTS_HD Jac<F> jac_add_aff(const Jac<F>& p, const Aff<F>& q) {
  if (q.inf) return p;
  if (is_zero(p.z)) return {q.x, q.y, one_of<F>()};
  F Z1Z1 = sqr(p.z);
  F U2 = q.x * Z1Z1;
  F S2 = q.y * p.z * Z1Z1;
  F H = U2 - p.x;
  F rr = S2 - p.y;
  if (is_zero(H)) {
    if (is_zero(rr)) return jac_dbl(p);
    return jac_inf<F>();
  }
  F HH = sqr(H);
  F I = HH + HH;
  I = I + I;
  F J = H * I;
  rr = rr + rr;
  F V = p.x * I;
  F X3 = sqr(rr) - J - V - V;
  F Y1J = p.y * J;
  F Y3 = rr * (V - X3) - Y1J - Y1J;
  F t = p.z + H;
  F Z3 = sqr(t) - Z1Z1 - HH;
  return {X3, Y3, Z3};
}

// add-2007-bl: Jacobian + Jacobian, 11M + 5S (inline body; jac_add below is
// the out-of-line call most sites use to keep code size down)
template <class F>
FTS_HD Jac<F> jac_add_inl(const Jac<F>& p, const Jac<F>& q) {
  if (is_zero(p.z)) return q;
  if (is_zero(q.z)) return p;
  F Z1Z1 = sqr(p.z);
  F Z2Z2 = sqr(q.z);
  F U1 = p.x * Z2Z2;
  F U2 = q.x * Z1Z1;
  F S1 = p.y * q.z * Z2Z2;
  F S2 = q.y * p.z * Z1Z1;
  F H = U2 - U1;
  F rr = S2 - S1;
  if (is_zero(H)) {
    if (is_zero(rr)) return jac_dbl(p);
    return jac_inf<F>();
  }
  F I = H + H;
  I = sqr(I);
  F J = H * I;
  rr = rr + rr;
  F V = U1 * I;
  F X3 = sqr(rr) - J - V - V;
  F S1J = S1 * J;
  F Y3 = rr * (V - X3) - S1J - S1J;
  F t = p.z + q.z;
  F Z3 = (sqr(t) - Z1Z1 - Z2Z2) * H;
  return {X3, Y3, Z3};
}

template <class F>
FTS_HDN Jac<F> jac_add(const Jac<F>& p, const Jac<F>& q) {
  return jac_add_inl(p, q);
}

template <class F>
FTS_HD F inv_inl(const F& a) {  // other fields: their own inv()
  return inv(a);
}
FTS_HD fp inv_inl(const fp& a) { return fp_inv_var(a); }
FTS_HD fp2 inv_inl(const fp2& a) { return f2_inv_inl(a); }

// inline body (callers with the registers for it, e.g. the one-lane line
// stage); jac_to_aff below is the out-of-line form
template <class F>
FTS_HD Aff<F> jac_to_aff_inl(const Jac<F>& p) {
  Aff<F> r;
  if (is_zero(p.z)) {
    r.x = zero_of<F>();
    r.y = zero_of<F>();
    r.inf = true;
    return r;
  }
  F zi = inv_inl(p.z);
  F zi2 = sqr(zi);
  r.x = p.x * zi2;
  r.y = p.y * zi2 * zi;
  r.inf = false;
  return r;
}
template <class F>
FTS_HDN Aff<F> jac_to_aff(const Jac<F>& p) {
  return jac_to_aff_inl(p);
}

// variable-base scalar multiplication, scalar given as 8 little-endian limbs
// (any value < 2^256; points have order r so no reduction is needed).
// Left-to-right double-and-add with mixed additions.
template <class F>
FTS_HDN Jac<F> aff_mul(const Aff<F>& p, const uint32_t k[8]) {
  Jac<F> acc = jac_inf<F>();
  if (p.inf) return acc;
  bool started = false;
#pragma nounroll
  for (int i = 255; i >= 0; i--) {
    if (started) acc = jac_dbl(acc);
    if ((k[i >> 5] >> (i & 31)) & 1) {
      acc = jac_add_aff(acc, p);
      started = true;
    }
  }
  return acc;
}

// small (<= 64-bit) scalar multiplication
template <class F>
FTS_HDN Jac<F> aff_mul_u64(const Aff<F>& p, uint64_t k) {
  Jac<F> acc = jac_inf<F>();
  if (p.inf) return acc;
  bool started = false;
#pragma nounroll
  for (int i = 63; i >= 0; i--) {
    if (started) acc = jac_dbl(acc);
    if ((k >> i) & 1) {
      acc = jac_add_aff(acc, p);
      started = true;
    }
  }
  return acc;
}

// curve membership of an affine point (Montgomery coordinates)
FTS_HD bool g1_on_curve(const g1a& a) {
  if (a.inf) return true;
  fp three = fe_one<ModP>() + fe_one<ModP>() + fe_one<ModP>();
  return fe_eq(sqr(a.y), sqr(a.x) * a.x + three);
}

// gnark G1Affine.SetBytes via mathlib NewG1FromBytes:
// flags 00 uncompressed (coordinates reduced mod p, (0,0) = infinity, must be
// on the curve), 01 infinity, 10/11 compressed (smallest/largest root); false
// when SetBytes returns an error (a is then the point at infinity).
FTS_HD bool g1_setbytes(const uint8_t* b, uint32_t len, g1a& a) {
  a.inf = false;
  bool ok = true;
  uint8_t m = len >= 1 ? (b[0] & 0xC0) : 0;
  if (len < 32) {
    ok = false;
    a.inf = true;
  } else if (m == 0x40) {
    a.inf = true;
  } else if (m == 0x00) {
    if (len < 64) {
      ok = false;
      a.inf = true;
    } else {
      uint32_t t[8];
      be32_to_limbs_g(t, b);
      a.x = fe_from_int<ModP>(t);
      be32_to_limbs_g(t, b + 32);
      a.y = fe_from_int<ModP>(t);
      if (is_zero(a.x) && is_zero(a.y)) {
        a.inf = true;
      } else {
        ok = g1_on_curve(a);
      }
    }
  } else {
    uint8_t xb[32];
    for (int k = 0; k < 32; k++) xb[k] = b[k];
    xb[0] &= 0x3F;
    uint32_t t[8];
    be32_to_limbs(t, xb);
    uint32_t mm[8];
    for (int k = 0; k < 8; k++) mm[k] = P_MOD[k];
    uint32_t tmp[8];
    if (!sub8(tmp, t, mm)) {
      ok = false;  // X >= p
      a.inf = true;
    } else {
      a.x = fe_from_int<ModP>(t);
      fp three = fe_one<ModP>() + fe_one<ModP>() + fe_one<ModP>();
      fp rhs = sqr(a.x) * a.x + three;
      fp y;
      if (!fp_sqrt(y, rhs)) {
        ok = false;
        a.inf = true;
      } else {
        // gnark LexicographicallyLargest: y > (p-1)/2 as integers
        fp ny = fe_neg(y);
        uint32_t yi[8], nyi[8], d[8];
        fe_to_int(yi, y);
        fe_to_int(nyi, ny);
        bool largest = sub8(d, nyi, yi) != 0;  // y > -y
        bool want_largest = (m == 0xC0);
        a.y = (largest == want_largest) ? y : ny;
      }
    }
  }
  return ok;
}

FTS_HD bool g2_on_curve(const g2a& a) {
  if (a.inf) return true;
  return f2_eq(sqr(a.y), sqr(a.x) * a.x + f2_const(TWIST_B));
}

// gnark RawBytes encodings (canonical big-endian; infinity -> all zero bytes)
FTS_HD void g1_to_bytes(uint8_t* out, const g1a& a) {
  if (a.inf) {
    for (int i = 0; i < 64; i++) out[i] = 0;
    return;
  }
  uint32_t t[8];
  fe_to_int(t, a.x);
  limbs_to_be32(out, t);
  fe_to_int(t, a.y);
  limbs_to_be32(out + 32, t);
}

// gnark RawBytes into global memory (vector stores when 16-byte aligned)
FTS_HD void g1_to_bytes_g(uint8_t* out, const g1a& a) {
  uint32_t t[8];
  if (a.inf) {
    for (int i = 0; i < 8; i++) t[i] = 0;
    limbs_to_be32_g(out, t);
    limbs_to_be32_g(out + 32, t);
    return;
  }
  fe_to_int(t, a.x);
  limbs_to_be32_g(out, t);
  fe_to_int(t, a.y);
  limbs_to_be32_g(out + 32, t);
}

FTS_HD void g2_to_bytes(uint8_t* out, const g2a& a) {
  if (a.inf) {
    for (int i = 0; i < 128; i++) out[i] = 0;
    return;
  }
  uint32_t t[8];
  fe_to_int(t, a.x.c1);
  limbs_to_be32(out, t);
  fe_to_int(t, a.x.c0);
  limbs_to_be32(out + 32, t);
  fe_to_int(t, a.y.c1);
  limbs_to_be32(out + 64, t);
  fe_to_int(t, a.y.c0);
  limbs_to_be32(out + 96, t);
}

}  // namespace fts

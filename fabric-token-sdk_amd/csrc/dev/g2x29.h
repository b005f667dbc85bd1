// Fixed-base G2 partial sums (k_g2_part) on the carry-free balanced form of the
// sextet kernels (dev/fp29.h q2, dev/sx29.h w29_redc): the XYZZ mixed addition
// (madd-2008-s, 8M + 2S; x2q_madd) over balanced Fp2 values instead of the
// 32-bit Jacobian one of curve.h (a Jacobian q2 form, j2b_madd, is the
// FTS_G2_PART_XYZZ=0 option: 8 % more VALU).  The rare doubling case (a running
// sum equal to its next table point) redoes the lane in the 32-bit code, so
// that its registers stay out of the loop (two waves per SIMD).
//
// One Fp2 product is q2_mulb: three 81-MAD limb-product rows (Karatsuba) folded
// by columns into the two rows the balanced reductions need, reduced while they
// are scanned -- against three 32-bit Montgomery products with a carry add per
// MAD.  The partial leaves in 32-bit Jacobian form, so job_g2lines_parts (the
// one-lane line kernel) reads it unchanged; t' = the sum of the four partials
// in affine form does not depend on their representatives, so g2out and every
// line byte are identical to job_g2_part's.
//
// Bounds: coordinates between operations are balanced (q2_mulb and f29_lin2 /
// f29_lin4 outputs: limbs in [-2^28, 2^28], |value| <= p/2 + e); q2_mulb
// takes operands with limbs within 2^29 (a difference of two balanced values),
// q2_sqrb balanced ones.
#pragma once
#include "jobs.h"
#include "sx29.h"

namespace fts {

#ifndef FTS_G2_PART_XYZZ
#define FTS_G2_PART_XYZZ 1  // 1: the parts in XYZZ form (x2q_madd), 0: Jacobian (j2b_madd)
#endif

// Product scanning: column k of both result rows is formed, the reduction's
// multiples m_i p_j (i + j = k) of the digits already chosen are added, and
// the column either yields the next balanced digit m_k (k < 9: the running sum
// then divides exactly by 2^29) or the next output digit -- w29_redc's digits
// and output, with two running sums and the 18 digits live instead of the
// 34 columns of each row (a lone product here sits next to four coordinates).
struct Scan2 {
  int64_t ar, ai;
  int32_t mr[9], mi[9];
};
FTS_HD void scan2_step(Scan2& s, int k, int64_t re, int64_t im, q2& r) {
  s.ar += re;
  s.ai += im;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int j = k - i;
    if (i >= k || j < 0 || j > 8) continue;
    s.ar += (int64_t)s.mr[i] * P29B[j];
    s.ai += (int64_t)s.mi[i] * P29B[j];
  }
  if (k < 9) {
    const uint32_t m0 = ((uint32_t)s.ar * P29_INV) & (uint32_t)F29_MASK;
    const uint32_t m1 = ((uint32_t)s.ai * P29_INV) & (uint32_t)F29_MASK;
    s.mr[k] = (int32_t)((m0 + (uint32_t)F29_HALF) & (uint32_t)F29_MASK) - F29_HALF;
    s.mi[k] = (int32_t)((m1 + (uint32_t)F29_HALF) & (uint32_t)F29_MASK) - F29_HALF;
    s.ar = (s.ar + (int64_t)s.mr[k] * P29B[0]) >> 29;  // a multiple of 2^29 now
    s.ai = (s.ai + (int64_t)s.mi[k] * P29B[0]) >> 29;
  } else {
    r.c0.l[k - 9] = f29_bdigit(s.ar);
    r.c1.l[k - 9] = f29_bdigit(s.ai);
    s.ar = (s.ar + F29_HALF) >> 29;
    s.ai = (s.ai + F29_HALF) >> 29;
  }
}
// a b (limbs within 2^29): the Karatsuba columns of sx29.h w29_prod1, scanned
FTS_HD q2 q2_mulb(const q2& a, const q2& b) {
  FTS_COUNT_MAD(192);
  FTS_SCHED_FENCE();
  const f29 sa = f29_add(a.c0, a.c1), sb = f29_add(b.c0, b.c1);
  Scan2 s;
  s.ar = s.ai = 0;
  q2 r;
#pragma unroll
  for (int k = 0; k < 17; k++) {
    uint64_t u = 0, v = 0, w = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j < 0 || j > 8) continue;
      u += w29_p(a.c0.l[i], b.c0.l[j]);
      v += w29_p(a.c1.l[i], b.c1.l[j]);
      w += w29_p(sa.l[i], sb.l[j]);
    }
    scan2_step(s, k, (int64_t)(u - v), (int64_t)(w - (u + v)), r);
  }
  r.c0.l[8] = (int32_t)s.ar;
  r.c1.l[8] = (int32_t)s.ai;
  return r;
}
// a b + c d with one reduction (a, c limbs within 2^29; b, d balanced): the
// four rows' columns stay below 36 x 2^57 + the reduction's terms < 2^63
FTS_HD q2 q2_mul2b(const q2& a, const q2& b, const q2& c, const q2& d) {
  FTS_COUNT_MAD(384);
  FTS_SCHED_FENCE();
  const f29 sa = f29_add(a.c0, a.c1), sb = f29_add(b.c0, b.c1);
  const f29 sc = f29_add(c.c0, c.c1), sd = f29_add(d.c0, d.c1);
  Scan2 s;
  s.ar = s.ai = 0;
  q2 r;
#pragma unroll
  for (int k = 0; k < 17; k++) {
    uint64_t u = 0, v = 0, w = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j < 0 || j > 8) continue;
      u += w29_p(a.c0.l[i], b.c0.l[j]) + w29_p(c.c0.l[i], d.c0.l[j]);
      v += w29_p(a.c1.l[i], b.c1.l[j]) + w29_p(c.c1.l[i], d.c1.l[j]);
      w += w29_p(sa.l[i], sb.l[j]) + w29_p(sc.l[i], sd.l[j]);
    }
    scan2_step(s, k, (int64_t)(u - v), (int64_t)(w - (u + v)), r);
  }
  r.c0.l[8] = (int32_t)s.ar;
  r.c1.l[8] = (int32_t)s.ai;
  return r;
}
// a^2 = (a0 + a1)(a0 - a1) + 2 a0 a1 u (a balanced): two limb-product rows
FTS_HD q2 q2_sqrb(const q2& a) {
  FTS_COUNT_MAD(128);
  FTS_SCHED_FENCE();
  const f29 s0 = f29_add(a.c0, a.c1), d = f29_sub(a.c0, a.c1), t = f29_add(a.c0, a.c0);
  Scan2 s;
  s.ar = s.ai = 0;
  q2 r;
#pragma unroll
  for (int k = 0; k < 17; k++) {
    int64_t re = 0, im = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j < 0 || j > 8) continue;
      re += (int64_t)s0.l[i] * d.l[j];
      im += (int64_t)t.l[i] * a.c1.l[j];
    }
    scan2_step(s, k, re, im, r);
  }
  r.c0.l[8] = (int32_t)s.ar;
  r.c1.l[8] = (int32_t)s.ai;
  return r;
}
FTS_HD q2 q2_lin2b(const q2& a, int32_t ca, const q2& b, int32_t cb) {
  return {f29_lin2(a.c0, ca, b.c0, cb), f29_lin2(a.c1, ca, b.c1, cb)};
}
FTS_HD q2 q2_lin3b(const q2& a, int32_t ca, const q2& b, int32_t cb, const q2& c, int32_t cc) {
  return {f29_lin4(a.c0, ca, b.c0, cb, c.c0, cc, c.c0, 0), f29_lin4(a.c1, ca, b.c1, cb, c.c1, cc, c.c1, 0)};
}
FTS_HD q2 q2_subr(const q2& a, const q2& b) { return {f29_sub(a.c0, b.c0), f29_sub(a.c1, b.c1)}; }
FTS_HD bool q2_rzero(const q2& a) { return f29_reduced_zero(a.c0) && f29_reduced_zero(a.c1); }
FTS_HD q2 q2_one_b() { return {f29_breduce(f29_from_fp(fe_one<ModP>())), q2_zero().c1}; }

// x = X / ZZ, y = Y / ZZZ, ZZ^3 = ZZZ^2
struct x2q {
  q2 x, y, zz, zzz;
  bool inf;
};

// 2 (x, y) for an affine point (balanced), mdbl-2008-s-1 (a = 0)
FTS_HD x2q x2q_dbl_aff(const q2& x, const q2& y) {
  const q2 U = q2_lin2b(y, 2, y, 0);
  const q2 V = q2_sqrb(U);
  const q2 W = q2_mulb(U, V);
  const q2 S = q2_mulb(x, V);
  const q2 M = q2_lin2b(q2_sqrb(x), 3, x, 0);
  const q2 X3 = q2_lin3b(q2_sqrb(M), 1, S, -2, S, 0);
  const q2 Y3 = q2_lin2b(q2_mulb(M, q2_subr(S, X3)), 1, q2_mulb(W, y), -1);
  return {X3, Y3, V, W, false};
}

// p + (x2, y2), (x2, y2) affine (balanced) and not the identity: madd-2008-s.
// P = U2 - X vanishes iff the x coordinates agree: the sum is then a doubling
// (R = 0) or the identity.
FTS_HD x2q x2q_madd(const x2q& p, const q2& x2, const q2& y2, bool* dbl = nullptr) {
  if (p.inf) {
    const q2 one = q2_one_b();
    return {x2, y2, one, one, false};
  }
  const q2 P = q2_lin2b(q2_mulb(x2, p.zz), 1, p.x, -1);
  const q2 R = q2_lin2b(q2_mulb(y2, p.zzz), 1, p.y, -1);
  if (q2_rzero(P)) {
    if (q2_rzero(R)) {
      if (dbl) {  // as j2b_madd: the caller redoes the lane in the 32-bit code
        *dbl = true;
        return p;
      }
      return x2q_dbl_aff(x2, y2);
    }
    x2q o = p;
    o.inf = true;
    return o;
  }
  // ordered so that each input dies at its last use (the accumulator, the
  // operands and one product's 34 columns are live together)
  const q2 PP = q2_sqrb(P);
  const q2 ZZ3 = q2_mulb(p.zz, PP);
  const q2 PPP = q2_mulb(P, PP);
  const q2 ZZZ3 = q2_mulb(p.zzz, PPP);
  const q2 Q = q2_mulb(p.x, PP);
  const q2 X3 = q2_lin3b(q2_sqrb(R), 1, PPP, -1, Q, -2);
  const q2 YP = q2_mulb(p.y, PPP);
  const q2 Y3 = q2_lin2b(q2_mulb(R, q2_subr(Q, X3)), 1, YP, -1);
  return {X3, Y3, ZZ3, ZZZ3, false};
}

// to 32-bit Jacobian without an inversion: Z' = ZZ ZZZ, X' = X ZZ ZZZ^2,
// Y' = Y ZZZ^4 (X'/Z'^2 = X/ZZ and Y'/Z'^3 = Y/ZZZ since ZZ^3 = ZZZ^2)
FTS_HD g2j x2q_to_g2j(const x2q& p) {
  if (p.inf) return jac_inf<fp2>();
  const q2 t = q2_sqrb(p.zzz);
  const q2 X = q2_mulb(q2_mulb(p.x, p.zz), t);
  const q2 Y = q2_mulb(p.y, q2_sqrb(t));
  const q2 Z = q2_mulb(p.zz, p.zzz);
  return {q2_to_fp2(X), q2_to_fp2(Y), q2_to_fp2(Z)};
}

// Jacobian form (X / Z^2, Y / Z^3): madd-2007-bl, 7M + 4S -- the same product
// rows as the XYZZ addition with one coordinate fewer to keep live, which
// brings the part kernel under the 256 registers of two waves per SIMD
struct j2b {
  q2 x, y, z;
  bool inf;
};
// dbl-2009-l (a = 0), p not the identity
FTS_HD j2b j2b_dbl(const j2b& p) {
  const q2 A = q2_sqrb(p.x);
  const q2 B = q2_sqrb(p.y);
  const q2 C = q2_sqrb(B);
  const q2 D = q2_lin3b(q2_sqrb(q2_lin2b(p.x, 1, B, 1)), 2, A, -2, C, -2);  // 2((X + B)^2 - A - C)
  const q2 E = q2_lin2b(A, 3, A, 0);
  const q2 X3 = q2_lin3b(q2_sqrb(E), 1, D, -2, D, 0);
  const q2 Y3 = q2_lin2b(q2_mulb(E, q2_subr(D, X3)), 1, C, -8);
  const q2 Z3 = q2_lin2b(q2_mulb(p.y, p.z), 2, p.y, 0);
  return {X3, Y3, Z3, false};
}
// p + (x2, y2), (x2, y2) affine (balanced) and not the identity.  H = U2 - X
// vanishes iff the x coordinates agree: the identity (r != 0), or p equals the
// point -- then *dbl is set and p returned unchanged (the caller doubles; the
// part kernel redoes the lane in the 32-bit code, so that the doubling's
// registers do not count against the loop's)
FTS_HD j2b j2b_madd(const j2b& p, const q2& x2, const q2& y2, bool* dbl = nullptr) {
  if (p.inf) return {x2, y2, q2_one_b(), false};
  const q2 Z1Z1 = q2_sqrb(p.z);
  const q2 H = q2_lin2b(q2_mulb(x2, Z1Z1), 1, p.x, -1);
  const q2 r = q2_lin2b(q2_mulb(y2, q2_mulb(p.z, Z1Z1)), 2, p.y, -2);  // 2 (S2 - Y)
  if (q2_rzero(H)) {
    if (q2_rzero(r)) {
      if (dbl) {
        *dbl = true;
        return p;
      }
      return j2b_dbl({x2, y2, q2_one_b(), false});
    }
    j2b o = p;
    o.inf = true;
    return o;
  }
  const q2 HH = q2_sqrb(H);
  const q2 Z3 = q2_lin3b(q2_sqrb(q2_lin2b(p.z, 1, H, 1)), 1, Z1Z1, -1, HH, -1);  // 2 Z H
  const q2 I = q2_lin2b(HH, 4, HH, 0);
  const q2 J = q2_mulb(H, I);
  const q2 V = q2_mulb(p.x, I);
  const q2 X3 = q2_lin3b(q2_sqrb(r), 1, J, -1, V, -2);
  const q2 Y3 = q2_lin2b(q2_mulb(r, q2_subr(V, X3)), 1, q2_mulb(p.y, J), -2);
  return {X3, Y3, Z3, false};
}
FTS_HD g2j j2b_to_g2j(const j2b& p) {
  if (p.inf) return jac_inf<fp2>();
  return {q2_to_fp2(p.x), q2_to_fp2(p.y), q2_to_fp2(p.z)};
}

// job_g2_part (dev/jobs.h) on this form: lane q of a job sums the table points
// of the (base, window) positions q, q + 4, ...
FTS_HD void job_g2_part_x29(const G2Job& g, int q, const uint32_t (*scal)[8], const G2Dev* tab, G2PartDev& out) {
#if FTS_G2_PART_XYZZ
  x2q acc;
  acc.inf = true;
  acc.x = acc.y = acc.zz = acc.zzz = q2_zero();
  bool dbl = false;
#else
  j2b acc;
  acc.inf = true;
  acc.x = acc.y = acc.z = q2_zero();
  bool dbl = false;
#endif
#pragma nounroll
  for (int p = q; p < 3 * G2TAB_WINDOWS; p += 4) {
    int f = p / G2TAB_WINDOWS, w = p % G2TAB_WINDOWS;
    if (f < g.nfix) {
      int32_t d = sdigit_at(scal[g.fscal[f]], G2TAB_C, w);
      if (d) {
        g2a T = g2_load(tab[((size_t)g.fbase[f] * G2TAB_WINDOWS + w) * G2TAB_DIGITS + (uint32_t)(d < 0 ? -d : d) - 1]);
        const q2 x2 = q2_from_fp2(T.x);
        q2 y2 = q2_from_fp2(T.y);
        if (d < 0) y2 = q2_neg(y2);
#if FTS_G2_PART_XYZZ
        acc = x2q_madd(acc, x2, y2, &dbl);
        if (dbl) break;
#else
        acc = j2b_madd(acc, x2, y2, &dbl);
        if (dbl) break;
#endif
      }
    }
  }
  if (dbl) {
    job_g2_part(g, q, scal, tab, out);  // a running sum met its next table point
    return;
  }
#if FTS_G2_PART_XYZZ
  g2part_store(out, x2q_to_g2j(acc));
#else
  g2part_store(out, j2b_to_g2j(acc));
#endif
}

}  // namespace fts

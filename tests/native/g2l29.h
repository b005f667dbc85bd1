// TEST-ONLY (host emulation, tests/native/sx_emu.cpp): an experimental carry-free
// variant of the line stage kept for its parity test; no kernel includes it.
// k_g2lines in one lane per membership digit, on the carry-free balanced
// 29-bit field form (dev/fp29.h q2, dev/sx29.h w29 rows):
//   phase A  t' = c PK0 + v PK1 + h PK2 (pok.go:175-183, folded) from the
//            signed-window fixed-base tables: Jacobian + affine additions
//            (madd-2007-bl) on q2, exceptional sums through the 32-bit code,
//            one inversion (32-bit) for the affine t' the G2 output holds;
//   phase B  the 88 Miller lines of t' evaluated at R (65 doublings, 21 NAF
//            additions, 2 Frobenius lines), written in the component planes
//            of EvLineDev that k_miller reads.
// Same points and lines as job_g2lines (dev/jobs.h) up to one factor in Fp
// per line: the doubling runs on 4 T (homogeneous projective, the same point)
// so that no halving is needed (A' = XY, G' = B + F; 4 X3 = 2 A'(B - F),
// 4 Y3 = G'^2 - 12 E^2, 4 Z3 = 4 B H), and every later line is homogeneous in
// T's coordinates.  A line scaled by an element of Fp (or Fp2) multiplies the
// Miller value by an element the final exponentiation sends to 1, so the GT
// bytes are identical (tests/native/sx_emu.cpp sxe_g2lines29 checks them).
//
// Bounds (|limb| <= 2^28 "balanced", products < 2^63 per 64-bit column):
//   q2_mul / row products: 18 limb products per column; one operand may have
//     limbs up to 2^30 when the other is balanced (18 x 2^58 < 2^62.2);
//   q2_sqr29: (a0 + a1)(a0 - a1) and (2 a0) a1 need balanced a;
//   q2_lin: |coefficients| <= 16, input limbs <= 2^29; output balanced.
#pragma once
#include "../../fabric-token-sdk_amd/csrc/dev/jobs.h"
#include "../../fabric-token-sdk_amd/csrc/dev/sx29.h"
#include "../../fabric-token-sdk_amd/csrc/dev/g2lines29.h"

namespace fts {

FTS_HD q2 q2_sub(const q2& a, const q2& b) { return {f29_sub(a.c0, b.c0), f29_sub(a.c1, b.c1)}; }
// ca a + cb b, balanced
FTS_HD q2 q2_lin(const q2& a, int32_t ca, const q2& b, int32_t cb) {
  return {f29_lin2(a.c0, ca, b.c0, cb), f29_lin2(a.c1, ca, b.c1, cb)};
}
FTS_HD q2 q2_scale(const q2& a, int32_t c) { return q2_lin(a, c, a, 0); }
FTS_HD bool q2_reduced_zero(const q2& a) { return f29_reduced_zero(a.c0) && f29_reduced_zero(a.c1); }

// a (Fp2) times s (Fp): two rows
FTS_HD q2 q2_mul_f29(const q2& a, const f29& s) { return {f29_mulb(a.c0, s), f29_mulb(a.c1, s)}; }

// a^2 = (a0 + a1)(a0 - a1) + 2 a0 a1 u: two rows
FTS_HD q2 q2_sqr29(const q2& a) {
  FTS_COUNT_MAD(128);
  const f29 s = f29_add(a.c0, a.c1), d = f29_sub(a.c0, a.c1), t = f29_add(a.c0, a.c0);
  int64_t re[17], im[17];
#pragma unroll
  for (int i = 0; i < 17; i++) re[i] = im[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++)
#pragma unroll
    for (int j = 0; j < 9; j++) {
      re[i + j] += (int64_t)s.l[i] * d.l[j];
      im[i + j] += (int64_t)t.l[i] * a.c1.l[j];
    }
  return {w29_redc(re), w29_redc(im)};
}


// Constants of phase B (G2L29_CONST, g2c_f / g2c_q, q2_one29): dev/g2lines29.h

// Jacobian point on the twist in this form (inf: the identity)
struct j2q {
  q2 x, y, z;
  bool inf;
};

FTS_HD g2j j2q_to32(const j2q& p) {
  if (p.inf) return jac_inf<fp2>();
  return {q2_to_fp2(p.x), q2_to_fp2(p.y), q2_to_fp2(p.z)};
}
FTS_HD j2q j2q_from32(const g2j& p) {
  if (is_zero(p.z)) return {q2_zero(), q2_zero(), q2_zero(), true};
  return {q2_from_fp2(p.x), q2_from_fp2(p.y), q2_from_fp2(p.z), false};
}

// p + (x2, y2) (affine, not the identity; x2, y2 limbs < 2^29), madd-2007-bl
// with H and 2H from one difference: 7 products, 3 squarings
FTS_HD j2q j2q_madd(const j2q& p, const q2& x2, const q2& y2) {
  if (p.inf) return {q2_scale(x2, 1), q2_scale(y2, 1), q2_one29(), false};
  q2 Z1Z1 = q2_sqr29(p.z);
  q2 U2 = q2_mul(x2, Z1Z1);
  q2 S2 = q2_mul(y2, q2_mul(p.z, Z1Z1));
  q2 H = q2_lin(U2, 1, p.x, -1);
  q2 r2 = q2_lin(S2, 2, p.y, -2);  // 2 rr
  if (q2_reduced_zero(H)) {
    // p = +-(x2, y2): a doubling (rr = 0) or the identity -- through the 32-bit code
    if (q2_reduced_zero(r2)) return j2q_from32(jac_dbl(j2q_to32(p)));
    return {q2_zero(), q2_zero(), q2_zero(), true};
  }
  q2 H2 = q2_scale(H, 2);
  q2 I = q2_sqr29(H2);  // 4 HH
  q2 J = q2_mul(H, I);
  q2 V = q2_mul(p.x, I);
  q2 X3 = q2_lin(q2_sub(q2_sqr29(r2), J), 1, V, -2);
  W29 w;
  w29_init(w);
  w29_mac(w, r2, q2_sub(V, X3));
  w29_mac(w, p.y, q2_scale(J, -2));
  q2 Y3 = w29_reduce(w);
  q2 Z3 = q2_mul(p.z, H2);
  return {X3, Y3, Z3, false};
}

// T <- 4 (2T) = 2T; line (-H, 3J, I) evaluated: c0 = -H yP, c3 = 3J xP, c4 = I
FTS_HD void g2l29_dbl(q2& X, q2& Y, q2& Z, const f29& yP, const f29& xP, q2& c0, q2& c3, q2& c4) {
  q2 XY = q2_mul(X, Y);
  q2 B = q2_sqr29(Y);
  q2 C = q2_sqr29(Z);
  q2 E = q2_mul(C, g2c_q(G2C_B3));  // 3 b' Z^2
  q2 H = q2_sub(q2_sub(q2_sqr29(q2_lin(Y, 1, Z, 1)), B), C);  // 2 Y Z, limbs <= 3 x 2^28
  c0 = q2_mul_f29(q2_neg(H), yP);
  c4 = q2_lin(E, 1, B, -1);
  c3 = q2_scale(q2_mul_f29(q2_sqr29(X), xP), 3);
  q2 BmF = q2_lin(B, 1, E, -3), Gp = q2_lin(B, 1, E, 3);
  q2 EE = q2_sqr29(E);
  q2 X3 = q2_scale(q2_mul(XY, BmF), 2);
  Y = q2_lin(q2_sqr29(Gp), 1, EE, -12);
  Z = q2_scale(q2_mul(B, H), 4);
  X = X3;
}

// T <- T + (Qx, Qy) (affine, balanced); line (L, -O, Qx O - L Qy) evaluated:
// c0 = L yP, c3 = -O xP, c4 = Qx O - L Qy
FTS_HD void g2l29_add(q2& X, q2& Y, q2& Z, const q2& Qx, const q2& Qy, const f29& yP, const f29& xP, q2& c0,
                       q2& c3, q2& c4) {
  q2 O = q2_lin(Y, 1, q2_mul(Qy, Z), -1);
  q2 L = q2_lin(X, 1, q2_mul(Qx, Z), -1);
  q2 C = q2_sqr29(O);
  q2 D = q2_sqr29(L);
  q2 E = q2_mul(L, D);
  q2 F = q2_mul(Z, C);
  q2 G = q2_mul(X, D);
  q2 H = q2_add(q2_lin(E, 1, G, -2), F);  // limbs <= 2^29
  c0 = q2_mul_f29(L, yP);
  c3 = q2_mul_f29(q2_neg(O), xP);
  W29 w;
  w29_init(w);
  w29_mac(w, Qx, O);
  w29_mac(w, L, q2_neg(Qy));
  c4 = w29_reduce(w);
  q2 X3 = q2_mul(L, H);
  w29_init(w);
  w29_mac(w, q2_sub(G, H), O);
  w29_mac(w, Y, q2_neg(E));
  Y = w29_reduce(w);
  Z = q2_mul(E, Z);
  X = X3;
}

// out-of-line copies (one code copy per call site class keeps the loop bodies
// inside the instruction cache; state passes through the call frame)
FTS_HDN void j2q_madd_call(j2q& acc, const q2& x2, const q2& y2) { acc = j2q_madd(acc, x2, y2); }
FTS_HDN void g2l29_dbl_call(q2& X, q2& Y, q2& Z, const f29& yP, const f29& xP, q2& c0, q2& c3, q2& c4) {
  g2l29_dbl(X, Y, Z, yP, xP, c0, c3, c4);
}
FTS_HDN void g2l29_add_call(q2& X, q2& Y, q2& Z, const q2& Qx, const q2& Qy, const f29& yP, const f29& xP, q2& c0,
                            q2& c3, q2& c4) {
  g2l29_add(X, Y, Z, Qx, Qy, yP, xP, c0, c3, c4);
}

FTS_HD void evline_put29(EvLineDev* base, uint32_t s, int c, uint32_t idx, uint32_t njobs, const f29& b) {
  int32_t* o = (int32_t*)base + evl_off(s, c, idx, njobs);
#pragma unroll
  for (int i = 0; i < 9; i++) o[i] = b.l[i];
  o[9] = 0;
}
FTS_HD void evline_store29(EvLineDev* base, uint32_t s, uint32_t idx, uint32_t njobs, const q2& c0, const q2& c3,
                           const q2& c4) {
  evline_put29(base, s, 0, idx, njobs, c0.c0);
  evline_put29(base, s, 1, idx, njobs, c0.c1);
  evline_put29(base, s, 2, idx, njobs, c3.c0);
  evline_put29(base, s, 3, idx, njobs, c3.c1);
  evline_put29(base, s, 4, idx, njobs, c4.c0);
  evline_put29(base, s, 5, idx, njobs, c4.c1);
}

FTS_HD q2 q2_ld_raw(const uint32_t a[8], const uint32_t b[8]) {
  fp x, y;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    x.v[i] = a[i];
    y.v[i] = b[i];
  }
  return {f29_from_fp(x), f29_from_fp(y)};  // limbs < 2^29, value < 32 p
}

// CALLS: bit 0 the phase-A addition, bit 1 the line addition, bit 2 the line
// doubling run out of line
template <int CALLS>
FTS_HD void job_g2lines29(const G2Job& g, const PairJob& j, const uint32_t (*scal)[8], const G2Dev* tab,
                          G2Dev* g2out, const G1Dev* pts, EvLineDev* lines, uint32_t idx, uint32_t njobs) {
  // ---- phase A
  j2q acc = {q2_zero(), q2_zero(), q2_zero(), true};
  for (int f = 0; f < g.nfix; f++) {
    const G2Dev* tb = tab + (size_t)g.fbase[f] * G2TAB_WINDOWS * G2TAB_DIGITS;
    const uint32_t* s = scal[g.fscal[f]];
#pragma nounroll
    for (int w = 0; w < G2TAB_WINDOWS; w++) {
      int32_t d = sdigit_at(s, G2TAB_C, w);
      if (d) {
        const G2Dev& T = tb[(size_t)w * G2TAB_DIGITS + (uint32_t)(d < 0 ? -d : d) - 1];
        q2 x2 = q2_ld_raw(T.x0, T.x1), y2 = q2_ld_raw(T.y0, T.y1);
        if (d < 0) y2 = q2_neg(y2);
        if (CALLS & 1)
          j2q_madd_call(acc, x2, y2);
        else
          acc = j2q_madd(acc, x2, y2);
      }
    }
  }
  g2a Q = jac_to_aff(j2q_to32(acc));
  {
    G2Dev d;
    g2_store(d, Q);
    g2out[g.out] = d;
  }
  // ---- phase B
  g1a P = g1_load(pts[j.p2]);
  const bool use = !(P.inf || Q.inf);
  const f29 yP = f29_breduce(f29_from_fp(P.y)), xP = f29_breduce(f29_from_fp(P.x));
  const q2 Qx = q2_from_fp2(Q.x), Qy = q2_from_fp2(Q.y);
  q2 X = Qx, Y = Qy, Z = q2_one29();
  int i = 64, sign = 0;
  bool pend = false;
  // one loop over the 88 lines (each step function inlined once): doubling,
  // addition of +-Q (NAF digit), then pi(Q) and -pi^2(Q)
#pragma nounroll
  for (int s = 0; s < MILLER_LINES; s++) {
    bool dbl = false;
    q2 Ax = Qx, Ay = Qy;
    if (s == MILLER_LINES - 2) {
      Ax = q2_mul(q2_conj(Qx), g2c_q(G2C_FX));
      Ay = q2_mul(q2_conj(Qy), g2c_q(G2C_FY));
    } else if (s == MILLER_LINES - 1) {
      Ax = q2_mul_f29(Qx, g2c_f(G2C_F2X));
      Ay = q2_mul_f29(q2_neg(Qy), g2c_f(G2C_F2Y));
    } else if (!pend) {
      dbl = true;
      sign = naf_digit(i);
      pend = sign != 0;
      if (!pend) i--;
    } else {
      if (sign < 0) Ay = q2_neg(Qy);
      pend = false;
      i--;
    }
    q2 c0, c3, c4;
    if (dbl) {
      if (CALLS & 4)
        g2l29_dbl_call(X, Y, Z, yP, xP, c0, c3, c4);
      else
        g2l29_dbl(X, Y, Z, yP, xP, c0, c3, c4);
    } else {
      if (CALLS & 2)
        g2l29_add_call(X, Y, Z, Ax, Ay, yP, xP, c0, c3, c4);
      else
        g2l29_add(X, Y, Z, Ax, Ay, yP, xP, c0, c3, c4);
    }
    if (!use) {
      c0 = q2_one29();
      c3 = c4 = q2_zero();
    }
    evline_store29(lines, (uint32_t)s, idx, njobs, c0, c3, c4);
  }
}

// k_g2_part on the carry-free form: the same Jacobian partial as job_g2_part
// (j2q_madd runs madd-2007-bl's formulas, so X, Y, Z agree mod p and the
// canonical 32-bit words written are byte-identical).  Measured as a kernel:
// 256 VGPRs, one wave per SIMD, 3.69 vs 3.57 ms for the t' + lines stage --
// not launched (profiles/r02g_norm_ab.txt).
FTS_HD void job_g2_part29(const G2Job& g, int q, const uint32_t (*scal)[8], const G2Dev* tab, G2PartDev& out) {
  j2q acc = {q2_zero(), q2_zero(), q2_zero(), true};
#pragma nounroll
  for (int p = q; p < 3 * G2TAB_WINDOWS; p += 4) {
    int f = p / G2TAB_WINDOWS, w = p % G2TAB_WINDOWS;
    if (f < g.nfix) {
      int32_t d = sdigit_at(scal[g.fscal[f]], G2TAB_C, w);
      if (d) {
        const G2Dev& T = tab[((size_t)g.fbase[f] * G2TAB_WINDOWS + w) * G2TAB_DIGITS + (uint32_t)(d < 0 ? -d : d) - 1];
        q2 x2 = q2_ld_raw(T.x0, T.x1), y2 = q2_ld_raw(T.y0, T.y1);
        if (d < 0) y2 = q2_neg(y2);
        acc = j2q_madd(acc, x2, y2);
      }
    }
  }
  g2part_store(out, j2q_to32(acc));
}

}  // namespace fts

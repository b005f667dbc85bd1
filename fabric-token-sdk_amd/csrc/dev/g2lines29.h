// The pair-2 line chain of k_g2lines1 (one lane per membership digit) on the
// carry-free balanced form: the 88 Miller lines of t' evaluated at R (65
// doublings, 21 NAF additions, 2 Frobenius lines) with q2 values and the
// product-scanned Fp2 products of dev/g2x29.h, written in EvLineDev's balanced
// planes as the 32-bit chain (job_g2lines_parts) writes them.
//
// Same points as the 32-bit chain, and the same lines up to one factor in Fp
// per line: the doubling runs on 4 T (homogeneous projective, the same point)
// so that no halving is needed -- A' = XY, G' = B + F: 4 X3 = 2 A'(B - F),
// 4 Y3 = G'^2 - 12 E^2, 4 Z3 = 4 B H -- and every later line is homogeneous in
// T's coordinates.  A line scaled by an element of Fp multiplies the Miller
// value by an element the final exponentiation sends to 1, so every GT byte is
// identical (tests/test_sextet.py test_g2_lines_carry_free checks them).
//
// Bounds: every value between operations is balanced (q2_mulb / q2_sqrb /
// f29_lin2 / f29_lin4 outputs: limbs in [-2^28, 2^28], |value| <= p/2 + e);
// q2_mulb's operands are balanced or differences of two balanced values.
#pragma once
#include "g2x29.h"

namespace fts {

// 3 b' (the twist's b' = 3 / (9 + u)) in the balanced R = 2^261 form, as
// literals (scalar operands); tests/native/sx_emu.cpp sxe_g2l29_consts
// re-derives them from dev/constants.h
static constexpr int32_t G2L_B3[2][9] = {
    {-253769606, 6731155, -156399417, 46225477, -175165556, 162336334, -209914092, -192467748, -1389658},
    {31837202, -172120824, -128414024, 15984953, -118312780, 62914239, -210424777, 247765560, 1563920},
};
FTS_HD q2 g2l_b3() {
  q2 r;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    r.c0.l[k] = G2L_B3[0][k];
    r.c1.l[k] = G2L_B3[1][k];
  }
  return r;
}

FTS_HD q2 q2_scaleb(const q2& a, int32_t c) { return q2_lin2b(a, c, a, 0); }

// a (Fp2) times s (Fp), both balanced: two rows scanned together
FTS_HD q2 q2_mulfb(const q2& a, const f29& s) {
  FTS_COUNT_MAD(128);
  FTS_SCHED_FENCE();
  Scan2 st;
  st.ar = st.ai = 0;
  q2 r;
#pragma unroll
  for (int k = 0; k < 17; k++) {
    int64_t re = 0, im = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j < 0 || j > 8) continue;
      re += (int64_t)a.c0.l[i] * s.l[j];
      im += (int64_t)a.c1.l[i] * s.l[j];
    }
    scan2_step(st, k, re, im, r);
  }
  r.c0.l[8] = (int32_t)st.ar;
  r.c1.l[8] = (int32_t)st.ai;
  return r;
}

// T <- 4 (2T) = 2T; the line (-H, 3J, I) evaluated: c0 = -H yP, c3 = 3 X^2 xP,
// c4 = E - B
FTS_HD void g2l_dbl(q2& X, q2& Y, q2& Z, const f29& yP, const f29& xP, q2& c0, q2& c3, q2& c4) {
  const q2 B = q2_sqrb(Y);
  const q2 C = q2_sqrb(Z);
  const q2 H = q2_lin3b(q2_sqrb(q2_lin2b(Y, 1, Z, 1)), 1, B, -1, C, -1);  // 2 Y Z
  const q2 XY = q2_mulb(X, Y);
  const q2 E = q2_mulb(C, g2l_b3());  // 3 b' Z^2
  c0 = q2_mulfb(q2_neg(H), yP);
  c3 = q2_scaleb(q2_mulfb(q2_sqrb(X), xP), 3);
  c4 = q2_lin2b(E, 1, B, -1);
  X = q2_scaleb(q2_mulb(XY, q2_lin2b(B, 1, E, -3)), 2);
  Y = q2_lin2b(q2_sqrb(q2_lin2b(B, 1, E, 3)), 1, q2_sqrb(E), -12);
  Z = q2_scaleb(q2_mulb(B, H), 4);
}

// T <- T + (Qx, Qy) (affine, balanced); the line (L, -O, Qx O - L Qy)
// evaluated: c0 = L yP, c3 = -O xP, c4 = Qx O - L Qy
FTS_HD void g2l_add(q2& X, q2& Y, q2& Z, const q2& Qx, const q2& Qy, const f29& yP, const f29& xP, q2& c0, q2& c3,
                    q2& c4) {
  const q2 O = q2_lin2b(Y, 1, q2_mulb(Qy, Z), -1);
  const q2 L = q2_lin2b(X, 1, q2_mulb(Qx, Z), -1);
  const q2 D = q2_sqrb(L);
  const q2 E = q2_mulb(L, D);
  const q2 G = q2_mulb(X, D);
  const q2 H = q2_lin3b(E, 1, G, -2, q2_mulb(Z, q2_sqrb(O)), 1);
  c0 = q2_mulfb(L, yP);
  c3 = q2_mulfb(q2_neg(O), xP);
  c4 = q2_lin2b(q2_mulb(Qx, O), 1, q2_mulb(L, Qy), -1);
  const q2 Y3 = q2_lin2b(q2_mulb(q2_subr(G, H), O), 1, q2_mulb(Y, E), -1);
  X = q2_mulb(L, H);
  Y = Y3;
  Z = q2_mulb(E, Z);
}

FTS_HD void evline_put_b(EvLineDev* base, uint32_t s, int c, uint32_t idx, uint32_t njobs, const f29& b) {
  int32_t* o = (int32_t*)base + evl_off(s, c, idx, njobs);
#pragma unroll
  for (int i = 0; i < 9; i++) o[i] = b.l[i];
  o[9] = 0;
}

// job_g2lines_parts (dev/jobs.h) with the line chain on this form: the four
// partial sums of t' are added and normalised in the 32-bit code (the G2
// output), then the lines
FTS_HD void job_g2lines_parts_x29(const G2Job& g, const PairJob& j, const G2PartDev* part, G2Dev* g2out,
                                  const G1Dev* pts, EvLineDev* lines, uint32_t idx, uint32_t njobs) {
  g2j acc = g2part_load(part[idx]);
#pragma nounroll
  for (int q = 1; q < 4; q++) acc = jac_add_inl(acc, g2part_load(part[(size_t)q * njobs + idx]));
  G2Dev d;
  const g2a Q = jac_to_aff_inl(acc);
  g2_store(d, Q);
  g2out[g.out] = d;
  const g1a P = g1_load(pts[j.p2]);
  const bool use = !(P.inf || Q.inf);
  const f29 yP = f29_breduce(f29_from_fp(P.y)), xP = f29_breduce(f29_from_fp(P.x));
  const q2 Qx = q2_from_fp2(Q.x), Qy = q2_from_fp2(Q.y);
  q2 X = Qx, Y = Qy, Z = q2_one_b();
  const q2 one = q2_one_b();
#pragma nounroll
  for (int s = 0; s < MILLER_LINES; s++) {
    const int t = MILLER_STEPS.t[s];
    q2 c0, c3, c4;
    if (t == STEP_DBL) {
      g2l_dbl(X, Y, Z, yP, xP, c0, c3, c4);
    } else {
      q2 Ax = Qx, Ay = Qy;
      if (t == STEP_FROB1 || t == STEP_FROB2) {
        const g2a A = t == STEP_FROB1 ? tw_frob(Q) : tw_frob2_neg(Q);
        Ax = q2_from_fp2(A.x);
        Ay = q2_from_fp2(A.y);
      } else if (t == STEP_SUB) {
        Ay = q2_neg(Qy);
      }
      g2l_add(X, Y, Z, Ax, Ay, yP, xP, c0, c3, c4);
    }
    if (!use) {
      c0 = one;
      c3 = c4 = q2_zero();
    }
    evline_put_b(lines, (uint32_t)s, 0, idx, njobs, c0.c0);
    evline_put_b(lines, (uint32_t)s, 1, idx, njobs, c0.c1);
    evline_put_b(lines, (uint32_t)s, 2, idx, njobs, c3.c0);
    evline_put_b(lines, (uint32_t)s, 3, idx, njobs, c3.c1);
    evline_put_b(lines, (uint32_t)s, 4, idx, njobs, c4.c0);
    evline_put_b(lines, (uint32_t)s, 5, idx, njobs, c4.c1);
  }
}

}  // namespace fts

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

#ifndef FTS_G2L_FUSED
#define FTS_G2L_FUSED 0  // 1: the addition step's two sums of two products with one reduction each (stage -2%, device-only -2.5% on one box: off)
#endif

// Constants of the line chain in the balanced R = 2^261 form (from
// dev/constants.h by q2_from_fp2 / f29_breduce; tests/native/sx_emu.cpp
// sxe_g2l29_consts re-derives them): 3 b' (b' = 3 / (9 + u)), the twist
// Frobenius factors of pi(Q) and -pi^2(Q), one.  As literals they are scalar
// operands, not lane VGPRs.
static constexpr int32_t G2L29_CONST[9][9] = {
  {-253769606, 6731155, -156399417, 46225477, -175165556, 162336334, -209914092, -192467748, -1389658},  // 3 b' c0
  {31837202, -172120824, -128414024, 15984953, -118312780, 62914239, -210424777, 247765560, 1563920},  // 3 b' c1
  {203985993, 99656738, 260427116, -196420981, 88012806, 31651349, 187173606, 203914975, -774555},  // TW_FROB_X c0
  {-250335503, 187804872, -44558148, -133497832, -94169217, -176792772, -242256849, 104485019, 1269326},  // TW_FROB_X c1
  {44173617, 40868432, -156996498, -175615513, 213596584, -200916108, -28519026, -208385841, -1252753},  // TW_FROB_Y c0
  {-106543147, -100798548, -40739557, 220163168, 145517765, -5938662, -212924673, 161949719, 1410845},  // TW_FROB_Y c1
  {-120801391, -145023941, 193189603, 244240497, -226312478, 69340805, -1834625, -184005301, 1478938},  // TW_FROB2_X
  {176370655, 199481511, 128831276, -21759002, -178483129, 45989682, 237679608, -86689705, -903222},  // TW_FROB2_Y
  {-176370655, -199481511, -128831276, 21759002, 178483129, -45989682, -237679608, 86689705, 903222},  // one
};
enum { G2C_B3 = 0, G2C_FX = 2, G2C_FY = 4, G2C_F2X = 6, G2C_F2Y = 7, G2C_ONE = 8 };
FTS_HD f29 g2c_f(int i) {
  f29 r;
#pragma unroll
  for (int k = 0; k < 9; k++) r.l[k] = G2L29_CONST[i][k];
  return r;
}
FTS_HD q2 g2c_q(int i) { return {g2c_f(i), g2c_f(i + 1)}; }
FTS_HD q2 q2_one29() { return {g2c_f(G2C_ONE), q2_zero().c1}; }

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

// Each step hands its three evaluated coefficients to emit(c, value) (c = 0:
// c0, 1: c3, 2: c4) as soon as they are formed, so that none of them stays live
// through the rest of the step.
//
// T <- 4 (2T) = 2T; the line (-H, 3J, I) evaluated: c0 = -H yP, c3 = 3 X^2 xP,
// c4 = E - B
template <class Emit>
FTS_HD void g2l_dbl(q2& X, q2& Y, q2& Z, const f29& yP, const f29& xP, const Emit& emit) {
  const q2 B = q2_sqrb(Y);
  const q2 C = q2_sqrb(Z);
  const q2 H = q2_lin3b(q2_sqrb(q2_lin2b(Y, 1, Z, 1)), 1, B, -1, C, -1);  // 2 Y Z
  emit(0, q2_mulfb(q2_neg(H), yP));
  emit(1, q2_scaleb(q2_mulfb(q2_sqrb(X), xP), 3));
  const q2 E = q2_mulb(C, g2c_q(G2C_B3));  // 3 b' Z^2
  emit(2, q2_lin2b(E, 1, B, -1));
  X = q2_scaleb(q2_mulb(q2_mulb(X, Y), q2_lin2b(B, 1, E, -3)), 2);
  Y = q2_lin2b(q2_sqrb(q2_lin2b(B, 1, E, 3)), 1, q2_sqrb(E), -12);
  Z = q2_scaleb(q2_mulb(B, H), 4);
}

// T <- T + (Qx, Qy) (affine, balanced); the line (L, -O, Qx O - L Qy)
// evaluated: c0 = L yP, c3 = -O xP, c4 = Qx O - L Qy
template <class Emit>
FTS_HD void g2l_add(q2& X, q2& Y, q2& Z, const q2& Qx, const q2& Qy, const f29& yP, const f29& xP,
                    const Emit& emit) {
  const q2 O = q2_lin2b(Y, 1, q2_mulb(Qy, Z), -1);
  const q2 L = q2_lin2b(X, 1, q2_mulb(Qx, Z), -1);
  emit(0, q2_mulfb(L, yP));
  emit(1, q2_mulfb(q2_neg(O), xP));
#if FTS_G2L_FUSED
  emit(2, q2_mul2b(Qx, O, L, q2_neg(Qy)));
#else
  emit(2, q2_lin2b(q2_mulb(Qx, O), 1, q2_mulb(L, Qy), -1));
#endif
  const q2 D = q2_sqrb(L);
  const q2 E = q2_mulb(L, D);
  const q2 G = q2_mulb(X, D);
  const q2 H = q2_lin3b(E, 1, G, -2, q2_mulb(Z, q2_sqrb(O)), 1);
#if FTS_G2L_FUSED
  const q2 Y3 = q2_mul2b(q2_subr(G, H), O, Y, q2_neg(E));  // one reduction for the two products
#else
  const q2 Y3 = q2_lin2b(q2_mulb(q2_subr(G, H), O), 1, q2_mulb(Y, E), -1);
#endif
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

// The four partial sums of t' added in the 32-bit Jacobian form and written
// over part 0, and the norm N(Z) = Z0^2 + Z1^2 of the sum (in Fp, zero only
// for Z = 0: -1 is not a square mod p) parked in part 1's first eight words,
// for the launch's batched inversion (k_g2_sum, k_g2_binv, dev/binv.h)
FTS_HD void job_g2_sum(G2PartDev* part, uint32_t idx, uint32_t njobs) {
  g2j acc = g2part_load(part[idx]);
#pragma nounroll
  for (int q = 1; q < 4; q++) acc = jac_add_inl(acc, g2part_load(part[(size_t)q * njobs + idx]));
  g2part_store(part[idx], acc);
  const fp nz = fe_sqr(acc.z.c0) + fe_sqr(acc.z.c1);
#pragma unroll
  for (int i = 0; i < 8; i++) part[njobs + idx].w[i] = nz.v[i];
}
// t' in affine form from the sum and N(Z)^-1 (part 1 after k_g2_binv):
// Z^-1 = conj(Z) N(Z)^-1, as f2_inv_inl, then jac_to_aff_inl's products
FTS_HD g2a g2_sum_aff(const G2PartDev* part, uint32_t idx, uint32_t njobs) {
  const g2j acc = g2part_load(part[idx]);
  g2a r;
  if (is_zero(acc.z)) {
    r.x = zero_of<fp2>();
    r.y = zero_of<fp2>();
    r.inf = true;
    return r;
  }
  fp ni;
#pragma unroll
  for (int i = 0; i < 8; i++) ni.v[i] = part[njobs + idx].w[i];
  const fp2 zi = {acc.z.c0 * ni, fe_neg(acc.z.c1 * ni)};
  const fp2 zi2 = sqr(zi);
  r.x = acc.x * zi2;
  r.y = acc.y * zi2 * zi;
  r.inf = false;
  return r;
}

// job_g2lines_parts (dev/jobs.h) with the line chain on this form: t' (Q,
// affine) is written to the G2 output, then the lines
FTS_HD void g2lines_chain_x29(const g2a& Q, const G2Job& g, const PairJob& j, G2Dev* g2out, const G1Dev* pts,
                              EvLineDev* lines, uint32_t idx, uint32_t njobs) {
  G2Dev d;
  g2_store(d, Q);
  g2out[g.out] = d;
  const g1a P = g1_load(pts[j.p2]);
  const bool use = !(P.inf || Q.inf);
  const f29 yP = f29_breduce(f29_from_fp(P.y)), xP = f29_breduce(f29_from_fp(P.x));
  const q2 Qx = q2_from_fp2(Q.x), Qy = q2_from_fp2(Q.y);
  q2 X = Qx, Y = Qy, Z = q2_one29();
#pragma nounroll
  for (int s = 0; s < MILLER_LINES; s++) {
    const int t = MILLER_STEPS.t[s];
    // a pair with an infinity point contributes 1 (gnark's MillerLoop skips it)
    auto emit = [&](int c, const q2& v) {
      const q2 w = use ? v : (c == 0 ? q2_one29() : q2_zero());
      evline_put_b(lines, (uint32_t)s, 2 * c, idx, njobs, w.c0);
      evline_put_b(lines, (uint32_t)s, 2 * c + 1, idx, njobs, w.c1);
    };
    if (t == STEP_DBL) {
      g2l_dbl(X, Y, Z, yP, xP, emit);
    } else {
      q2 Ax = Qx, Ay = Qy;
      if (t == STEP_FROB1 || t == STEP_FROB2) {
        // t' re-read from the output just written (this lane's own store): no
        // 32-bit copy of it stays live through the loop
        const g2a Qr = g2_load(g2out[g.out]);
        const g2a A = t == STEP_FROB1 ? tw_frob(Qr) : tw_frob2_neg(Qr);
        Ax = q2_from_fp2(A.x);
        Ay = q2_from_fp2(A.y);
      } else if (t == STEP_SUB) {
        Ay = q2_neg(Qy);
      }
      g2l_add(X, Y, Z, Ax, Ay, yP, xP, emit);
    }
  }
}
// the four partial sums added and normalised in the 32-bit code (one
// inversion per lane), then the chain
FTS_HD void job_g2lines_parts_x29(const G2Job& g, const PairJob& j, const G2PartDev* part, G2Dev* g2out,
                                  const G1Dev* pts, EvLineDev* lines, uint32_t idx, uint32_t njobs) {
  g2j acc = g2part_load(part[idx]);
#pragma nounroll
  for (int q = 1; q < 4; q++) acc = jac_add_inl(acc, g2part_load(part[(size_t)q * njobs + idx]));
  g2lines_chain_x29(jac_to_aff_inl(acc), g, j, g2out, pts, lines, idx, njobs);
}
// the same after job_g2_sum and the batched inversion
FTS_HD void job_g2lines_summed_x29(const G2Job& g, const PairJob& j, const G2PartDev* part, G2Dev* g2out,
                                   const G1Dev* pts, EvLineDev* lines, uint32_t idx, uint32_t njobs) {
  g2lines_chain_x29(g2_sum_aff(part, idx, njobs), g, j, g2out, pts, lines, idx, njobs);
}

}  // namespace fts

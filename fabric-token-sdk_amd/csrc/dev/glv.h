// GLV scalar split on BN254 G1 (phi(x, y) = (beta x, y) = [lambda] P), shared
// by the zkatdlog jobs (jobs.h g1_mul_glv*) and the BN254 idemix host planner
// (host/idemix.cpp nym_glv_split_bn).
#pragma once
#include "curve.h"
#include "fp_wide.h"

namespace fts {

// r[na + nb] = a[na] * b[nb]  (schoolbook, small operands)
FTS_HD void mul_small(uint32_t* r, const uint32_t* a, int na, const uint32_t* b, int nb) {
  for (int i = 0; i < na + nb; i++) r[i] = 0;
  for (int i = 0; i < na; i++) {
    uint32_t c = 0;
    for (int j = 0; j < nb; j++) {
      uint64_t t = (uint64_t)a[i] * b[j] + r[i + j] + c;
      r[i + j] = (uint32_t)t;
      c = (uint32_t)(t >> 32);
    }
    r[i + nb] = c;
  }
}

// k = k1 + k2 lambda (mod r) with |k1|, |k2| < 2^128 (constants from
// gen_constants.py: c1 = (k g1) >> 256, c2 = (k g2) >> 256, k2 = c1 |b1| - c2 b2,
// k1 = k - k2 lambda mod r taken in (-r/2, r/2]).
FTS_HD void glv_split(const uint32_t k[8], uint32_t k1[4], bool& n1, uint32_t k2[4], bool& n2) {
  uint32_t g[8], w[16], c1[4], c2[4];
  for (int i = 0; i < 8; i++) g[i] = GLV_G1[i];
  mul_wide(w, k, g);
  for (int i = 0; i < 4; i++) c1[i] = w[8 + i];
  for (int i = 0; i < 8; i++) g[i] = GLV_G2[i];
  mul_wide(w, k, g);
  for (int i = 0; i < 4; i++) c2[i] = w[8 + i];
  uint32_t b1[2] = {GLV_B1ABS[0], GLV_B1ABS[1]}, b2[4] = {GLV_B2[0], GLV_B2[1], GLV_B2[2], GLV_B2[3]};
  uint32_t t1[6], t2[6], d[6];
  mul_small(t1, c1, 4, b1, 2);
  mul_small(t2, c2, 2, b2, 4);
  uint32_t br = 0;
  for (int i = 0; i < 6; i++) d[i] = subb32(t1[i], t2[i], br, &br);
  n2 = br != 0;  // |t1 - t2| < 2^128 <<< 2^192: the borrow is the sign
  if (n2) {
    uint32_t c = 1;
    for (int i = 0; i < 6; i++) d[i] = addc32(~d[i], 0, c, &c);
  }
  for (int i = 0; i < 4; i++) k2[i] = d[i];
  // k1 = k - k2 lambda  (mod r)
  uint32_t k2f[8] = {k2[0], k2[1], k2[2], k2[3], 0, 0, 0, 0};
  fr t = fe_from_int<ModR>(k2f) * fe_const<ModR>(GLV_LAMBDA);
  fr K = fe_from_int<ModR>(k);
  fr r1 = n2 ? K + t : K - t;
  uint32_t v[8], u[8], h[8], rm[8];
  fe_to_int(v, r1);
  for (int i = 0; i < 8; i++) {
    h[i] = R_HALF[i];
    rm[i] = R_MOD[i];
  }
  n1 = sub8(u, h, v) != 0;  // v > (r-1)/2
  if (n1) sub8(v, rm, v);
  for (int i = 0; i < 4; i++) k1[i] = v[i];
}

}  // namespace fts

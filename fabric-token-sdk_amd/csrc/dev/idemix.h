// Idemix owner-signature verification job: IBM/idemix
// NymSignature.Ver on FP256BN, one lane per signature.  The reference calls it
// per input token from TransferSignatureValidate
// (zkatdlog/crypto/validator/validator_transfer.go:42-82) through
// identity/msp/idemix/deserializer.go:153-163 Verifier.Verify.  [EXT] IBM/idemix
// v0.0.0-20220113150823-80dd4cb2d74e (go.mod:6), restated:
//   t = HSk^ProofSSk * HRand^ProofSRNym * Nym^-ProofC
//   c = HashToZr("sign" || t || Nym || ipk.Hash || msg)     (G1 = 0x04||X||Y)
//   accept  <=>  ProofC == HashToZr(c || Nonce)            (raw 32-byte integers)
// The host (host/idemix.cpp) decodes the owner identity and the signature proto
// and lays out per signature: the six 32-byte integers, a 176-byte transcript
// prefix slot ("sign" and the IPK hash already in place) and the message.
#pragma once
#include "fp256bn.h"
#include "sha256.h"

namespace fts {

// fixed-base tables of HSk and HRand: NYM_WINDOWS windows of 8 bits, entries
// d * 2^(8w) * H for d = 1..255, Montgomery affine (never infinity: d 2^(8w) < n)
static constexpr int NYM_WBITS = 8;
static constexpr int NYM_WINDOWS = 32;
static constexpr int NYM_TAB_PER_BASE = NYM_WINDOWS * 255;
struct QDev {
  uint32_t x[8], y[8];
};

struct NymJob {
  uint32_t sc;       // blob offset (16-aligned) of NYM_SC_BYTES: NymX, NymY, ProofC, ProofSSk, ProofSRNym, Nonce
                     // (32 bytes BE each), then the GLV split of ProofC (12 u32, host/idemix.h nym_glv_split)
  uint32_t pre;      // blob offset (16-aligned) of the transcript prefix: "sign" | t (65) | Nym (65) | hash (32)
  uint32_t msg;      // blob offset of the message, = 6 mod 16 so that stream byte 192 is 16-aligned
  uint32_t msg_len;
};
static constexpr uint32_t NYM_PRE = 4 + 65 + 65 + 32;  // 166
static constexpr uint32_t NYM_SC_BYTES = 240;
struct QJDev {
  uint32_t x[8], y[8], z[8];
};

FTS_HD q1a q1_load(const QDev& d) {
  q1a a;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a.x.v[i] = d.x[i];
    a.y.v[i] = d.y[i];
  }
  a.inf = false;
  return a;
}

FTS_HD void q1_store(QDev& d, const q1a& a) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    d.x[i] = a.x.v[i];
    d.y[i] = a.y.v[i];
  }
}

// amcl ECP.ToBytes(b, false): 0x04 || X || Y; the point at infinity as amcl's
// (0, 1) representative [EXT]
FTS_HD void q1_bytes65(uint8_t* out, const q1a& a) {
  uint32_t x[8], y[8];
  if (a.inf) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      x[i] = 0;
      y[i] = i == 0;
    }
  } else {
    fq_to_int(x, a.x);
    fq_to_int(y, a.y);
  }
  out[0] = 0x04;
  limbs_to_be32(out + 1, x);
  limbs_to_be32(out + 33, y);
}

// sum over the 32 byte-windows of k of tab[w][byte_w - 1]
FTS_HD q1j q1_fixed_mul(const QDev* tab, const uint32_t k[8]) {
  q1j acc = jac_inf<fq>();
#pragma nounroll
  for (int w = 0; w < NYM_WINDOWS; w++) {
    uint32_t d = (k[w >> 2] >> (8 * (w & 3))) & 0xffu;
    if (d) acc = jac_add_aff(acc, q1_load(tab[w * 255 + d - 1]));
  }
  return acc;
}

// NewECPbigs(x, y) of the nym: coordinates mod q, off-curve -> infinity
FTS_HD q1a nym_load(const uint8_t* sc) {
  uint32_t x[8], y[8];
  be32_to_limbs_g(x, sc);
  be32_to_limbs_g(y, sc + 32);
  q1a nym;
  nym.x = fq_from_int(x);
  nym.y = fq_from_int(y);
  nym.inf = false;
  if (!q1_on_curve(nym)) nym.inf = true;
  return nym;
}

// Part `part` (0..3) of t = s_sk HSk + s_rnym HRand - c Nym, four lanes per
// signature: with -c = k1 + k2 lambda (GLV, split on the host) part 0 computes
// k1 (-Nym) and part 1 k2 phi(-Nym) (129-bit double-and-add with mixed
// additions), part 2 s_sk HSk and part 3 s_rnym HRand (32 fixed-base table
// additions each).
FTS_HD q1j job_nym_part(const NymJob& j, const uint8_t* blob, const QDev* tab, uint32_t part) {
  const uint8_t* sc = blob + j.sc;
  if (part >= 2) {
    uint32_t s[8];
    be32_to_limbs_g(s, sc + (part == 3 ? 128 : 96));
    return q1_fixed_mul(tab + (part - 2) * NYM_TAB_PER_BASE, s);
  }
  q1a P = aff_neg(nym_load(sc));
  const uint32_t* glv = reinterpret_cast<const uint32_t*>(sc + 192);
  uint32_t k[5];
#pragma unroll
  for (int i = 0; i < 5; i++) k[i] = glv[5 * part + i];
  if (part) P.x = P.x * fq_const(Q_GLV_BETA);
  if ((glv[10] >> part) & 1) P = aff_neg(P);
  q1j acc = jac_inf<fq>();
  if (P.inf) return acc;
  // bits 128..0, consumed from the top by shifting (a dynamically indexed limb
  // array would live in scratch memory)
  uint32_t u0 = k[0], u1 = k[1], u2 = k[2], u3 = k[3], u4 = k[4];
#pragma nounroll
  for (int i = 128; i >= 0; i--) {
    acc = jac_dbl(acc);
    uint32_t bit = u4 & 1;
    u4 = u3 >> 31;
    u3 = (u3 << 1) | (u2 >> 31);
    u2 = (u2 << 1) | (u1 >> 31);
    u1 = (u1 << 1) | (u0 >> 31);
    u0 <<= 1;
    if (bit) acc = jac_add_aff(acc, P);
  }
  return acc;
}

// The rest of NymSignature.Ver for one signature given t in Jacobian form:
// 1 = accept, 0 = "pseudonym signature invalid".  The prefix slot at
// blob + j.pre receives t and Nym (device-computed bytes).
FTS_HD uint8_t job_nym_fin(const NymJob& j, uint8_t* blob, const q1j& tj) {
  const uint8_t* sc = blob + j.sc;
  q1a t = jac_to_aff(tj);
  uint8_t* pre = blob + j.pre;
  q1_bytes65(pre + 4, t);
  q1_bytes65(pre + 69, nym_load(sc));
  Sha256 s;
  s.init();
  s.update(pre, NYM_PRE);
  uint32_t head = j.msg_len < 26 ? j.msg_len : 26;  // completes the third block
  s.update(blob + j.msg, head);
  s.update(blob + j.msg + head, j.msg_len - head);
  uint8_t d[32];
  s.final(d);
  uint32_t c[8], v[8];
  digest_mod_n(c, d);
  // ProofC == HashToZr(c || Nonce), Nonce as its raw 32 bytes
  uint8_t cb[64];
  limbs_to_be32(cb, c);
  be32_to_limbs_g(v, sc + 160);
  limbs_to_be32(cb + 32, v);
  s.init();
  s.update(cb, 64);
  s.final(d);
  digest_mod_n(c, d);
  be32_to_limbs_g(v, sc + 64);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= c[i] ^ v[i];
  return o == 0 ? 1 : 0;
}

FTS_HD void qj_store(QJDev& d, const q1j& p) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    d.x[i] = p.x.v[i];
    d.y[i] = p.y.v[i];
    d.z[i] = p.z.v[i];
  }
}
FTS_HD q1j qj_load(const QJDev& d) {
  q1j p;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    p.x.v[i] = d.x[i];
    p.y.v[i] = d.y[i];
    p.z.v[i] = d.z[i];
  }
  return p;
}

// Auditor owner match (AuditInfo.Match -> IBM/idemix AuditNymEid [EXT]), one
// lane per token: HAttrs[2]^HashToZr(eid) * HRand^RNymEid == EidNym.Nym.  The
// job's 128 bytes: SHA-256(eid), RNymEid, EidNym X, EidNym Y (32 bytes BE each,
// host/idemix.cpp decode_owner_audit).  Returns 1 on a match.
static constexpr uint32_t EID_JOB_BYTES = 128;
static constexpr int NYM_TAB_HEID = 2;  // table index of HAttrs[2] (HSk 0, HRand 1)
FTS_HD uint8_t job_eid(const uint8_t* in, const QDev* tab) {
  uint32_t h[8], r[8];
  digest_mod_n(h, in);
  be32_to_limbs_g(r, in + 32);
  q1j p = jac_add(q1_fixed_mul(tab + NYM_TAB_HEID * NYM_TAB_PER_BASE, h), q1_fixed_mul(tab + NYM_TAB_PER_BASE, r));
  q1a e = nym_load(in + 64);  // NewECPbigs: off-curve -> infinity
  if (is_zero(p.z) || e.inf) return (is_zero(p.z) && e.inf) ? 1 : 0;
  // X == x Z^2 and Y == y Z^3 (amcl ECP.Equals)
  fq z2 = sqr(p.z);
  fq dx = p.x - e.x * z2, dy = p.y - e.y * z2 * p.z;
  return (is_zero(dx) && is_zero(dy)) ? 1 : 0;
}

// Host: the fixed-base tables of HSk, HRand and HAttrs[2] (tab[b * NYM_TAB_PER_BASE +
// w * 255 + d - 1] = d 2^(8w) H_b), built once per issuer key.  Window bases by
// doublings, entries by mixed additions, one batch inversion per window.
inline void nym_build_tables(const q1a* bases, int nb, QDev* tab) {
  for (int b = 0; b < nb; b++) {
    q1a bw = bases[b];
    for (int w = 0; w < NYM_WINDOWS; w++) {
      q1j e[255];
      e[0] = jac_from_aff(bw);
      for (int d = 1; d < 255; d++) e[d] = jac_add_aff(e[d - 1], bw);
      // batch inversion of the 255 Z coordinates (none is zero: d 2^(8w) < n)
      fq pre[255];
      pre[0] = e[0].z;
      for (int d = 1; d < 255; d++) pre[d] = pre[d - 1] * e[d].z;
      fq inv_all = inv(pre[254]);
      for (int d = 254; d >= 0; d--) {
        fq zi = d ? inv_all * pre[d - 1] : inv_all;
        if (d) inv_all = inv_all * e[d].z;
        fq zi2 = sqr(zi);
        q1a a;
        a.x = e[d].x * zi2;
        a.y = e[d].y * zi2 * zi;
        a.inf = false;
        q1_store(tab[b * NYM_TAB_PER_BASE + w * 255 + d], a);
      }
      // next window base: 2^8 bw
      q1j nb = jac_from_aff(bw);
      for (int k = 0; k < NYM_WBITS; k++) nb = jac_dbl(nb);
      bw = jac_to_aff(nb);
    }
  }
}

// 32 big-endian bytes -> Montgomery affine point (amcl NewECPbigs); false if
// off the curve
inline bool nym_point_from_be(const uint8_t* xb, const uint8_t* yb, q1a& out) {
  uint32_t x[8], y[8];
  be32_to_limbs(x, xb);
  be32_to_limbs(y, yb);
  out.x = fq_from_int(x);
  out.y = fq_from_int(y);
  out.inf = false;
  return q1_on_curve(out);
}

}  // namespace fts

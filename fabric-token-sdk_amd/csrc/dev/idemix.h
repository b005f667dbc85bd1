// Idemix owner-signature verification job: IBM/idemix
// NymSignature.Ver, one lane per signature, on either idemix curve the
// reference's deserializer accepts (identity/msp/idemix/deserializer.go:40-51):
// FP256BN_AMCL (amcl translator; the unit tests' keys) and BN254 (gurvy
// translator; what cmd/pp/dlog/gen.go:117 and every NWO topology deploy).  The
// reference calls it per input token from TransferSignatureValidate
// (zkatdlog/crypto/validator/validator_transfer.go:42-82) through
// identity/msp/idemix/deserializer.go:153-163 Verifier.Verify.  [EXT] IBM/idemix
// v0.0.0-20220113150823-80dd4cb2d74e (go.mod:6), restated:
//   t = HSk^ProofSSk * HRand^ProofSRNym * Nym^-ProofC
//   c = HashToZr("sign" || t || Nym || ipk.Hash || msg)
//   accept  <=>  ProofC == HashToZr(c || Nonce)
// The G1 encoding inside the transcript is the curve's Bytes(): amcl 0x04||X||Y
// (65 bytes) on FP256BN, gnark RawBytes X||Y (64 bytes) on BN254, in a buffer
// sized for 65-byte points either way (so BN254 leaves 2 trailing bytes).
// The host (host/idemix.cpp) decodes the owner identity and the signature proto
// and lays out per signature: the six 32-byte integers, a 176-byte transcript
// prefix slot ("sign", the IPK hash and, on BN254, the 2 tail bytes already in
// place) and the message.  The group law is curve.h's, written once over the
// coordinate field (fq: FP256BN, fp: BN254); NymCurve<F> below supplies the
// per-curve pieces.
#pragma once
#include "fp256bn.h"
#include "glv.h"
#include "sha256.h"

namespace fts {

// fixed-base tables of HSk and HRand: NYM_WINDOWS windows of 8 bits, entries
// d * 2^(8w) * H for d = 1..255, Montgomery affine (never infinity: d 2^(8w) is
// below 2^256 and no multiple of the prime group order)
static constexpr int NYM_WBITS = 8;
static constexpr int NYM_WINDOWS = 32;
static constexpr int NYM_TAB_PER_BASE = NYM_WINDOWS * 255;
struct QDev {
  uint32_t x[8], y[8];
};

struct NymJob {
  uint32_t sc;       // blob offset (16-aligned) of NYM_SC_BYTES: NymX, NymY, ProofC, ProofSSk, ProofSRNym, Nonce
                     // (32 bytes BE each), then the GLV split of ProofC (12 u32, host/idemix.h nym_glv_split)
  uint32_t pre;      // blob offset (16-aligned) of the 176-byte transcript prefix slot
  uint32_t msg;      // blob offset of the message, = NymCurve<F>::PRE mod 16 so that stream byte 192 is 16-aligned
  uint32_t msg_len;
};
static constexpr uint32_t NYM_SC_BYTES = 240;
static constexpr uint32_t NYM_PRE_SLOT = 176;
struct QJDev {
  uint32_t x[8], y[8], z[8];
};

template <class F>
struct NymCurve;

// FP256BN_AMCL (amcl translator): nym coordinates arrive as raw FromBytes
// integers and are read by NewECPbigs (mod q, off-curve -> infinity [EXT]);
// ProofC is split as k mod n; the transcript point is 0x04||X||Y.
template <>
struct NymCurve<fq> {
  static constexpr uint32_t G1_BYTES = 65;
  static constexpr uint32_t PRE = 4 + 65 + 65 + 32;  // 166: the message follows directly
  static constexpr uint32_t TAIL = 0;
  FTS_HD static fq beta() { return fq_const(Q_GLV_BETA); }
  FTS_HD static fq from_canon(const uint32_t a[8]) { return fq_from_int(a); }
  FTS_HD static void to_int(uint32_t out[8], const fq& a) { fq_to_int(out, a); }
  FTS_HD static bool on_curve(const Aff<fq>& a) { return q1_on_curve(a); }
  FTS_HD static void digest_mod(uint32_t out[8], const uint8_t d[32]) { digest_mod_n(out, d); }
  // NewECPbigs(x, y) of 32-byte big-endian integers: coordinates mod q, off-curve -> infinity
  FTS_HD static Aff<fq> load_point(const uint8_t* xy) {
    uint32_t x[8], y[8];
    be32_to_limbs_g(x, xy);
    be32_to_limbs_g(y, xy + 32);
    Aff<fq> p;
    p.x = fq_from_int(x);
    p.y = fq_from_int(y);
    p.inf = false;
    if (!q1_on_curve(p)) p.inf = true;
    return p;
  }
  // amcl ECP.ToBytes(b, false): 0x04 || X || Y; infinity as amcl's (0, 1) representative [EXT]
  FTS_HD static void point_bytes(uint8_t* out, const Aff<fq>& a) {
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
};

// BN254 (gurvy translator): the host decodes every point with gnark SetBytes
// (G1FromProto) and hands over canonical coordinates, all-zero for infinity;
// scalars arrive reduced mod r; the transcript point is RawBytes X||Y.
template <>
struct NymCurve<fp> {
  static constexpr uint32_t G1_BYTES = 64;
  static constexpr uint32_t PRE = 4 + 64 + 64 + 32;  // 164, then the message, then TAIL bytes
  // proofData is sized for 65-byte points, so two zero bytes follow the message
  // [EXT, parity unpinned: the issuer key's own proof uses the same sizing, no
  // reference file holds a BN254 NymSignature]
  static constexpr uint32_t TAIL = 2;
  FTS_HD static fp beta() { return fe_const<ModP>(GLV_BETA); }
  FTS_HD static fp from_canon(const uint32_t a[8]) { return fe_from_int<ModP>(a); }
  FTS_HD static void to_int(uint32_t out[8], const fp& a) { fe_to_int(out, a); }
  FTS_HD static bool on_curve(const Aff<fp>& a) { return g1_on_curve(a); }
  FTS_HD static void digest_mod(uint32_t out[8], const uint8_t d[32]) { digest_mod_r(out, d); }
  FTS_HD static Aff<fp> load_point(const uint8_t* xy) {
    uint32_t x[8], y[8];
    be32_to_limbs_g(x, xy);
    be32_to_limbs_g(y, xy + 32);
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) o |= x[i] | y[i];
    Aff<fp> p;
    p.x = fe_from_int<ModP>(x);
    p.y = fe_from_int<ModP>(y);
    p.inf = o == 0;
    return p;
  }
  FTS_HD static void point_bytes(uint8_t* out, const Aff<fp>& a) { g1_to_bytes(out, a); }
};

template <class F>
FTS_HD Aff<F> q1_load(const QDev& d) {
  Aff<F> a;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a.x.v[i] = d.x[i];
    a.y.v[i] = d.y[i];
  }
  a.inf = false;
  return a;
}

template <class F>
FTS_HD void q1_store(QDev& d, const Aff<F>& a) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    d.x[i] = a.x.v[i];
    d.y[i] = a.y.v[i];
  }
}

// sum over the 32 byte-windows of k of tab[w][byte_w - 1]
template <class F>
FTS_HD Jac<F> q1_fixed_mul(const QDev* tab, const uint32_t k[8]) {
  Jac<F> acc = jac_inf<F>();
#pragma nounroll
  for (int w = 0; w < NYM_WINDOWS; w++) {
    uint32_t d = (k[w >> 2] >> (8 * (w & 3))) & 0xffu;
    if (d) acc = jac_add_aff(acc, q1_load<F>(tab[w * 255 + d - 1]));
  }
  return acc;
}

// Part `part` (0..3) of t = s_sk HSk + s_rnym HRand - c Nym, four lanes per
// signature: with -c = k1 + k2 lambda (GLV, split on the host) part 0 computes
// k1 (-Nym) and part 1 k2 phi(-Nym) (129-bit double-and-add with mixed
// additions), part 2 s_sk HSk and part 3 s_rnym HRand (32 fixed-base table
// additions each).
template <class F>
FTS_HD Jac<F> job_nym_part(const NymJob& j, const uint8_t* blob, const QDev* tab, uint32_t part) {
  const uint8_t* sc = blob + j.sc;
  if (part >= 2) {
    uint32_t s[8];
    be32_to_limbs_g(s, sc + (part == 3 ? 128 : 96));
    return q1_fixed_mul<F>(tab + (part - 2) * NYM_TAB_PER_BASE, s);
  }
  Aff<F> P = aff_neg(NymCurve<F>::load_point(sc));
  const uint32_t* glv = reinterpret_cast<const uint32_t*>(sc + 192);
  uint32_t k[5];
#pragma unroll
  for (int i = 0; i < 5; i++) k[i] = glv[5 * part + i];
  if (part) P.x = P.x * NymCurve<F>::beta();
  if ((glv[10] >> part) & 1) P = aff_neg(P);
  Jac<F> acc = jac_inf<F>();
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
template <class F>
FTS_HD uint8_t job_nym_fin(const NymJob& j, uint8_t* blob, const Jac<F>& tj) {
  typedef NymCurve<F> C;
  const uint8_t* sc = blob + j.sc;
  Aff<F> t = jac_to_aff(tj);
  uint8_t* pre = blob + j.pre;
  C::point_bytes(pre + 4, t);
  C::point_bytes(pre + 4 + C::G1_BYTES, C::load_point(sc));
  Sha256 s;
  s.init();
  s.update(pre, C::PRE);
  uint32_t head = j.msg_len < 192 - C::PRE ? j.msg_len : 192 - C::PRE;  // completes the third block
  s.update(blob + j.msg, head);
  s.update(blob + j.msg + head, j.msg_len - head);
  if (C::TAIL) s.update(pre + C::PRE, C::TAIL);
  uint8_t d[32];
  s.final(d);
  uint32_t c[8], v[8];
  C::digest_mod(c, d);
  // ProofC == HashToZr(c || Nonce), Nonce as its 32 bytes
  uint8_t cb[64];
  limbs_to_be32(cb, c);
  be32_to_limbs_g(v, sc + 160);
  limbs_to_be32(cb + 32, v);
  s.init();
  s.update(cb, 64);
  s.final(d);
  C::digest_mod(c, d);
  be32_to_limbs_g(v, sc + 64);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= c[i] ^ v[i];
  return o == 0 ? 1 : 0;
}

template <class F>
FTS_HD void qj_store(QJDev& d, const Jac<F>& p) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    d.x[i] = p.x.v[i];
    d.y[i] = p.y.v[i];
    d.z[i] = p.z.v[i];
  }
}
template <class F>
FTS_HD Jac<F> qj_load(const QJDev& d) {
  Jac<F> p;
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
template <class F>
FTS_HD uint8_t job_eid(const uint8_t* in, const QDev* tab) {
  uint32_t h[8], r[8];
  NymCurve<F>::digest_mod(h, in);
  be32_to_limbs_g(r, in + 32);
  Jac<F> p = jac_add(q1_fixed_mul<F>(tab + NYM_TAB_HEID * NYM_TAB_PER_BASE, h), q1_fixed_mul<F>(tab + NYM_TAB_PER_BASE, r));
  Aff<F> e = NymCurve<F>::load_point(in + 64);
  if (is_zero(p.z) || e.inf) return (is_zero(p.z) && e.inf) ? 1 : 0;
  // X == x Z^2 and Y == y Z^3 (ECP.Equals / G1Jac.Equal)
  F z2 = sqr(p.z);
  F dx = p.x - e.x * z2, dy = p.y - e.y * z2 * p.z;
  return (is_zero(dx) && is_zero(dy)) ? 1 : 0;
}

// Host: the fixed-base tables of HSk, HRand and HAttrs[2] (tab[b * NYM_TAB_PER_BASE +
// w * 255 + d - 1] = d 2^(8w) H_b), built once per issuer key.  Window bases by
// doublings, entries by mixed additions, one batch inversion per window.  The
// bases must not be the point at infinity.
template <class F>
inline void nym_build_tables(const Aff<F>* bases, int nb, QDev* tab) {
  for (int b = 0; b < nb; b++) {
    Aff<F> bw = bases[b];
    for (int w = 0; w < NYM_WINDOWS; w++) {
      Jac<F> e[255];
      e[0] = jac_from_aff(bw);
      for (int d = 1; d < 255; d++) e[d] = jac_add_aff(e[d - 1], bw);
      // batch inversion of the 255 Z coordinates (none is zero, see above)
      F pre[255];
      pre[0] = e[0].z;
      for (int d = 1; d < 255; d++) pre[d] = pre[d - 1] * e[d].z;
      F inv_all = inv(pre[254]);
      for (int d = 254; d >= 0; d--) {
        F zi = d ? inv_all * pre[d - 1] : inv_all;
        if (d) inv_all = inv_all * e[d].z;
        F zi2 = sqr(zi);
        Aff<F> a;
        a.x = e[d].x * zi2;
        a.y = e[d].y * zi2 * zi;
        a.inf = false;
        q1_store(tab[b * NYM_TAB_PER_BASE + w * 255 + d], a);
      }
      // next window base: 2^8 bw
      Jac<F> nbj = jac_from_aff(bw);
      for (int k = 0; k < NYM_WBITS; k++) nbj = jac_dbl(nbj);
      bw = jac_to_aff(nbj);
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

// Gurvy G1FromProto on 32-byte X and Y (gnark SetBytes of X || Y): false on a
// decoding error
inline bool bn_point_from_xy(const uint8_t* xb, const uint8_t* yb, g1a& out) {
  uint8_t b[64];
  for (int i = 0; i < 32; i++) {
    b[i] = xb[i];
    b[32 + i] = yb[i];
  }
  return g1_setbytes(b, 64, out);
}

}  // namespace fts

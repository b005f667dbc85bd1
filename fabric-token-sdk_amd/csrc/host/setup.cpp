// crypto.Setup natively: the public parameters of the
// zkatdlog driver, as /root/reference/token/core/zkatdlog/crypto/setup.go:214-236
// SetupWithCustomLabel builds them --
//   pssign.NewSigner + KeyGen(1)       (pssign/sign.go:43-67): Q = s_Q G2,
//                                       SK[0..2], PK[i] = SK[i] Q
//   GeneratePedersenParameters         (setup.go:153-166): PedGen, PedParams[3]
//                                       = random multiples of the G1 generator
//   GenerateRangeProofParameters       (setup.go:168-184): SignedValues[m] =
//                                       Sign([m]) for m < base, with the
//                                       pssign/sign.go:97-98 quirk (R stays the
//                                       G1 generator: Mul's result is dropped),
//                                       S = (SK0 + m SK1 + H(m) SK2) R,
//                                       H(m) = HashToZr(m.Bytes()) (:198-206)
//   Exponent, QuantityPrecision = 64, IdemixIssuerPK, IdemixCurveID
// -- and Serialize (setup.go:119-128) writes: json.Marshal(pp) wrapped in
// driver.SerializedPublicParameters{Identifier, Raw}.  The reference draws its
// scalars from crypto/rand; here rand(tag) = SHA-256(seed||tag||0) ||
// SHA-256(seed||tag||1) mod r (the prover's randomness, include/ftsamd.h), so
// a seed reproduces a parameter set (the golden fixtures' PP-A / PP-B).
// Runs once per network on the host with the same field / curve code the
// kernels use (dev/*.h compiled for the host); nothing here is on the hot path.
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../../include/ftsamd.h"
#include "../dev/jobs.h"
#include "gojson.h"

using namespace fts;

namespace {

fr setup_rand(const uint8_t* seed, size_t seed_len, const std::string& tag) {
  uint8_t h[2][32];
  for (int q = 0; q < 2; q++) {
    Sha256 s;
    s.init();
    s.update(seed, (uint32_t)seed_len);
    s.update(reinterpret_cast<const uint8_t*>(tag.data()), (uint32_t)tag.size());
    uint8_t b = (uint8_t)q;
    s.update(&b, 1);
    s.final(h[q]);
  }
  uint32_t t0[8], t1[8];
  be32_to_limbs(t0, h[0]);
  be32_to_limbs(t1, h[1]);
  return fe_from_int<ModR>(t0) * fe_const<ModR>(R_R2) + fe_from_int<ModR>(t1);
}

void ints(uint32_t out[8], const fr& a) { fe_to_int(out, a); }

std::string elem_json(const uint8_t* raw, size_t n) {
  std::string b;
  ftsh::b64_encode(raw, n, b);
  return "{\"curve\":1,\"element\":\"" + b + "\"}";
}
std::string g1_json(const g1j& p) {
  uint8_t raw[64];
  g1_to_bytes(raw, jac_to_aff(p));
  return elem_json(raw, 64);
}
std::string g2_json(const g2j& p) {
  uint8_t raw[128];
  g2_to_bytes(raw, jac_to_aff(p));
  return elem_json(raw, 128);
}
std::string bytes_json(const uint8_t* p, size_t n, bool nil) {
  if (nil) return "null";
  std::string b;
  ftsh::b64_encode(p, n, b);
  return "\"" + b + "\"";
}

}  // namespace

extern "C" int ftz_pp_setup(uint64_t base, uint32_t exponent, const uint8_t* idemix_pk, size_t idemix_pk_len,
                            int idemix_curve, const uint8_t* seed, size_t seed_len, uint8_t* out, size_t cap,
                            size_t* out_len) {
  if (!out_len || (!seed && seed_len) || (!idemix_pk && idemix_pk_len) || (!out && cap)) return FTZ_E_INVALID;
  if (base < 1 || base > (1u << 20)) return FTZ_E_INVALID;
  g1a G1 = {fe_const<ModP>(G1_GEN_X), fe_const<ModP>(G1_GEN_Y), false};
  g2a G2 = {{fe_const<ModP>(G2_GEN_X0), fe_const<ModP>(G2_GEN_X1)}, {fe_const<ModP>(G2_GEN_Y0), fe_const<ModP>(G2_GEN_Y1)},
            false};
  uint32_t k[8];
  // pssign KeyGen(1): Q, SK[0..2], PK[i] = SK[i] Q
  ints(k, setup_rand(seed, seed_len, "setup/Q"));
  g2a Q = jac_to_aff(aff_mul(G2, k));
  fr sk[3];
  std::string pks = "[";
  for (int i = 0; i < 3; i++) {
    sk[i] = setup_rand(seed, seed_len, "setup/sk/" + std::to_string(i));
    ints(k, sk[i]);
    pks += (i ? "," : "") + g2_json(aff_mul(Q, k));
  }
  pks += "]";
  // GeneratePedersenParameters
  ints(k, setup_rand(seed, seed_len, "setup/pedgen"));
  std::string pedgen = g1_json(aff_mul(G1, k));
  std::string peds = "[";
  for (int i = 0; i < 3; i++) {
    ints(k, setup_rand(seed, seed_len, "setup/ped/" + std::to_string(i)));
    peds += (i ? "," : "") + g1_json(aff_mul(G1, k));
  }
  peds += "]";
  // GenerateRangeProofParameters: SignedValues[m] = {R = G1, S = (sk0 + m sk1 + H(m) sk2) G1}
  uint8_t graw[64];
  g1_to_bytes(graw, G1);
  const std::string rj = elem_json(graw, 64);
  std::string sigs = "[";
  for (uint64_t m = 0; m < base; m++) {
    uint32_t mi[8] = {(uint32_t)m, (uint32_t)(m >> 32), 0, 0, 0, 0, 0, 0};
    uint8_t mb[32], d[32];
    limbs_to_be32(mb, mi);  // Zr.Bytes(): 32 bytes big-endian
    Sha256 s;
    s.init();
    s.update(mb, 32);
    s.final(d);
    uint32_t hm[8];
    digest_mod_r(hm, d);
    fr e = sk[0] + fe_from_int<ModR>(mi) * sk[1] + fe_from_int<ModR>(hm) * sk[2];
    ints(k, e);
    sigs += (m ? ",{\"R\":" : "{\"R\":") + rj + ",\"S\":" + g1_json(aff_mul(G1, k)) + "}";
  }
  sigs += "]";
  uint8_t qraw[128];
  g2_to_bytes(qraw, Q);
  std::string rpp = "{\"SignPK\":" + pks + ",\"SignedValues\":" + sigs + ",\"Q\":" + elem_json(qraw, 128) +
                    ",\"Exponent\":" + std::to_string(exponent) + "}";
  std::string raw = "{\"Label\":\"zkatdlog\",\"Curve\":1,\"PedGen\":" + pedgen + ",\"PedParams\":" + peds +
                    ",\"RangeProofParams\":" + rpp + ",\"IdemixCurveID\":" + std::to_string(idemix_curve) +
                    ",\"IdemixIssuerPK\":" + bytes_json(idemix_pk, idemix_pk_len, idemix_pk == nullptr) +
                    ",\"Auditor\":null,\"Issuers\":null,\"QuantityPrecision\":64}";
  std::string ser = "{\"Identifier\":\"zkatdlog\",\"Raw\":" +
                    bytes_json(reinterpret_cast<const uint8_t*>(raw.data()), raw.size(), false) + "}";
  *out_len = ser.size();
  if (ser.size() > cap) return FTZ_E_INVALID;
  memcpy(out, ser.data(), ser.size());
  return FTZ_SUCCESS;
}

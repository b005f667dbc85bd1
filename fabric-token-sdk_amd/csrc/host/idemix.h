// Host side of idemix owner-signature verification: the
// wire formats around IBM/idemix NymSignature.Ver, decoded as the reference's
// Go libraries decode them (paths relative to /root/reference/token/core/):
//   * RawOwner (identity/owner.go:23-37): Go encoding/asn1 of
//     struct{Type string; Identity []byte}; interop/htlc/deserializer.go:31-43
//     dispatches on Type ("si" idemix, "htlc" script -> left to Go);
//   * msp.SerializedIdentity{Mspid, IdBytes} and msp.SerializedIdemixIdentity
//     {NymX, NymY, Ou, Role, Proof}, msp.OrganizationUnit, msp.MSPRole
//     (identity/msp/idemix/common.go:40-117, Deserialize with checkValidity=false);
//   * idemix NymSignature{ProofC, ProofSSk, ProofSRNym, Nonce} and
//     IssuerPublicKey{..., HSk, HRand, ..., Hash} protos (IBM/idemix, [EXT]).
// Both idemix curves of identity/msp/idemix/deserializer.go:40-51 are read as
// their translator reads them (`curve` = FTZ_CURVE_FP256BN_AMCL or
// FTZ_CURVE_BN254): amcl FromBytes (first 32 bytes, unreduced) and NewECPbigs on
// FP256BN; gurvy G1FromProto (exactly 32-byte X and Y, gnark SetBytes) and
// big.Int SetBytes over whole fields on BN254 (dev/idemix.h, oracle idemix.py).
// Protobuf: google.golang.org/protobuf v1.27.1 proto3 rules (go.mod:10,226).
#pragma once
#include <stdint.h>

#include <functional>
#include <string>
#include <vector>

#include "../../../include/ftsamd.h"

namespace ftsh {

// One protobuf field as scanned: wire type 0 (value in v) or 2 (bytes p/len).
struct PbField {
  uint32_t num;
  uint8_t wt;
  uint64_t v;
  const uint8_t* p;
  size_t len;
};
// Scan a message: every field in order (other wire types are validated and
// skipped, groups included).  "" or the decoding error.
std::string pb_scan(const uint8_t* b, size_t n, std::vector<PbField>& out);
// Go utf8.Valid
bool utf8_valid(const uint8_t* p, size_t n);

struct IdemixIpk {
  std::vector<uint8_t> hsk_x, hsk_y, hrand_x, hrand_y;  // ECP coordinates (FromBytes: first 32 bytes)
  std::vector<std::vector<uint8_t>> hattrs_x, hattrs_y; // HAttrs[i] (an absent coordinate: empty)
  std::vector<uint8_t> hash;                            // IssuerPublicKey.Hash
};
// proto IssuerPublicKey: "" or the error
std::string parse_ipk(const uint8_t* p, size_t n, IdemixIpk& out);

// Result of decoding one (owner, signature) pair on the host.
struct NymDecoded {
  int code = 0;           // 0 = go to the device; else FTZ_ERR_OWNER / _SIGNATURE / _UNSUPPORTED
  std::string why;        // the reference's error text when code != 0
  uint8_t ints[6][32];    // NymX, NymY, ProofC, ProofSSk, ProofSRNym, Nonce (first 32 bytes each)
  uint32_t glv[12];       // ProofC mod n = k1 + k2 lambda: |k1| (5 limbs), |k2| (5), sign bits, 0
  // BN254: NymX / NymY canonical (gnark-decoded; all zero = infinity), ProofSSk and
  // ProofSRNym reduced mod r, ProofC all-0xff when its integer is >= r (it can then
  // never equal a HashToZr output), Nonce as Zr.Bytes() (its integer < 2^256)
};
// k (32 bytes big-endian, any value) mod n split as k1 + k2 lambda with
// |k1|, |k2| < 2^129: out = |k1| (5 limbs) | |k2| (5 limbs) | (k1 < 0) | (k2 < 0) << 1 | 0
void nym_glv_split(const uint8_t k[32], uint32_t out[12]);
// the same split on BN254 (k < r canonical; dev/jobs.h-style lattice, |k_i| < 2^128)
void nym_glv_split_bn(const uint8_t k[32], uint32_t out[12]);
// big-endian integer of any length mod r (BN254), 32 bytes big-endian
void be_mod_r(const uint8_t* p, size_t n, uint8_t out[32]);
// TransferSignatureValidate's per-input path up to the curve arithmetic:
// GetOwnerVerifier(owner) then the signature unmarshal of Verify(msg, sigma).
void decode_owner_signature(const uint8_t* owner, size_t owner_len, const uint8_t* sig, size_t sig_len,
                            NymDecoded& out, int curve = FTZ_CURVE_FP256BN_AMCL);

// Auditor owner match (crypto/audit/auditor.go:252-274 InspectTokenOwner ->
// idemix DeserializeAuditInfo + AuditInfo.Match, identity/msp/idemix/
// audit.go:32-83): everything up to the curve arithmetic.  [EXT] IBM/idemix
// AuditNymEid: Nym_eid = HAttrs[2]^HashToZr(Attributes[2]) * HRand^RNymEid must
// equal the identity proof's EidNym.Nym (idemix Signature proto field 18).
struct EidDecoded {
  int code = 0;             // 0 = go to the device; else FTZ_ERR_OWNER / _AUDIT / _UNSUPPORTED / _PANIC
  std::string why;
  uint8_t eid_digest[32];   // SHA-256(EnrollmentID) (HashToZr before the reduction mod n)
  uint8_t rnym[32];         // RNymEid (FP256BN: FromBytes, raw, unreduced; BN254: mod r)
  uint8_t nym_x[32], nym_y[32];  // EidNym.Nym X, Y (FP256BN: first 32 bytes; BN254: canonical, zero = infinity)
};
void decode_owner_audit(const uint8_t* owner, size_t owner_len, const uint8_t* audit_info, size_t audit_info_len,
                        size_t n_hattrs, EidDecoded& out, int curve = FTZ_CURVE_FP256BN_AMCL);

// Blob of one device pass over the signatures s[idx[0..m)] (all decoded with
// code 0): the NymJob array at offset 0, then per job the six integers and
// the GLV split of ProofC (dev/idemix.h NymJob.sc, 240 bytes) and the 176-byte
// transcript prefix ("sign", zeros for t and Nym, the IPK hash after them and,
// on BN254, the 2 tail bytes), then every distinct message (same pointer and
// length) once at an offset = NymCurve::PRE mod 16 (6 on FP256BN, 4 on BN254).
struct NymLayout {
  size_t total = 0;                                   // blob bytes (+ slack)
  std::vector<uint32_t> msg_off;                      // per job
  std::vector<std::pair<uint32_t, uint32_t>> distinct;  // (blob offset, job whose message is copied there)
};
void nym_plan_layout(const ftz_owner_sig* s, const uint32_t* idx, size_t m, NymLayout& L,
                     int curve = FTZ_CURVE_FP256BN_AMCL);
// fill the blob; `par` (optional) runs f(0..k) in parallel; ipk_hash = the whole
// IssuerPublicKey.Hash (copy(proofData[index:], ipk.Hash))
void nym_fill(const ftz_owner_sig* s, const uint32_t* idx, size_t m, const NymDecoded* dec,
              const std::vector<uint8_t>& ipk_hash, const NymLayout& L, uint8_t* blob,
              const std::function<void(size_t, const std::function<void(size_t)>&)>& par,
              int curve = FTZ_CURVE_FP256BN_AMCL);

}  // namespace ftsh

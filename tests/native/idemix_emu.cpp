// TEST-ONLY host build of the idemix owner-signature path: the product's host
// decoding (host/idemix.cpp) and blob layout, and the device job code
// (dev/idemix.h job_nym) run on the CPU, so the CPU test tier checks them
// against the oracle without a GPU.  Never loaded by the product.
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../fabric-token-sdk_amd/csrc/dev/idemix.h"
#include "../../fabric-token-sdk_amd/csrc/host/idemix.h"

using namespace fts;

struct EmuIdemix {
  uint8_t hash_slot[32] = {};
  std::vector<QDev> tab;
  size_t n_hattrs = 0;
};

extern "C" {

void* emu_idemix_create(const uint8_t* ipk, size_t len, char* err, size_t cap) {
  ftsh::IdemixIpk k;
  std::string e = ftsh::parse_ipk(ipk, len, k);
  q1a bases[3];
  if (e.empty() && (!nym_point_from_be(k.hsk_x.data(), k.hsk_y.data(), bases[0]) ||
                    !nym_point_from_be(k.hrand_x.data(), k.hrand_y.data(), bases[1])))
    e = "issuer public key: HSk / HRand not on FP256BN";
  bool heid = e.empty() && k.hattrs_x.size() > 2 && k.hattrs_x[2].size() >= 32 && k.hattrs_y[2].size() >= 32 &&
              nym_point_from_be(k.hattrs_x[2].data(), k.hattrs_y[2].data(), bases[2]);
  if (!e.empty()) {
    snprintf(err, cap, "%s", e.c_str());
    return nullptr;
  }
  EmuIdemix* ix = new EmuIdemix();
  memcpy(ix->hash_slot, k.hash.data(), k.hash.size() < 32 ? k.hash.size() : 32);
  ix->tab.resize((heid ? 3 : 2) * NYM_TAB_PER_BASE);
  nym_build_tables(bases, heid ? 3 : 2, ix->tab.data());
  ix->n_hattrs = heid ? k.hattrs_x.size() : 0;
  return ix;
}

void emu_idemix_destroy(void* p) { delete (EmuIdemix*)p; }

int emu_verify_owner_signatures(void* p, size_t n, const ftz_owner_sig* s, int32_t* codes) {
  EmuIdemix* ix = (EmuIdemix*)p;
  std::vector<ftsh::NymDecoded> dec(n);
  std::vector<uint32_t> idx;
  for (size_t i = 0; i < n; i++) {
    ftsh::decode_owner_signature(s[i].owner, s[i].owner_len, s[i].sig, s[i].sig_len, dec[i]);
    codes[i] = dec[i].code;
    if (dec[i].code == 0) idx.push_back((uint32_t)i);
  }
  if (idx.empty()) return 0;
  ftsh::NymLayout L;
  ftsh::nym_plan_layout(s, idx.data(), idx.size(), L);
  std::vector<uint8_t> blob(L.total + 16);
  uint8_t* b = blob.data() + ((16 - ((uintptr_t)blob.data() & 15)) & 15);  // the device blob is 256-aligned
  ftsh::nym_fill(s, idx.data(), idx.size(), dec.data(), ix->hash_slot, L, b,
                 [](size_t k, const std::function<void(size_t)>& f) {
                   for (size_t i = 0; i < k; i++) f(i);
                 });
  const NymJob* jobs = reinterpret_cast<const NymJob*>(b);
  for (size_t k = 0; k < idx.size(); k++) {
    q1j t = jac_add(jac_add(job_nym_part(jobs[k], b, ix->tab.data(), 0), job_nym_part(jobs[k], b, ix->tab.data(), 1)),
                    jac_add(job_nym_part(jobs[k], b, ix->tab.data(), 2), job_nym_part(jobs[k], b, ix->tab.data(), 3)));
    codes[idx[k]] = job_nym_fin(jobs[k], b, t) ? FTZ_OK : FTZ_ERR_SIGNATURE;
  }
  return 0;
}

// decoding only (host/idemix.cpp): code and the reference's error text
int emu_decode_owner_signature(const uint8_t* owner, size_t owner_len, const uint8_t* sig, size_t sig_len,
                               char* why, size_t cap) {
  ftsh::NymDecoded d;
  ftsh::decode_owner_signature(owner, owner_len, sig, sig_len, d);
  snprintf(why, cap, "%s", d.why.c_str());
  return d.code;
}

// auditor owner match: the product's host decoding + the device job code
int emu_audit_owners(void* p, size_t n, const ftz_owner_audit* it, int32_t* codes) {
  EmuIdemix* ix = (EmuIdemix*)p;
  for (size_t i = 0; i < n; i++) {
    ftsh::EidDecoded d;
    ftsh::decode_owner_audit(it[i].owner, it[i].owner_len, it[i].audit_info, it[i].audit_info_len, ix->n_hattrs, d);
    codes[i] = d.code;
    if (d.code) continue;
    uint8_t in[EID_JOB_BYTES];
    memcpy(in, d.eid_digest, 32);
    memcpy(in + 32, d.rnym, 32);
    memcpy(in + 64, d.nym_x, 32);
    memcpy(in + 96, d.nym_y, 32);
    codes[i] = job_eid(in, ix->tab.data()) ? FTZ_OK : FTZ_ERR_AUDIT;
  }
  return 0;
}

// host half of the auditor match alone: code and the reference's error text
int emu_decode_owner_audit(const uint8_t* o, size_t ol, const uint8_t* a, size_t al, size_t n_hattrs, char* why,
                           size_t cap) {
  ftsh::EidDecoded d;
  ftsh::decode_owner_audit(o, ol, a, al, n_hattrs, d);
  snprintf(why, cap, "%s", d.why.c_str());
  return d.code;
}

// host GLV split of a 32-byte scalar (host/idemix.cpp)
void emu_nym_glv_split(const uint8_t* k, uint32_t* out) { ftsh::nym_glv_split(k, out); }

}  // extern "C"

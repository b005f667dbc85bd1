// TEST-ONLY host build of the idemix owner-signature path: the product's host
// decoding (host/idemix.cpp) and blob layout, and the device job code
// (dev/idemix.h job_nym) run on the CPU, so the CPU test tier checks them
// against the oracle without a GPU.  Never loaded by the product.
#include <string.h>

#include <string>
#include <vector>

#include "../../fabric-token-sdk_amd/csrc/dev/idemix.h"
#include "../../fabric-token-sdk_amd/csrc/host/idemix.h"

using namespace fts;

struct EmuIdemix {
  uint8_t hash_slot[32] = {};
  std::vector<QDev> tab;
};

extern "C" {

void* emu_idemix_create(const uint8_t* ipk, size_t len, char* err, size_t cap) {
  ftsh::IdemixIpk k;
  std::string e = ftsh::parse_ipk(ipk, len, k);
  q1a bases[2];
  if (e.empty() && (!nym_point_from_be(k.hsk_x.data(), k.hsk_y.data(), bases[0]) ||
                    !nym_point_from_be(k.hrand_x.data(), k.hrand_y.data(), bases[1])))
    e = "issuer public key: HSk / HRand not on FP256BN";
  if (!e.empty()) {
    snprintf(err, cap, "%s", e.c_str());
    return nullptr;
  }
  EmuIdemix* ix = new EmuIdemix();
  memcpy(ix->hash_slot, k.hash.data(), k.hash.size() < 32 ? k.hash.size() : 32);
  ix->tab.resize(2 * NYM_TAB_PER_BASE);
  nym_build_tables(bases, ix->tab.data());
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

// host GLV split of a 32-byte scalar (host/idemix.cpp)
void emu_nym_glv_split(const uint8_t* k, uint32_t* out) { ftsh::nym_glv_split(k, out); }

}  // extern "C"

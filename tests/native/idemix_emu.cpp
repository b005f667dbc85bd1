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
  int curve = FTZ_CURVE_FP256BN_AMCL;
  std::vector<uint8_t> ipk_hash;
  std::vector<QDev> tab;
  size_t n_hattrs = 0;
};

template <class F>
static bool run_nym(const NymJob& j, uint8_t* b, const QDev* tab) {
  Jac<F> t = jac_add(jac_add(job_nym_part<F>(j, b, tab, 0), job_nym_part<F>(j, b, tab, 1)),
                     jac_add(job_nym_part<F>(j, b, tab, 2), job_nym_part<F>(j, b, tab, 3)));
  return job_nym_fin<F>(j, b, t) != 0;
}

extern "C" {

void* emu_idemix_create_curve(const uint8_t* ipk, size_t len, int curve, char* err, size_t cap) {
  ftsh::IdemixIpk k;
  std::string e = ftsh::parse_ipk(ipk, len, k);
  EmuIdemix* ix = new EmuIdemix();
  ix->curve = curve;
  bool heid = false;
  if (e.empty() && curve == FTZ_CURVE_BN254) {
    g1a bases[3];
    auto dec = [](const std::vector<uint8_t>& x, const std::vector<uint8_t>& y, g1a& a) {
      return x.size() == 32 && y.size() == 32 && bn_point_from_xy(x.data(), y.data(), a) && !a.inf;
    };
    if (!dec(k.hsk_x, k.hsk_y, bases[0]) || !dec(k.hrand_x, k.hrand_y, bases[1])) {
      e = "issuer public key: HSk / HRand not a finite BN254 point";
    } else {
      heid = k.hattrs_x.size() > 2 && dec(k.hattrs_x[2], k.hattrs_y[2], bases[2]);
      ix->tab.resize((heid ? 3 : 2) * NYM_TAB_PER_BASE);
      nym_build_tables(bases, heid ? 3 : 2, ix->tab.data());
    }
  } else if (e.empty()) {
    q1a bases[3];
    if (!nym_point_from_be(k.hsk_x.data(), k.hsk_y.data(), bases[0]) ||
        !nym_point_from_be(k.hrand_x.data(), k.hrand_y.data(), bases[1])) {
      e = "issuer public key: HSk / HRand not on FP256BN";
    } else {
      heid = k.hattrs_x.size() > 2 && k.hattrs_x[2].size() >= 32 && k.hattrs_y[2].size() >= 32 &&
             nym_point_from_be(k.hattrs_x[2].data(), k.hattrs_y[2].data(), bases[2]);
      ix->tab.resize((heid ? 3 : 2) * NYM_TAB_PER_BASE);
      nym_build_tables(bases, heid ? 3 : 2, ix->tab.data());
    }
  }
  if (!e.empty()) {
    snprintf(err, cap, "%s", e.c_str());
    delete ix;
    return nullptr;
  }
  ix->ipk_hash = k.hash;
  ix->n_hattrs = heid ? k.hattrs_x.size() : 0;
  return ix;
}

void* emu_idemix_create(const uint8_t* ipk, size_t len, char* err, size_t cap) {
  return emu_idemix_create_curve(ipk, len, FTZ_CURVE_FP256BN_AMCL, err, cap);
}

void emu_idemix_destroy(void* p) { delete (EmuIdemix*)p; }

int emu_verify_owner_signatures(void* p, size_t n, const ftz_owner_sig* s, int32_t* codes) {
  EmuIdemix* ix = (EmuIdemix*)p;
  std::vector<ftsh::NymDecoded> dec(n);
  std::vector<uint32_t> idx;
  for (size_t i = 0; i < n; i++) {
    ftsh::decode_owner_signature(s[i].owner, s[i].owner_len, s[i].sig, s[i].sig_len, dec[i], ix->curve);
    codes[i] = dec[i].code;
    if (dec[i].code == 0) idx.push_back((uint32_t)i);
  }
  if (idx.empty()) return 0;
  ftsh::NymLayout L;
  ftsh::nym_plan_layout(s, idx.data(), idx.size(), L, ix->curve);
  std::vector<uint8_t> blob(L.total + 16);
  uint8_t* b = blob.data() + ((16 - ((uintptr_t)blob.data() & 15)) & 15);  // the device blob is 256-aligned
  ftsh::nym_fill(s, idx.data(), idx.size(), dec.data(), ix->ipk_hash, L, b,
                 [](size_t k, const std::function<void(size_t)>& f) {
                   for (size_t i = 0; i < k; i++) f(i);
                 }, ix->curve);
  const NymJob* jobs = reinterpret_cast<const NymJob*>(b);
  for (size_t k = 0; k < idx.size(); k++)
    codes[idx[k]] = (ix->curve == FTZ_CURVE_BN254 ? run_nym<fp>(jobs[k], b, ix->tab.data())
                                                  : run_nym<fq>(jobs[k], b, ix->tab.data()))
                        ? FTZ_OK
                        : FTZ_ERR_SIGNATURE;
  return 0;
}

// decoding only (host/idemix.cpp): code and the reference's error text
int emu_decode_owner_signature_curve(const uint8_t* owner, size_t owner_len, const uint8_t* sig, size_t sig_len,
                                     int curve, char* why, size_t cap) {
  ftsh::NymDecoded d;
  ftsh::decode_owner_signature(owner, owner_len, sig, sig_len, d, curve);
  snprintf(why, cap, "%s", d.why.c_str());
  return d.code;
}
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
    ftsh::decode_owner_audit(it[i].owner, it[i].owner_len, it[i].audit_info, it[i].audit_info_len, ix->n_hattrs, d,
                             ix->curve);
    codes[i] = d.code;
    if (d.code) continue;
    uint8_t in[EID_JOB_BYTES];
    memcpy(in, d.eid_digest, 32);
    memcpy(in + 32, d.rnym, 32);
    memcpy(in + 64, d.nym_x, 32);
    memcpy(in + 96, d.nym_y, 32);
    codes[i] = (ix->curve == FTZ_CURVE_BN254 ? job_eid<fp>(in, ix->tab.data()) : job_eid<fq>(in, ix->tab.data()))
                   ? FTZ_OK
                   : FTZ_ERR_AUDIT;
  }
  return 0;
}

// host half of the auditor match alone: code and the reference's error text
int emu_decode_owner_audit_curve(const uint8_t* o, size_t ol, const uint8_t* a, size_t al, size_t n_hattrs, int curve,
                                 char* why, size_t cap) {
  ftsh::EidDecoded d;
  ftsh::decode_owner_audit(o, ol, a, al, n_hattrs, d, curve);
  snprintf(why, cap, "%s", d.why.c_str());
  return d.code;
}
int emu_decode_owner_audit(const uint8_t* o, size_t ol, const uint8_t* a, size_t al, size_t n_hattrs, char* why,
                           size_t cap) {
  ftsh::EidDecoded d;
  ftsh::decode_owner_audit(o, ol, a, al, n_hattrs, d);
  snprintf(why, cap, "%s", d.why.c_str());
  return d.code;
}

// host GLV split of a 32-byte scalar (host/idemix.cpp)
void emu_nym_glv_split(const uint8_t* k, uint32_t* out) { ftsh::nym_glv_split(k, out); }
void emu_nym_glv_split_bn(const uint8_t* k, uint32_t* out) { ftsh::nym_glv_split_bn(k, out); }
void emu_be_mod_r(const uint8_t* p, size_t n, uint8_t* out) { ftsh::be_mod_r(p, n, out); }

}  // extern "C"

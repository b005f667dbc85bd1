// C ABI of idemix owner-signature verification (include/ftsamd.h, SURVEY 8(f)
// row 3) on BN254 or FP256BN_AMCL: owner identity and signature protos decoded
// on the host pool (host/idemix.cpp), NymSignature.Ver's curve arithmetic and
// hashes on the GPU (k_nym_part/_fin, _bn for BN254; dev/idemix.h).
#include <hip/hip_runtime.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "host/idemix.h"
#include "launch.h"
#include "rt_internal.h"

// One pipeline slot: pinned staging, device blob / partials / verdicts, its stream.
struct NymSlot {
  PinnedMem h_blob, h_ok;
  DevMem d_blob, d_ok, d_part;
  hipStream_t st = nullptr;
  std::vector<uint32_t> idx;  // call-relative indices of the slot's signatures
  bool busy = false;
};

struct ftz_idemix {
  ftz_ctx* ctx = nullptr;
  int curve = FTZ_CURVE_FP256BN_AMCL;
  std::vector<uint8_t> ipk_hash;  // IssuerPublicKey.Hash (copy(proofData[index:], ipk.Hash))
  DBuf<QDev> tab;              // HSk, HRand (and HAttrs[2]) fixed-base tables
  size_t n_hattrs = 0;         // len(IssuerPublicKey.HAttrs)
  bool heid_ok = false;        // HAttrs[2] decoded on the curve (its table exists)
  bool strict_nym = false;     // ftz_idemix_set_strict_nym: reject off-curve nyms on the host
  PinnedMem h_eid, h_eid_ok;   // auditor owner match (ftz_audit_owners)
  DevMem d_eid, d_eid_ok;
  std::mutex mu;               // one call on the device at a time
  WorkPool* pool = nullptr;    // host decoding / layout threads
  NymSlot slot[2];             // chunk k+1 is decoded and laid out while chunk k runs
  ~ftz_idemix() {
    for (NymSlot& q : slot)
      if (q.st) {
        (void)hipStreamSynchronize(q.st);
        (void)hipStreamDestroy(q.st);
      }
    delete pool;
  }
};

extern "C" int ftz_idemix_create(ftz_ctx* ctx, const uint8_t* ipk, size_t ipk_len, int curve_id, ftz_idemix** out) {
  if (!ctx || !out || (!ipk && ipk_len)) return set_err(FTZ_E_INVALID, "null argument");
  if (curve_id != FTZ_CURVE_FP256BN_AMCL && curve_id != FTZ_CURVE_BN254)
    return set_err(FTZ_E_INVALID, "unsupported idemix curve id " + std::to_string(curve_id) +
                                      " (BN254 = 1 or FP256BN_AMCL = 0)");
  if (ipk_len == 0) return set_err(FTZ_E_PP, "empty idemix issuer public key");
  ftsh::IdemixIpk k;
  std::string e = ftsh::parse_ipk(ipk, ipk_len, k);
  if (!e.empty()) return set_err(FTZ_E_PP, e);
  bool heid = false;
  std::vector<QDev> tab;
  if (curve_id == FTZ_CURVE_BN254) {
    // gurvy G1FromProto: exactly 32-byte coordinates, gnark SetBytes
    g1a bases[3];
    auto dec = [](const std::vector<uint8_t>& x, const std::vector<uint8_t>& y, g1a& a) {
      return x.size() == 32 && y.size() == 32 && bn_point_from_xy(x.data(), y.data(), a) && !a.inf;
    };
    if (!dec(k.hsk_x, k.hsk_y, bases[0]) || !dec(k.hrand_x, k.hrand_y, bases[1]))
      return set_err(FTZ_E_PP, "issuer public key: HSk / HRand not a finite BN254 point");
    heid = k.hattrs_x.size() > 2 && dec(k.hattrs_x[2], k.hattrs_y[2], bases[2]);
    tab.resize((heid ? 3 : 2) * NYM_TAB_PER_BASE);
    nym_build_tables(bases, heid ? 3 : 2, tab.data());
  } else {
    q1a bases[3];
    if (!nym_point_from_be(k.hsk_x.data(), k.hsk_y.data(), bases[0]) ||
        !nym_point_from_be(k.hrand_x.data(), k.hrand_y.data(), bases[1]))
      return set_err(FTZ_E_PP, "issuer public key: HSk / HRand not on FP256BN");
    // HAttrs[2] (the enrollment-id base of the auditor's EidNym check)
    heid = k.hattrs_x.size() > 2 && k.hattrs_x[2].size() >= 32 && k.hattrs_y[2].size() >= 32 &&
           nym_point_from_be(k.hattrs_x[2].data(), k.hattrs_y[2].data(), bases[2]);
    tab.resize((heid ? 3 : 2) * NYM_TAB_PER_BASE);
    nym_build_tables(bases, heid ? 3 : 2, tab.data());
  }
  HC(hipSetDevice(ctx->device));
  ftz_idemix* ix = new ftz_idemix();
  ix->ctx = ctx;
  ix->pool = new WorkPool(ctx->opt.threads ? (int)ctx->opt.threads : 8);
  for (NymSlot& q : ix->slot) {
    hipError_t se = hipStreamCreateWithFlags(&q.st, hipStreamNonBlocking);
    if (se != hipSuccess) {
      delete ix;
      return set_err(FTZ_E_DEVICE, std::string("hipStreamCreate failed: ") + hipGetErrorString(se));
    }
  }
  ix->curve = curve_id;
  ix->ipk_hash = k.hash;
  ix->n_hattrs = k.hattrs_x.size();
  ix->heid_ok = heid;
  hipError_t he = ix->tab.upload(tab, ctx->stream);
  if (he == hipSuccess) he = hipStreamSynchronize(ctx->stream);
  if (he != hipSuccess) {
    delete ix;
    return set_err(FTZ_E_DEVICE, std::string("idemix table upload failed: ") + hipGetErrorString(he));
  }
  *out = ix;
  return FTZ_SUCCESS;
}

void ftz_idemix_destroy(ftz_idemix* ix) { delete ix; }

extern "C" int ftz_idemix_set_strict_nym(ftz_idemix* ix, int on) {
  if (!ix) return set_err(FTZ_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(ix->mu);
  ix->strict_nym = on != 0;
  return FTZ_SUCCESS;
}

namespace {
constexpr size_t NYM_CHUNK_BYTES = (size_t)1 << 30;  // keeps every blob offset in 32 bits
constexpr size_t NYM_CHUNK_SIGS = 4096;              // signatures per pipelined device pass

// collect the verdicts of a slot's pass
int nym_collect(NymSlot& q, int32_t* codes) {
  if (!q.busy) return FTZ_SUCCESS;
  q.busy = false;
  HC(hipStreamSynchronize(q.st));
  for (size_t k = 0; k < q.idx.size(); k++) codes[q.idx[k]] = q.h_ok.p[k] ? FTZ_OK : FTZ_ERR_SIGNATURE;
  return FTZ_SUCCESS;
}

// decode s[a..b) on the pool; queue the device pass of the ones that reach the curve arithmetic
int nym_chunk(ftz_idemix* ix, NymSlot& q, const ftz_owner_sig* s, size_t a, size_t b, int32_t* codes) {
  size_t n = b - a;
  std::vector<ftsh::NymDecoded> dec(n);
  ix->pool->run((n + 63) / 64, [&](size_t p) {
    for (size_t i = p * 64; i < n && i < (p + 1) * 64; i++)
      ftsh::decode_owner_signature(s[a + i].owner, s[a + i].owner_len, s[a + i].sig, s[a + i].sig_len, dec[i],
                                 ix->curve);
  });
  std::vector<uint32_t> idx;  // chunk-relative
  for (size_t i = 0; i < n; i++) {
    if (ix->strict_nym && ix->curve == FTZ_CURVE_FP256BN_AMCL && dec[i].code == 0) {
      q1a nym;
      if (!nym_point_from_be(dec[i].ints[0], dec[i].ints[1], nym)) {
        dec[i].code = FTZ_ERR_OWNER;
        dec[i].why = "pseudonym is not on FP256BN (strict nym import)";
      }
    }
    codes[a + i] = dec[i].code;
    if (dec[i].code == 0) idx.push_back((uint32_t)i);
  }
  if (idx.empty()) return FTZ_SUCCESS;
  size_t m = idx.size();
  ftsh::NymLayout L;
  ftsh::nym_plan_layout(s + a, idx.data(), m, L, ix->curve);
  HC(q.h_blob.reserve(L.total));
  HC(q.d_blob.reserve(L.total));
  HC(q.h_ok.reserve(m));
  HC(q.d_ok.reserve(m));
  HC(q.d_part.reserve(4 * m * sizeof(QJDev)));
  WorkPool* pool = ix->pool;
  ftsh::nym_fill(s + a, idx.data(), m, dec.data(), ix->ipk_hash, L, q.h_blob.p,
                 [pool](size_t k, const std::function<void(size_t)>& f) { pool->run(k, f); }, ix->curve);
  const NymJob* jobs = reinterpret_cast<const NymJob*>(q.d_blob.p);
  QJDev* part = reinterpret_cast<QJDev*>(q.d_part.p);
  HC(hipMemcpyAsync(q.d_blob.p, q.h_blob.p, L.total, hipMemcpyHostToDevice, q.st));
  const uint32_t gp = (uint32_t)((4 * m + 63) / 64), gf = (uint32_t)((m + 63) / 64);
  if (ix->curve == FTZ_CURVE_BN254) {
    k_nym_part_bn<<<gp, 64, 0, q.st>>>(jobs, (uint32_t)m, q.d_blob.p, ix->tab.p, part);
    k_nym_fin_bn<<<gf, 64, 0, q.st>>>(jobs, (uint32_t)m, q.d_blob.p, part, q.d_ok.p);
  } else {
    k_nym_part<<<gp, 64, 0, q.st>>>(jobs, (uint32_t)m, q.d_blob.p, ix->tab.p, part);
    k_nym_fin<<<gf, 64, 0, q.st>>>(jobs, (uint32_t)m, q.d_blob.p, part, q.d_ok.p);
  }
  HC(hipGetLastError());
  HC(hipMemcpyAsync(q.h_ok.p, q.d_ok.p, m, hipMemcpyDeviceToHost, q.st));
  q.idx.resize(m);
  for (size_t k = 0; k < m; k++) q.idx[k] = (uint32_t)(a + idx[k]);
  q.busy = true;
  return FTZ_SUCCESS;
}
}  // namespace

extern "C" int ftz_verify_owner_signatures(ftz_idemix* ix, size_t n, const ftz_owner_sig* s, int32_t* codes) {
  if (!ix || (n && (!s || !codes))) return set_err(FTZ_E_INVALID, "null argument");
  for (size_t i = 0; i < n; i++) {
    if ((!s[i].owner && s[i].owner_len) || (!s[i].msg && s[i].msg_len) || (!s[i].sig && s[i].sig_len))
      return set_err(FTZ_E_INVALID, "null buffer with non-zero length");
    if (s[i].msg_len > NYM_CHUNK_BYTES / 2) return set_err(FTZ_E_INVALID, "message larger than 512 MiB");
  }
  std::lock_guard<std::mutex> lk(ix->mu);
  HC(hipSetDevice(ix->ctx->device));
  // chunks of <= NYM_CHUNK_SIGS signatures and < NYM_CHUNK_BYTES of blob, alternating
  // between the two slots: chunk k+1 is decoded and laid out while chunk k runs
  size_t a = 0, c = 0;
  int rc = FTZ_SUCCESS;
  while (a < n && rc == FTZ_SUCCESS) {
    size_t b = a, bytes = 0;
    while (b < n && b - a < NYM_CHUNK_SIGS && (b == a || bytes + s[b].msg_len + 512 < NYM_CHUNK_BYTES)) {
      bytes += s[b].msg_len + 512;
      b++;
    }
    NymSlot& q = ix->slot[c & 1];
    rc = nym_collect(q, codes);
    if (rc == FTZ_SUCCESS) rc = nym_chunk(ix, q, s, a, b, codes);
    a = b;
    c++;
  }
  for (NymSlot& q : ix->slot) {
    int r2 = nym_collect(q, codes);
    if (rc == FTZ_SUCCESS) rc = r2;
  }
  return rc;
}

// Auditor owner match: decode on the pool, one device pass over the tokens
// whose check reaches the curve arithmetic
extern "C" int ftz_audit_owners(ftz_idemix* ix, size_t n, const ftz_owner_audit* it, int32_t* codes) {
  if (!ix || (n && (!it || !codes))) return set_err(FTZ_E_INVALID, "null argument");
  for (size_t i = 0; i < n; i++)
    if ((!it[i].owner && it[i].owner_len) || (!it[i].audit_info && it[i].audit_info_len))
      return set_err(FTZ_E_INVALID, "null buffer with non-zero length");
  if (n > (1u << 26)) return set_err(FTZ_E_INVALID, "too many tokens in one call");
  if (ix->n_hattrs > 2 && !ix->heid_ok) return set_err(FTZ_E_PP, "issuer public key: HAttrs[2] not on the idemix curve");
  std::vector<ftsh::EidDecoded> dec(n);
  ix->pool->run((n + 63) / 64, [&](size_t p) {
    for (size_t i = p * 64; i < n && i < (p + 1) * 64; i++)
      ftsh::decode_owner_audit(it[i].owner, it[i].owner_len, it[i].audit_info, it[i].audit_info_len, ix->n_hattrs,
                               dec[i], ix->curve);
  });
  std::vector<uint32_t> idx;
  for (size_t i = 0; i < n; i++) {
    codes[i] = dec[i].code;
    if (dec[i].code == 0) idx.push_back((uint32_t)i);
  }
  if (idx.empty()) return FTZ_SUCCESS;
  std::lock_guard<std::mutex> lk(ix->mu);
  HC(hipSetDevice(ix->ctx->device));
  size_t m = idx.size();
  HC(ix->h_eid.reserve(m * EID_JOB_BYTES));
  HC(ix->d_eid.reserve(m * EID_JOB_BYTES));
  HC(ix->h_eid_ok.reserve(m));
  HC(ix->d_eid_ok.reserve(m));
  for (size_t k = 0; k < m; k++) {
    const ftsh::EidDecoded& d = dec[idx[k]];
    uint8_t* o = ix->h_eid.p + k * EID_JOB_BYTES;
    memcpy(o, d.eid_digest, 32);
    memcpy(o + 32, d.rnym, 32);
    memcpy(o + 64, d.nym_x, 32);
    memcpy(o + 96, d.nym_y, 32);
  }
  hipStream_t st = ix->slot[0].st;
  HC(hipMemcpyAsync(ix->d_eid.p, ix->h_eid.p, m * EID_JOB_BYTES, hipMemcpyHostToDevice, st));
  if (ix->curve == FTZ_CURVE_BN254)
    k_eid_bn<<<(uint32_t)((m + 63) / 64), 64, 0, st>>>(ix->d_eid.p, (uint32_t)m, ix->tab.p, ix->d_eid_ok.p);
  else
    k_eid<<<(uint32_t)((m + 63) / 64), 64, 0, st>>>(ix->d_eid.p, (uint32_t)m, ix->tab.p, ix->d_eid_ok.p);
  HC(hipGetLastError());
  HC(hipMemcpyAsync(ix->h_eid_ok.p, ix->d_eid_ok.p, m, hipMemcpyDeviceToHost, st));
  HC(hipStreamSynchronize(st));
  for (size_t k = 0; k < m; k++) codes[idx[k]] = ix->h_eid_ok.p[k] ? FTZ_OK : FTZ_ERR_AUDIT;
  return FTZ_SUCCESS;
}

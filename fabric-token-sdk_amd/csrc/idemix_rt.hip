// C ABI of idemix owner-signature verification (include/ftsamd.h, SURVEY 8(f)
// row 3): owner identity and signature protos decoded on the calling thread
// (host/idemix.cpp), NymSignature.Ver's curve arithmetic and hashes on the GPU
// (k_nym, one lane per signature).
#include <hip/hip_runtime.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "host/idemix.h"
#include "launch.h"
#include "rt_internal.h"

struct ftz_idemix {
  ftz_ctx* ctx = nullptr;
  uint8_t hash_slot[32] = {};  // copy(proofData[index:], ipk.Hash) into the 32-byte slot
  DBuf<QDev> tab;              // HSk and HRand fixed-base tables
  std::mutex mu;               // one call on the device at a time
  PinnedMem h_blob, h_ok;
  DevMem d_blob, d_ok;
};

extern "C" int ftz_idemix_create(ftz_ctx* ctx, const uint8_t* ipk, size_t ipk_len, int curve_id, ftz_idemix** out) {
  if (!ctx || !out || (!ipk && ipk_len)) return set_err(FTZ_E_INVALID, "null argument");
  if (curve_id != FTZ_CURVE_FP256BN_AMCL)
    return set_err(FTZ_E_INVALID, "unsupported idemix curve id " + std::to_string(curve_id) + " (FP256BN_AMCL only)");
  if (ipk_len == 0) return set_err(FTZ_E_PP, "empty idemix issuer public key");
  ftsh::IdemixIpk k;
  std::string e = ftsh::parse_ipk(ipk, ipk_len, k);
  if (!e.empty()) return set_err(FTZ_E_PP, e);
  q1a bases[2];
  if (!nym_point_from_be(k.hsk_x.data(), k.hsk_y.data(), bases[0]) ||
      !nym_point_from_be(k.hrand_x.data(), k.hrand_y.data(), bases[1]))
    return set_err(FTZ_E_PP, "issuer public key: HSk / HRand not on FP256BN");
  std::vector<QDev> tab(2 * NYM_TAB_PER_BASE);
  nym_build_tables(bases, tab.data());
  HC(hipSetDevice(ctx->device));
  ftz_idemix* ix = new ftz_idemix();
  ix->ctx = ctx;
  memcpy(ix->hash_slot, k.hash.data(), k.hash.size() < 32 ? k.hash.size() : 32);
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

// one device pass over the decoded signatures idx[a..b) of a call
namespace {
constexpr size_t NYM_CHUNK_BYTES = (size_t)1 << 30;  // keeps every blob offset in 32 bits

int nym_pass(ftz_idemix* ix, const ftz_owner_sig* s, const std::vector<uint32_t>& idx,
             const std::vector<ftsh::NymDecoded>& dec, size_t a, size_t b, int32_t* codes) {
  size_t m = b - a;
  size_t total = ftsh::nym_layout(s, idx.data() + a, m, dec.data(), ix->hash_slot, nullptr);
  HC(ix->h_blob.reserve(total));
  HC(ix->d_blob.reserve(total));
  HC(ix->h_ok.reserve(m));
  HC(ix->d_ok.reserve(m));
  ftsh::nym_layout(s, idx.data() + a, m, dec.data(), ix->hash_slot, ix->h_blob.p);
  hipStream_t st = ix->ctx->stream;
  HC(hipMemcpyAsync(ix->d_blob.p, ix->h_blob.p, total, hipMemcpyHostToDevice, st));
  k_nym<<<(uint32_t)((m + 63) / 64), 64, 0, st>>>(reinterpret_cast<const NymJob*>(ix->d_blob.p), (uint32_t)m,
                                                   ix->d_blob.p, ix->tab.p, ix->d_ok.p);
  HC(hipGetLastError());
  HC(hipMemcpyAsync(ix->h_ok.p, ix->d_ok.p, m, hipMemcpyDeviceToHost, st));
  HC(hipStreamSynchronize(st));
  for (size_t k = 0; k < m; k++) codes[idx[a + k]] = ix->h_ok.p[k] ? FTZ_OK : FTZ_ERR_SIGNATURE;
  return FTZ_SUCCESS;
}
}  // namespace

extern "C" int ftz_verify_owner_signatures(ftz_idemix* ix, size_t n, const ftz_owner_sig* s, int32_t* codes) {
  if (!ix || (n && (!s || !codes))) return set_err(FTZ_E_INVALID, "null argument");
  std::vector<ftsh::NymDecoded> dec(n);
  std::vector<uint32_t> idx;
  for (size_t i = 0; i < n; i++) {
    if ((!s[i].owner && s[i].owner_len) || (!s[i].msg && s[i].msg_len) || (!s[i].sig && s[i].sig_len))
      return set_err(FTZ_E_INVALID, "null buffer with non-zero length");
    if (s[i].msg_len > NYM_CHUNK_BYTES / 2) return set_err(FTZ_E_INVALID, "message larger than 512 MiB");
    ftsh::decode_owner_signature(s[i].owner, s[i].owner_len, s[i].sig, s[i].sig_len, dec[i]);
    codes[i] = dec[i].code;
    if (dec[i].code == 0) idx.push_back((uint32_t)i);
  }
  if (idx.empty()) return FTZ_SUCCESS;
  std::lock_guard<std::mutex> lk(ix->mu);
  HC(hipSetDevice(ix->ctx->device));
  // cut into device passes whose blob stays below NYM_CHUNK_BYTES
  size_t a = 0;
  while (a < idx.size()) {
    size_t b = a, bytes = 0;
    while (b < idx.size() && (b == a || bytes + s[idx[b]].msg_len + 512 < NYM_CHUNK_BYTES) && b - a < (1u << 20)) {
      bytes += s[idx[b]].msg_len + 512;
      b++;
    }
    int rc = nym_pass(ix, s, idx, dec, a, b, codes);
    if (rc != FTZ_SUCCESS) return rc;
    a = b;
  }
  return FTZ_SUCCESS;
}

// Host decoding for idemix owner-signature verification (idemix.h).
#include "idemix.h"

#include <string.h>

#include <map>

#include "../dev/idemix.h"
#include "gojson.h"

namespace ftsh {

// ---------------------------------------------------------------- protobuf
// google.golang.org/protobuf v1.27.1 wire rules: tags are varints with field
// number in [1, 2^29 - 1]; varints are at most 10 bytes (the 10th <= 1); wire
// types 3/4 are groups (skipped with a matching end marker), 6/7 are reserved.
namespace {

bool pb_varint(const uint8_t* b, size_t n, size_t& i, uint64_t& v, std::string& err) {
  v = 0;
  for (int k = 0; k < 10; k++) {
    if (i >= n) {
      err = "unexpected EOF";
      return false;
    }
    uint8_t c = b[i++];
    if (k == 9 && c > 1) {
      err = "variable length integer overflow";
      return false;
    }
    v |= (uint64_t)(c & 0x7f) << (7 * k);
    if (c < 0x80) return true;
  }
  err = "variable length integer overflow";
  return false;
}

bool pb_tag(const uint8_t* b, size_t n, size_t& i, uint32_t& num, uint8_t& wt, std::string& err) {
  uint64_t t;
  if (!pb_varint(b, n, i, t, err)) return false;
  uint64_t f = t >> 3;
  if (f < 1 || f > (1u << 29) - 1) {
    err = "invalid field number";
    return false;
  }
  num = (uint32_t)f;
  wt = (uint8_t)(t & 7);
  return true;
}

bool pb_skip(const uint8_t* b, size_t n, size_t& i, uint32_t num, uint8_t wt, int depth, std::string& err) {
  uint64_t v;
  switch (wt) {
    case 0:
      return pb_varint(b, n, i, v, err);
    case 1:
      if (n - i < 8) {
        err = "unexpected EOF";
        return false;
      }
      i += 8;
      return true;
    case 5:
      if (n - i < 4) {
        err = "unexpected EOF";
        return false;
      }
      i += 4;
      return true;
    case 2:
      if (!pb_varint(b, n, i, v, err)) return false;
      if (v > n - i) {
        err = "unexpected EOF";
        return false;
      }
      i += (size_t)v;
      return true;
    case 3:
      if (depth > 10000) {
        err = "exceeded maximum recursion depth";
        return false;
      }
      for (;;) {
        if (i >= n) {
          err = "unexpected EOF";
          return false;
        }
        uint32_t n2;
        uint8_t w2;
        if (!pb_tag(b, n, i, n2, w2, err)) return false;
        if (w2 == 4) {
          if (n2 != num) {
            err = "mismatching end group marker";
            return false;
          }
          return true;
        }
        if (!pb_skip(b, n, i, n2, w2, depth + 1, err)) return false;
      }
    default:
      err = "cannot parse reserved wire type";
      return false;
  }
}

}  // namespace

std::string pb_scan(const uint8_t* b, size_t n, std::vector<PbField>& out) {
  out.clear();
  size_t i = 0;
  std::string err;
  while (i < n) {
    uint32_t num;
    uint8_t wt;
    if (!pb_tag(b, n, i, num, wt, err)) return err;
    if (wt == 4) return "unexpected end group";
    PbField f{num, wt, 0, nullptr, 0};
    if (wt == 0) {
      if (!pb_varint(b, n, i, f.v, err)) return err;
    } else if (wt == 2) {
      uint64_t L;
      if (!pb_varint(b, n, i, L, err)) return err;
      if (L > n - i) return "unexpected EOF";
      f.p = b + i;
      f.len = (size_t)L;
      i += (size_t)L;
    } else {
      if (!pb_skip(b, n, i, num, wt, 0, err)) return err;
      continue;  // fixed32/64, groups: no field of these messages uses them
    }
    out.push_back(f);
  }
  return "";
}

bool utf8_valid(const uint8_t* p, size_t n) {
  size_t i = 0;
  while (i < n) {
    uint8_t c = p[i];
    if (c < 0x80) {
      i++;
      continue;
    }
    int len;
    uint32_t cp, lo_min;
    if ((c & 0xe0) == 0xc0) {
      len = 2, cp = c & 0x1f, lo_min = 0x80;
    } else if ((c & 0xf0) == 0xe0) {
      len = 3, cp = c & 0x0f, lo_min = 0x800;
    } else if ((c & 0xf8) == 0xf0) {
      len = 4, cp = c & 0x07, lo_min = 0x10000;
    } else {
      return false;
    }
    if (n - i < (size_t)len) return false;
    for (int k = 1; k < len; k++) {
      uint8_t d = p[i + k];
      if ((d & 0xc0) != 0x80) return false;
      cp = (cp << 6) | (d & 0x3f);
    }
    if (cp < lo_min || cp > 0x10ffff || (cp >= 0xd800 && cp <= 0xdfff)) return false;
    i += len;
  }
  return true;
}

namespace {

// proto3 field kinds of the messages read here
enum PbKind { PK_BYTES, PK_STRING, PK_ENUM };

// Decode a message whose known fields are all singular bytes / string / enum:
// the last occurrence wins; a known field with another wire type is unknown.
// present[k] / val[k] for field numbers 1..nf (kinds[k-1]).
std::string pb_simple(const uint8_t* b, size_t n, int nf, const PbKind* kinds, bool* present, PbField* val) {
  std::vector<PbField> fs;
  std::string e = pb_scan(b, n, fs);
  if (!e.empty()) return e;
  for (int k = 0; k < nf; k++) present[k] = false;
  for (const PbField& f : fs) {
    if (f.num < 1 || (int)f.num > nf) continue;
    PbKind kd = kinds[f.num - 1];
    uint8_t want = kd == PK_ENUM ? 0 : 2;
    if (f.wt != want) continue;
    if (kd == PK_STRING && !utf8_valid(f.p, f.len)) return "string field contains invalid UTF-8";
    present[f.num - 1] = true;
    val[f.num - 1] = f;
  }
  return "";
}

// ---------------------------------------------------------------- ASN.1 RawOwner
// Go 1.18 encoding/asn1: definite minimal lengths; a string field takes
// PrintableString / IA5String / T61String / UTF8String / NumericString /
// BMPString / GeneralString with that type's character rules.
bool der_tlv(const uint8_t* b, size_t n, size_t& off, uint8_t& tag, size_t& len) {
  if (off >= n) return false;
  tag = b[off++];
  if ((tag & 0x1f) == 0x1f) return false;  // high-tag-number form: no universal tag used here fits
  if (off >= n) return false;
  uint8_t c = b[off++];
  size_t L = 0;
  if (c & 0x80) {
    int nb = c & 0x7f;
    if (nb == 0) return false;
    for (int k = 0; k < nb; k++) {
      if (off >= n) return false;
      if (L >= (1u << 23)) return false;
      L = (L << 8) | b[off++];
      if (L == 0) return false;
    }
    if (L < 0x80) return false;
  } else {
    L = c;
  }
  if (L > n - off) return false;
  len = L;
  return true;
}

bool printable(uint8_t c) {
  return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || strchr(" '()+,-./:=?*&", c) != nullptr;
}

// decode an ASN.1 string of universal tag `tag` into UTF-8 (false: Go rejects it)
bool asn1_string(uint8_t tag, const uint8_t* p, size_t n, std::string& out) {
  out.clear();
  switch (tag) {
    case 0x13:  // PrintableString
      for (size_t i = 0; i < n; i++)
        if (!printable(p[i]) || p[i] == 0) return false;
      out.assign((const char*)p, n);
      return true;
    case 0x16:  // IA5String
      for (size_t i = 0; i < n; i++)
        if (p[i] >= 0x80) return false;
      out.assign((const char*)p, n);
      return true;
    case 0x14:  // T61String
    case 0x1b:  // GeneralString: passed as 8-bit bytes
      out.assign((const char*)p, n);
      return true;
    case 0x0c:  // UTF8String
      if (!utf8_valid(p, n)) return false;
      out.assign((const char*)p, n);
      return true;
    case 0x12:  // NumericString
      for (size_t i = 0; i < n; i++)
        if (!((p[i] >= '0' && p[i] <= '9') || p[i] == ' ')) return false;
      out.assign((const char*)p, n);
      return true;
    case 0x1e: {  // BMPString: UTF-16BE, a trailing NUL pair stripped
      if (n % 2) return false;
      if (n >= 2 && p[n - 1] == 0 && p[n - 2] == 0) n -= 2;
      for (size_t i = 0; i < n; i += 2) {
        uint32_t u = ((uint32_t)p[i] << 8) | p[i + 1];
        if (u >= 0xd800 && u < 0xdc00 && i + 2 < n) {
          uint32_t u2 = ((uint32_t)p[i + 2] << 8) | p[i + 3];
          if (u2 >= 0xdc00 && u2 < 0xe000) {
            u = 0x10000 + ((u - 0xd800) << 10) + (u2 - 0xdc00);
            i += 2;
          } else {
            u = 0xfffd;
          }
        } else if (u >= 0xd800 && u < 0xe000) {
          u = 0xfffd;
        }
        if (u < 0x80) {
          out.push_back((char)u);
        } else if (u < 0x800) {
          out.push_back((char)(0xc0 | (u >> 6)));
          out.push_back((char)(0x80 | (u & 0x3f)));
        } else if (u < 0x10000) {
          out.push_back((char)(0xe0 | (u >> 12)));
          out.push_back((char)(0x80 | ((u >> 6) & 0x3f)));
          out.push_back((char)(0x80 | (u & 0x3f)));
        } else {
          out.push_back((char)(0xf0 | (u >> 18)));
          out.push_back((char)(0x80 | ((u >> 12) & 0x3f)));
          out.push_back((char)(0x80 | ((u >> 6) & 0x3f)));
          out.push_back((char)(0x80 | (u & 0x3f)));
        }
      }
      return true;
    }
    default:
      return false;
  }
}

// identity.UnmarshallRawOwner (identity/owner.go:30-37)
bool raw_owner(const uint8_t* b, size_t n, std::string& type, const uint8_t*& ident, size_t& ident_len) {
  size_t off = 0, len;
  uint8_t tag;
  if (!der_tlv(b, n, off, tag, len) || tag != 0x30) return false;
  const uint8_t* s = b + off;
  size_t k = 0, l1;
  if (!der_tlv(s, len, k, tag, l1)) return false;
  if (!asn1_string(tag, s + k, l1, type)) return false;
  k += l1;
  size_t l2;
  if (!der_tlv(s, len, k, tag, l2) || tag != 0x04) return false;
  ident = s + k;
  ident_len = l2;
  return true;  // trailing elements inside the SEQUENCE and bytes after it are ignored
}

}  // namespace

std::string parse_ipk(const uint8_t* p, size_t n, IdemixIpk& out) {
  std::vector<PbField> fs;
  std::string e = pb_scan(p, n, fs);
  if (!e.empty()) return "issuer public key: " + e;
  bool have_hsk = false, have_hrand = false;
  for (const PbField& f : fs) {
    if (f.wt != 2) continue;
    if (f.num == 1 && !utf8_valid(f.p, f.len)) return "issuer public key: invalid UTF-8 attribute name";
    if (f.num == 2 || f.num == 3) {  // ECP{X = 1, Y = 2}; a repeated singular message merges
      static const PbKind kinds[2] = {PK_BYTES, PK_BYTES};
      bool pr[2];
      PbField v[2];
      e = pb_simple(f.p, f.len, 2, kinds, pr, v);
      if (!e.empty()) return "issuer public key: " + e;
      std::vector<uint8_t>& x = f.num == 2 ? out.hsk_x : out.hrand_x;
      std::vector<uint8_t>& y = f.num == 2 ? out.hsk_y : out.hrand_y;
      if (pr[0]) x.assign(v[0].p, v[0].p + v[0].len);
      if (pr[1]) y.assign(v[1].p, v[1].p + v[1].len);
      (f.num == 2 ? have_hsk : have_hrand) = true;
    }
    if (f.num == 4) {  // repeated ECP HAttrs
      static const PbKind kinds[2] = {PK_BYTES, PK_BYTES};
      bool pr[2];
      PbField v[2];
      e = pb_simple(f.p, f.len, 2, kinds, pr, v);
      if (!e.empty()) return "issuer public key: " + e;
      out.hattrs_x.emplace_back(pr[0] ? std::vector<uint8_t>(v[0].p, v[0].p + v[0].len) : std::vector<uint8_t>());
      out.hattrs_y.emplace_back(pr[1] ? std::vector<uint8_t>(v[1].p, v[1].p + v[1].len) : std::vector<uint8_t>());
    }
    if (f.num == 10) out.hash.assign(f.p, f.p + f.len);
  }
  if (!have_hsk || !have_hrand) return "issuer public key: some part of the public key is undefined";
  if (out.hsk_x.size() < 32 || out.hsk_y.size() < 32 || out.hrand_x.size() < 32 || out.hrand_y.size() < 32)
    return "issuer public key: coordinate shorter than 32 bytes";
  return "";
}

namespace {
// strip leading zero bytes of a big-endian integer
void be_strip(const uint8_t*& p, size_t& n) {
  while (n && *p == 0) {
    p++;
    n--;
  }
}
// big-endian integer of at most 32 significant bytes -> 32 bytes; false if wider
bool be_to32(const uint8_t* p, size_t n, uint8_t out[32]) {
  be_strip(p, n);
  if (n > 32) return false;
  memset(out, 0, 32 - n);
  if (n) memcpy(out + 32 - n, p, n);
  return true;
}
bool be32_geq_r(const uint8_t b[32]) {
  uint32_t v[8], t[8], rm[8];
  fts::be32_to_limbs(v, b);
  for (int i = 0; i < 8; i++) rm[i] = fts::R_MOD[i];
  return fts::sub8(t, v, rm) == 0;
}
void canon_xy(const fts::g1a& a, uint8_t x[32], uint8_t y[32]) {
  uint32_t t[8];
  if (a.inf) {
    memset(x, 0, 32);
    memset(y, 0, 32);
    return;
  }
  fts::fe_to_int(t, a.x);
  fts::limbs_to_be32(x, t);
  fts::fe_to_int(t, a.y);
  fts::limbs_to_be32(y, t);
}
}  // namespace

void be_mod_r(const uint8_t* p, size_t n, uint8_t out[32]) {
  using namespace fts;
  be_strip(p, n);
  uint32_t w[8] = {0, 1, 0, 0, 0, 0, 0, 0};
  const fr two32 = fe_from_int<ModR>(w);
  fr acc = fe_zero<ModR>();
  size_t lead = n % 4;
  auto word = [&](uint32_t v) {
    uint32_t a[8] = {v, 0, 0, 0, 0, 0, 0, 0};
    acc = acc * two32 + fe_from_int<ModR>(a);
  };
  if (lead) {
    uint32_t v = 0;
    for (size_t i = 0; i < lead; i++) v = (v << 8) | p[i];
    word(v);
  }
  for (size_t i = lead; i < n; i += 4)
    word(((uint32_t)p[i] << 24) | ((uint32_t)p[i + 1] << 16) | ((uint32_t)p[i + 2] << 8) | p[i + 3]);
  uint32_t t[8];
  fe_to_int(t, acc);
  limbs_to_be32(out, t);
}

void decode_owner_signature(const uint8_t* owner, size_t owner_len, const uint8_t* sig, size_t sig_len,
                            NymDecoded& out, int curve) {
  out.code = 0;
  out.why.clear();
  auto fail = [&](int code, const char* why) {
    out.code = code;
    out.why = why;
  };
  // ---- GetOwnerVerifier: htlc.Deserializer -> RawOwnerIdentityDeserializer -> idemix
  std::string type;
  const uint8_t* ident;
  size_t ident_len;
  if (!raw_owner(owner, owner_len, type, ident, ident_len)) return fail(FTZ_ERR_OWNER, "failed to unmarshal RawOwner");
  if (type == "htlc") return fail(FTZ_ERR_UNSUPPORTED, "htlc script owner: verified in Go");
  if (type != "si") {
    out.code = FTZ_ERR_OWNER;
    out.why = "failed to deserialize RawOwner: Unknown owner type " + type;
    return;
  }
  static const PbKind k_si[2] = {PK_STRING, PK_BYTES};
  bool pr[5];
  PbField v[5];
  if (!pb_simple(ident, ident_len, 2, k_si, pr, v).empty())
    return fail(FTZ_ERR_OWNER, "failed to unmarshal to msp.SerializedIdentity{}");
  const uint8_t* idb = pr[1] ? v[1].p : nullptr;
  size_t idn = pr[1] ? v[1].len : 0;
  static const PbKind k_ser[5] = {PK_BYTES, PK_BYTES, PK_BYTES, PK_BYTES, PK_BYTES};
  if (!pb_simple(idb, idn, 5, k_ser, pr, v).empty())
    return fail(FTZ_ERR_OWNER, "could not deserialize a SerializedIdemixIdentity");
  // proto3 bytes without presence decode through consumeBytesNoZero (append([]byte(nil), v...)):
  // an empty NymX / NymY is nil even when it is on the wire (common.go:52 nil check)
  if (!pr[0] || !pr[1] || v[0].len == 0 || v[1].len == 0)
    return fail(FTZ_ERR_OWNER, "unable to deserialize idemix identity: pseudonym is invalid");
  // NymPublicKey import: raw = NymX || NymY split in halves.  FP256BN: FromBytes
  // reads 32 bytes of each (NewECPbigs later); BN254: G1FromProto wants halves of
  // exactly 32 bytes and gnark SetBytes must accept X || Y
  size_t tot = v[0].len + v[1].len, half = tot / 2;
  bool bn = curve == FTZ_CURVE_BN254;
  if (half < 32 || (bn && tot != 64)) return fail(FTZ_ERR_OWNER, "failed to import nym public key");
  auto raw_at = [&](size_t i) { return i < v[0].len ? v[0].p[i] : v[1].p[i - v[0].len]; };
  for (int i = 0; i < 32; i++) {
    out.ints[0][i] = raw_at(i);
    out.ints[1][i] = raw_at(half + i);
  }
  if (bn) {
    fts::g1a a;
    if (!fts::bn_point_from_xy(out.ints[0], out.ints[1], a)) return fail(FTZ_ERR_OWNER, "failed to import nym public key");
    canon_xy(a, out.ints[0], out.ints[1]);
  }
  PbField ou = v[2], role = v[3];
  bool has_ou = pr[2], has_role = pr[3];
  static const PbKind k_ou[3] = {PK_STRING, PK_STRING, PK_BYTES};
  if (!pb_simple(has_ou ? ou.p : nullptr, has_ou ? ou.len : 0, 3, k_ou, pr, v).empty())
    return fail(FTZ_ERR_OWNER, "cannot deserialize the OU of the identity");
  static const PbKind k_role[2] = {PK_STRING, PK_ENUM};
  if (!pb_simple(has_role ? role.p : nullptr, has_role ? role.len : 0, 2, k_role, pr, v).empty())
    return fail(FTZ_ERR_OWNER, "cannot deserialize the role of the identity");
  // ---- Verifier.Verify: the NymSignature proto
  if (sig_len == 0) return fail(FTZ_ERR_SIGNATURE, "invalid signature, it must not be empty");
  static const PbKind k_sig[4] = {PK_BYTES, PK_BYTES, PK_BYTES, PK_BYTES};
  std::string pe = pb_simple(sig, sig_len, 4, k_sig, pr, v);
  if (!pe.empty()) {
    out.code = FTZ_ERR_SIGNATURE;
    out.why = "error unmarshalling signature: " + pe;
    return;
  }
  if (bn) {  // big.Int SetBytes over each whole field (absent = 0)
    const uint8_t* fp_[4];
    size_t fl[4];
    for (int q = 0; q < 4; q++) {
      fp_[q] = pr[q] ? v[q].p : nullptr;
      fl[q] = pr[q] ? v[q].len : 0;
    }
    // Zr.Bytes() of the Nonce (common.BigToBytes): an integer >= 2^256 panics
    // [EXT, parity unpinned: no reference file holds a BN254 NymSignature;
    // tests/golden/idemix_bn254_golden.json "parity"]
    if (!be_to32(fp_[3], fl[3], out.ints[5]))
      return fail(FTZ_ERR_SIGNATURE, "failure [runtime error: makeslice: len out of range]");
    uint8_t cr[32];
    be_mod_r(fp_[0], fl[0], cr);
    // ProofC >= r (or longer than 32 bytes) can never equal HashToZr(c || Nonce) < r:
    // an all-ones sentinel that no hash matches [EXT, parity unpinned]
    if (!be_to32(fp_[0], fl[0], out.ints[2]) || be32_geq_r(out.ints[2])) memset(out.ints[2], 0xff, 32);
    be_mod_r(fp_[1], fl[1], out.ints[3]);
    be_mod_r(fp_[2], fl[2], out.ints[4]);
    nym_glv_split_bn(cr, out.glv);
    return;
  }
  for (int q = 0; q < 4; q++) {
    if (!pr[q] || v[q].len < 32) return fail(FTZ_ERR_SIGNATURE, "failure [index out of range]");
    memcpy(out.ints[2 + q], v[q].p, 32);
  }
  nym_glv_split(out.ints[2], out.glv);
}

namespace {
// little-endian 32-bit limb arithmetic for the host GLV split
void mp_mul(const uint32_t* a, int na, const uint32_t* b, int nb, uint32_t* r) {
  for (int i = 0; i < na + nb; i++) r[i] = 0;
  for (int i = 0; i < na; i++) {
    uint64_t c = 0;
    for (int j = 0; j < nb; j++) {
      uint64_t t = (uint64_t)a[i] * b[j] + r[i + j] + c;
      r[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    r[i + nb] = (uint32_t)c;
  }
}
int mp_cmp(const uint32_t* a, const uint32_t* b, int n) {
  for (int i = n - 1; i >= 0; i--)
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return 0;
}
void mp_sub(uint32_t* r, const uint32_t* a, const uint32_t* b, int n) {
  uint64_t br = 0;
  for (int i = 0; i < n; i++) {
    uint64_t t = (uint64_t)a[i] - b[i] - br;
    r[i] = (uint32_t)t;
    br = (t >> 63) & 1;
  }
}
void mp_add(uint32_t* r, const uint32_t* a, const uint32_t* b, int n) {
  uint64_t c = 0;
  for (int i = 0; i < n; i++) {
    uint64_t t = (uint64_t)a[i] + b[i] + c;
    r[i] = (uint32_t)t;
    c = t >> 32;
  }
}
// |x - y| and the sign of x - y (n limbs)
bool mp_signed_diff(uint32_t* r, const uint32_t* x, const uint32_t* y, int n) {
  if (mp_cmp(x, y, n) >= 0) {
    mp_sub(r, x, y, n);
    return false;
  }
  mp_sub(r, y, x, n);
  return true;
}
}  // namespace

void nym_glv_split(const uint8_t kb[32], uint32_t out[12]) {
  uint32_t k[12] = {0}, t[24];
  fts::be32_to_limbs(k, kb);
  if (mp_cmp(k, fts::N_MOD, 8) >= 0) mp_sub(k, k, fts::N_MOD, 8);  // k < 2^256 < 2n
  uint32_t c1[12] = {0}, c2[12] = {0};
  mp_mul(k, 8, fts::Q_GLV_G1, 8, t);
  for (int i = 0; i < 8; i++) c1[i] = t[8 + i];
  mp_mul(k, 8, fts::Q_GLV_G2, 8, t);
  for (int i = 0; i < 8; i++) c2[i] = t[8 + i];
  // k1 = k - c1 a1 - c2 a2, k2 = c1 |b1| - c2 b2 (c_i < 2^130, basis entries < 2^129)
  uint32_t x[12], y[12], z[12], k1[12], k2[12];
  mp_mul(c1, 6, fts::Q_GLV_A1, 6, x);
  mp_mul(c2, 6, fts::Q_GLV_A2, 6, y);
  mp_add(z, x, y, 12);
  bool n1 = mp_signed_diff(k1, k, z, 12);
  mp_mul(c1, 6, fts::Q_GLV_B1ABS, 6, x);
  mp_mul(c2, 6, fts::Q_GLV_B2, 6, y);
  bool n2 = mp_signed_diff(k2, x, y, 12);
  for (int i = 0; i < 5; i++) {
    out[i] = k1[i];
    out[5 + i] = k2[i];
  }
  out[10] = (n1 ? 1u : 0u) | (n2 ? 2u : 0u);
  out[11] = 0;
}

void nym_glv_split_bn(const uint8_t kb[32], uint32_t out[12]) {
  uint32_t k[8], k1[4], k2[4];
  bool n1, n2;
  fts::be32_to_limbs(k, kb);
  fts::glv_split(k, k1, n1, k2, n2);
  for (int i = 0; i < 4; i++) {
    out[i] = k1[i];
    out[5 + i] = k2[i];
  }
  out[4] = out[9] = 0;
  out[10] = (n1 ? 1u : 0u) | (n2 ? 2u : 0u);
  out[11] = 0;
}

void nym_plan_layout(const ftz_owner_sig* s, const uint32_t* idx, size_t m, NymLayout& L, int curve) {
  constexpr size_t PER_JOB = fts::NYM_SC_BYTES + fts::NYM_PRE_SLOT;
  const size_t align = (curve == FTZ_CURVE_BN254 ? fts::NymCurve<fts::fp>::PRE : fts::NymCurve<fts::fq>::PRE) % 16;
  size_t off = ((m * sizeof(fts::NymJob) + 15) & ~(size_t)15) + m * PER_JOB;
  std::map<std::pair<const uint8_t*, size_t>, uint32_t> at;
  L.msg_off.resize(m);
  L.distinct.clear();
  for (size_t k = 0; k < m; k++) {
    const ftz_owner_sig& q = s[idx[k]];
    auto key = std::make_pair(q.msg, q.msg_len);
    auto it = at.find(key);
    if (it == at.end()) {
      off = ((off + 15) & ~(size_t)15) + align;
      it = at.emplace(key, (uint32_t)off).first;
      L.distinct.push_back({(uint32_t)off, (uint32_t)k});
      off += q.msg_len;
    }
    L.msg_off[k] = it->second;
  }
  L.total = off + 64;  // + slack: the hash reads whole 16-byte words
}

void nym_fill(const ftz_owner_sig* s, const uint32_t* idx, size_t m, const NymDecoded* dec,
              const std::vector<uint8_t>& ipk_hash, const NymLayout& L, uint8_t* blob,
              const std::function<void(size_t, const std::function<void(size_t)>&)>& par, int curve) {
  constexpr size_t SC = fts::NYM_SC_BYTES, PRE = fts::NYM_PRE_SLOT, PIECE = 256;
  const bool bn = curve == FTZ_CURVE_BN254;
  // copy(proofData[4 + 2 G:], ipk.Hash): the 32-byte slot after t and Nym (G = 65 / 64)
  const size_t hash_at = bn ? 4 + 2 * 64 : 4 + 2 * 65, tail_at = fts::NymCurve<fts::fp>::PRE;
  uint8_t hash_slot[32] = {};
  memcpy(hash_slot, ipk_hash.data(), ipk_hash.size() < 32 ? ipk_hash.size() : 32);
  size_t base = (m * sizeof(fts::NymJob) + 15) & ~(size_t)15;
  size_t jp = (m + PIECE - 1) / PIECE, mp = (L.distinct.size() + 15) / 16;
  par(jp + mp, [&](size_t p) {
    if (p < jp) {
      for (size_t k = p * PIECE; k < m && k < (p + 1) * PIECE; k++) {
        fts::NymJob j;
        j.sc = (uint32_t)(base + k * (SC + PRE));
        j.pre = (uint32_t)(j.sc + SC);
        j.msg = L.msg_off[k];
        j.msg_len = (uint32_t)s[idx[k]].msg_len;
        memcpy(blob + k * sizeof(fts::NymJob), &j, sizeof j);
        memcpy(blob + j.sc, dec[idx[k]].ints, 192);
        memcpy(blob + j.sc + 192, dec[idx[k]].glv, 48);
        uint8_t* pre = blob + j.pre;
        memset(pre, 0, PRE);
        memcpy(pre, "sign", 4);
        memcpy(pre + hash_at, hash_slot, 32);
        if (bn)  // BN254: the 2 bytes after the message are ipk.Hash's bytes there, if it is that long, else 0
          for (size_t q = 0; q < 2; q++) {
            size_t hi = 32 + j.msg_len + q;
            pre[tail_at + q] = hi < ipk_hash.size() ? ipk_hash[hi] : 0;
          }
      }
    } else {
      size_t d0 = (p - jp) * 16;
      for (size_t d = d0; d < L.distinct.size() && d < d0 + 16; d++) {
        const ftz_owner_sig& q = s[idx[L.distinct[d].second]];
        if (q.msg_len) memcpy(blob + L.distinct[d].first, q.msg, q.msg_len);
      }
    }
  });
}

}  // namespace ftsh

namespace ftsh {

namespace {

// a singular message field (possibly repeated on the wire: occurrences merge):
// decode each occurrence's ECP{X = 1, Y = 2}, the last X / Y present wins
std::string merge_ecp(const PbField& f, std::vector<uint8_t>& x, std::vector<uint8_t>& y, bool& seen) {
  static const PbKind kinds[2] = {PK_BYTES, PK_BYTES};
  bool pr[2];
  PbField v[2];
  std::string e = pb_simple(f.p, f.len, 2, kinds, pr, v);
  if (!e.empty()) return e;
  if (pr[0]) x.assign(v[0].p, v[0].p + v[0].len);
  if (pr[1]) y.assign(v[1].p, v[1].p + v[1].len);
  seen = true;
  return "";
}

// mathlib Zr UnmarshalJSON on the idemix curve: D_NIL, D_OK, D_ERR (Unmarshal
// error), D_PANIC (a Zr of another curve: the driver's type assertion on use).
// FP256BN_AMCL: FromBytes reads the first 32 raw bytes (a shorter element
// panics); BN254: big.Int SetBytes over the whole element, out = its value mod r.
DecStatus zr_json(const JDoc& d, int64_t node, uint8_t out[32], int want_curve) {
  if (node < 0 || d.at((uint32_t)node).type == J_NULL) return D_NIL;
  if (d.at((uint32_t)node).type != J_OBJ) return D_ERR;
  int64_t curve = 0;
  if (dec_int(d, d.field((uint32_t)node, "curve"), curve) == D_ERR) return D_ERR;
  std::vector<uint8_t> raw;
  if (dec_bytes(d, d.field((uint32_t)node, "element"), raw) == D_ERR) return D_ERR;
  if (curve != want_curve) return D_PANIC;
  if (want_curve == FTZ_CURVE_BN254) {
    be_mod_r(raw.data(), raw.size(), out);
    return D_OK;
  }
  if (raw.size() < 32) return D_PANIC;
  memcpy(out, raw.data(), 32);
  return D_OK;
}

}  // namespace

// crypto/audit/auditor.go:252-274 InspectTokenOwner up to the curve arithmetic
// of AuditInfo.Match (identity/msp/idemix/audit.go:51-83); see idemix.h
void decode_owner_audit(const uint8_t* owner, size_t owner_len, const uint8_t* ai, size_t ai_len, size_t n_hattrs,
                        EidDecoded& out, int curve) {
  out = EidDecoded();
  auto fail = [&](int code, const std::string& why) {
    out.code = code;
    out.why = why;
  };
  if (owner_len == 0) return fail(FTZ_ERR_OWNER, "token is a redeem token, cannot inspect ownership");
  if (ai_len == 0) return fail(FTZ_ERR_OWNER, "failed to inspect owner: owner info is nil");
  std::string type;
  const uint8_t* ident;
  size_t ident_len;
  if (!raw_owner(owner, owner_len, type, ident, ident_len)) return fail(FTZ_ERR_OWNER, "owner cannot be unwrapped");
  if (type != "si") return fail(FTZ_ERR_UNSUPPORTED, "script owner: inspected in Go");
  // GetOwnerMatcher: json.Unmarshal(OwnerInfo, &AuditInfo{}) -- RNymEid and EID of the
  // embedded *NymEIDAuditData, Attributes [][]byte
  JDoc d;
  if (!d.parse(ai, ai_len)) return fail(FTZ_ERR_OWNER, "failed to get owner matcher");
  uint32_t root = d.root();
  bool nil_ai = d.at(root).type == J_NULL;
  if (!nil_ai && d.at(root).type != J_OBJ) return fail(FTZ_ERR_OWNER, "failed to get owner matcher");
  DecStatus rs = D_NIL;
  std::vector<std::vector<uint8_t>> attrs;
  bool attrs_nil = true;
  if (!nil_ai) {
    uint8_t tmp[32];
    rs = zr_json(d, d.field(root, "RNymEid"), out.rnym, curve);
    DecStatus es = zr_json(d, d.field(root, "EID"), tmp, curve);
    if (rs == D_ERR || es == D_ERR) return fail(FTZ_ERR_OWNER, "failed to get owner matcher");
    int64_t an = d.field(root, "Attributes");
    if (an >= 0 && d.at((uint32_t)an).type != J_NULL) {
      if (d.at((uint32_t)an).type != J_ARR) return fail(FTZ_ERR_OWNER, "failed to get owner matcher");
      attrs_nil = false;
      for (uint32_t k = 0; k < d.len((uint32_t)an); k++) {
        std::vector<uint8_t> b;
        if (dec_bytes(d, d.elem((uint32_t)an, k), b) == D_ERR) return fail(FTZ_ERR_OWNER, "failed to get owner matcher");
        attrs.push_back(std::move(b));
      }
    }
    if (rs == D_PANIC || es == D_PANIC) return fail(FTZ_ERR_PANIC, "panic: mathlib Zr of another curve");
  }
  // Match: the msp protos
  static const PbKind k_si[2] = {PK_STRING, PK_BYTES};
  bool pr[5];
  PbField v[5];
  if (!pb_simple(ident, ident_len, 2, k_si, pr, v).empty())
    return fail(FTZ_ERR_AUDIT, "failed to unmarshal to msp.SerializedIdentity{}");
  const uint8_t* idb = pr[1] ? v[1].p : nullptr;
  size_t idn = pr[1] ? v[1].len : 0;
  static const PbKind k_ser[5] = {PK_BYTES, PK_BYTES, PK_BYTES, PK_BYTES, PK_BYTES};
  if (!pb_simple(idb, idn, 5, k_ser, pr, v).empty())
    return fail(FTZ_ERR_AUDIT, "could not deserialize a SerializedIdemixIdentity");
  const uint8_t* proof = pr[4] ? v[4].p : nullptr;
  size_t proof_len = pr[4] ? v[4].len : 0;
  // EidNymAuditOpts{EnrollmentID: string(a.Attributes[2])}: index out of range panics
  if (attrs_nil || attrs.size() <= 2) return fail(FTZ_ERR_PANIC, "panic: index out of range");
  // AuditNymEid: the idemix Signature proto of the identity's proof
  std::vector<PbField> fs;
  std::string pe = pb_scan(proof, proof_len, fs);
  if (!pe.empty()) return fail(FTZ_ERR_AUDIT, "error while verifying the nym eid: " + pe);
  std::vector<uint8_t> ex, ey;
  bool eid_nym = false, nym_seen = false;
  static const PbKind k_nonrev[2] = {PK_ENUM, PK_BYTES};
  static const PbKind k_ecp2[4] = {PK_BYTES, PK_BYTES, PK_BYTES, PK_BYTES};
  for (const PbField& f : fs) {
    if (f.num == 16 || f.wt != 2 || f.num > 18) continue;  // epoch (varint) / unknown / wrong wire type
    std::vector<uint8_t> dx, dy;
    bool dummy = false;
    std::string e;
    if (f.num == 1 || f.num == 2 || f.num == 3 || f.num == 12) e = merge_ecp(f, dx, dy, dummy);
    if (f.num == 14) e = pb_simple(f.p, f.len, 4, k_ecp2, pr, v);
    if (f.num == 17) e = pb_simple(f.p, f.len, 2, k_nonrev, pr, v);
    if (f.num == 18) {  // EIDNym{Nym = 1 (ECP), ProofSEid = 2}
      std::vector<PbField> es;
      e = pb_scan(f.p, f.len, es);
      for (size_t q = 0; e.empty() && q < es.size(); q++)
        if (es[q].num == 1 && es[q].wt == 2) e = merge_ecp(es[q], ex, ey, nym_seen);
      eid_nym = true;
    }
    if (!e.empty()) return fail(FTZ_ERR_AUDIT, "error while verifying the nym eid: " + e);
  }
  if (!eid_nym || !nym_seen) return fail(FTZ_ERR_AUDIT, "error while verifying the nym eid: no EidNym provided");
  if (n_hattrs <= 2)
    return fail(FTZ_ERR_AUDIT, "error while verifying the nym eid: could not access H_a_eid in array");
  if (curve == FTZ_CURVE_BN254) {
    // AuditNymEid on BN254: EidNym through G1FromProto (an error is a Match
    // error) before Mul2 dereferences RNymEid
    fts::g1a a;
    if (ex.size() != 32 || ey.size() != 32 || !fts::bn_point_from_xy(ex.data(), ey.data(), a))
      return fail(FTZ_ERR_AUDIT, "error while verifying the nym eid: could not deserialize EidNym");
    if (nil_ai || rs == D_NIL) return fail(FTZ_ERR_PANIC, "panic: nil RNymEid");
    canon_xy(a, out.nym_x, out.nym_y);
  } else {
    if (nil_ai || rs == D_NIL) return fail(FTZ_ERR_PANIC, "panic: nil RNymEid");
    if (ex.size() < 32 || ey.size() < 32) return fail(FTZ_ERR_PANIC, "panic: index out of range");
    memcpy(out.nym_x, ex.data(), 32);
    memcpy(out.nym_y, ey.data(), 32);
  }
  // HashToZr(EnrollmentID): SHA-256 read big-endian, reduced mod n on the device
  fts::Sha256 h;
  h.init();
  h.update(attrs[2].data(), attrs[2].size());
  h.final(out.eid_digest);
}

}  // namespace ftsh

// Host decoding of raw token requests (request.h).
#include "request.h"

#include <string.h>

#include <thread>

#include "gojson.h"

namespace ftsh {

// ---------------------------------------------------------------- ASN.1 DER
// Go encoding/asn1 (Go 1.18) parseTagAndLength + parseField / parseSequenceOf
// restricted to driver.TokenRequest.  Tags: class universal, the compound bit
// and tag number must match exactly, and a high-tag-number form of a tag below
// 31 is "non-minimal", so the identifier byte is exactly 0x30 or 0x04.
namespace {

struct Der {
  const uint8_t* b;
  size_t n;
};

// header at off: identifier byte must be `want`; on success body = [off, off+len)
std::string der_header(const Der& d, size_t& off, uint8_t want, size_t& len) {
  if (off >= d.n) return "sequence truncated";
  uint8_t id = d.b[off++];
  if ((id & 0x1f) == 0x1f) {  // high-tag-number form: tags 4 and 16 cannot use it
    return "tags don't match";
  }
  if (id != want) return "tags don't match";
  if (off >= d.n) return "truncated tag or length";
  uint8_t b = d.b[off++];
  size_t L = 0;
  if (b & 0x80) {
    int nb = b & 0x7f;
    if (nb == 0) return "indefinite length found (not DER)";
    for (int k = 0; k < nb; k++) {
      if (off >= d.n) return "truncated tag or length";
      uint8_t v = d.b[off++];
      if (L >= (1u << 23)) return "length too large";
      L = (L << 8) | v;
      if (L == 0) return "superfluous leading zeros in length";
    }
    if (L < 0x80) return "non-minimal length";
  } else {
    L = b & 0x7f;
  }
  if (L > d.n - off) return "data truncated";
  len = L;
  return "";
}

// SEQUENCE OF OCTET STRING at off (advances off past it)
std::string der_seq_of_octets(const Der& d, size_t& off, std::vector<Slice>& out) {
  size_t len;
  std::string e = der_header(d, off, 0x30, len);
  if (!e.empty()) return e;
  Der inner{d.b + off, len};
  size_t k = 0;
  out.clear();
  while (k < inner.n) {
    size_t el;
    e = der_header(inner, k, 0x04, el);
    if (!e.empty()) return e == "tags don't match" ? "sequence tag mismatch" : e;
    out.push_back(Slice{inner.b + k, el});
    k += el;
  }
  off += len;
  return "";
}

}  // namespace

std::string der_token_request(const uint8_t* raw, size_t len, std::vector<Slice> out[4]) {
  for (int f = 0; f < 4; f++) out[f].clear();
  if (len == 0) return "empty token request";
  Der d{raw, len};
  size_t off = 0, body;
  std::string e = der_header(d, off, 0x30, body);
  if (!e.empty()) return "failed to unmarshal token request: " + e;
  Der inner{raw + off, body};
  size_t k = 0;
  for (int f = 0; f < 4; f++) {
    e = der_seq_of_octets(inner, k, out[f]);
    if (!e.empty()) return "failed to unmarshal token request: " + e;
  }
  // bytes after the fourth field (inside the SEQUENCE) and after the SEQUENCE
  // are ignored, as Go's parseField and FromBytes do
  return "";
}

// ---------------------------------------------------------------- JSON actions
namespace {

DecStatus dec_bool(const JDoc& d, int64_t node, bool& out) {
  if (node < 0 || d.at((uint32_t)node).type == J_NULL) return D_NIL;  // left unchanged
  if (d.at((uint32_t)node).type != J_BOOL) return D_ERR;
  out = d.at((uint32_t)node).bval != 0;
  return D_OK;
}

// math.G1 field: decoded into a 64-byte slot of `pool` (gnark SetBytes reads 64
// bytes for an uncompressed encoding and 32 for a compressed one; the rest of
// the slot is zero).  A buffer too short for its flags fails SetBytes inside
// UnmarshalJSON whatever the curve arithmetic says (`bad`).
DecStatus dec_g1(const JDoc& d, int64_t node, ElemRef& r, std::vector<uint8_t>& pool) {
  ElemBytes e = dec_elem(d, node);
  r.st = e.st;
  r.bad = 0;
  r.off = 0;
  if (e.st != D_OK && e.st != D_PANIC) return e.st;
  size_t L = e.raw.size();
  uint8_t m = L ? (e.raw[0] & 0xC0) : 0;
  if (L < 32 || (m == 0x00 && L < 64)) r.bad = 1;
  r.off = pool.size();
  pool.resize(r.off + 64, 0);
  memcpy(pool.data() + r.off, e.raw.data(), L < 64 ? L : 64);
  return e.st;
}

// OutputTokens: []*token.Token, each {"Owner": []byte, "Data": *math.G1}
std::string dec_outputs(const JDoc& d, int64_t node, ActionOut& o, std::vector<uint8_t>& pool) {
  o.data.clear();
  o.nil_token = false;
  if (node < 0 || d.at((uint32_t)node).type == J_NULL) return "";
  if (d.at((uint32_t)node).type != J_ARR) return "cannot unmarshal into []*token.Token";
  uint32_t cnt = d.len((uint32_t)node);
  std::vector<uint8_t> tmp;
  for (uint32_t k = 0; k < cnt; k++) {
    uint32_t t = d.elem((uint32_t)node, k);
    ElemRef r{D_NIL, 0, 0};
    if (d.at(t).type == J_NULL) {
      o.nil_token = true;
    } else {
      if (d.at(t).type != J_OBJ) return "cannot unmarshal into token.Token";
      if (dec_bytes(d, d.field(t, "Owner"), tmp) == D_ERR) return "bad Owner";
      if (dec_g1(d, d.field(t, "Data"), r, pool) == D_ERR) return "bad Data";
      if (r.st == D_OK && r.bad) return "bad Data";
    }
    o.data.push_back(r);
  }
  return "";
}

// Metadata map[string][]byte: an object of base64 strings (or null)
std::string check_metadata(const JDoc& d, int64_t node) {
  if (node < 0 || d.at((uint32_t)node).type == J_NULL) return "";
  if (d.at((uint32_t)node).type != J_OBJ) return "cannot unmarshal into map[string][]byte";
  const JNode& o = d.at((uint32_t)node);
  std::vector<uint8_t> tmp;
  for (uint32_t k = 0; k < o.count; k++)
    if (dec_bytes(d, d.kids[o.first + 2 * k + 1], tmp) == D_ERR) return "bad Metadata value";
  return "";
}

// JSON null at the top level leaves the struct untouched (Go Unmarshal into a
// pointer to a struct); anything else but an object is a type error
bool top_object(JDoc& d, const uint8_t* p, size_t n, std::string& err, bool& is_null,
                const JField* schema = nullptr) {
  is_null = false;
  if (!d.parse(p, n)) {
    err = "invalid JSON";
    return false;
  }
  if (schema) go_merge(d, schema);
  JType t = d.at(d.root()).type;
  if (t == J_NULL) {
    is_null = true;
    return true;
  }
  if (t != J_OBJ) {
    err = "cannot unmarshal into struct";
    return false;
  }
  return true;
}

thread_local JDoc tl_doc;

// []*token.Token fields: duplicate keys merge into the tokens already decoded
// (go_merge; transfer.go / issue.go action structs)
const JField TOKEN_F[] = {{nullptr, JF_STRUCT, nullptr}};
const JField TRANSFER_F[] = {{"OutputTokens", JF_SLICE, TOKEN_F}, {nullptr, JF_STRUCT, nullptr}};
const JField ISSUE_F[] = {{"outputs", JF_SLICE, TOKEN_F}, {nullptr, JF_STRUCT, nullptr}};

}  // namespace

std::string dec_transfer_action(const uint8_t* p, size_t n, TransferAct& a, std::vector<uint8_t>& pool) {
  a = TransferAct();
  std::string err;
  bool is_null;
  JDoc& d = tl_doc;
  if (!top_object(d, p, n, err, is_null, TRANSFER_F)) return err;
  if (is_null) return "";
  uint32_t root = d.root();
  // Inputs []string
  int64_t in = d.field(root, "Inputs");
  if (in >= 0 && d.at((uint32_t)in).type != J_NULL) {
    if (d.at((uint32_t)in).type != J_ARR) return "cannot unmarshal into []string";
    for (uint32_t k = 0; k < d.len((uint32_t)in); k++) {
      std::string s;
      if (dec_string(d, d.elem((uint32_t)in, k), s) == D_ERR) return "cannot unmarshal into string";
      a.inputs.push_back(s);
    }
  }
  // InputCommitments []*math.G1: decoded (and checked) but not used by the verifier
  int64_t ic = d.field(root, "InputCommitments");
  if (ic >= 0 && d.at((uint32_t)ic).type != J_NULL) {
    if (d.at((uint32_t)ic).type != J_ARR) return "cannot unmarshal into []*math.G1";
    for (uint32_t k = 0; k < d.len((uint32_t)ic); k++) {
      ElemRef r;
      if (dec_g1(d, d.elem((uint32_t)ic, k), r, pool) == D_ERR) return "bad InputCommitments element";
      if (r.st == D_OK && r.bad) return "bad InputCommitments element";
      a.in_coms.push_back(r);
    }
  }
  err = dec_outputs(d, d.field(root, "OutputTokens"), a.out, pool);
  if (!err.empty()) return err;
  DecStatus ps = dec_bytes(d, d.field(root, "Proof"), a.proof);
  if (ps == D_ERR) return "bad Proof";
  a.proof_nil = ps == D_NIL;
  return check_metadata(d, d.field(root, "Metadata"));
}

std::string dec_issue_action(const uint8_t* p, size_t n, IssueAct& a, std::vector<uint8_t>& pool) {
  a = IssueAct();
  std::string err;
  bool is_null;
  JDoc& d = tl_doc;
  if (!top_object(d, p, n, err, is_null, ISSUE_F)) return err;
  if (is_null) return "";
  uint32_t root = d.root();
  std::vector<uint8_t> tmp;
  if (dec_bytes(d, d.field(root, "Issuer"), tmp) == D_ERR) return "bad Issuer";
  // OutputTokens carries the tag json:"outputs,omitempty" (issue.go:24)
  err = dec_outputs(d, d.field(root, "outputs"), a.out, pool);
  if (!err.empty()) return err;
  if (dec_bytes(d, d.field(root, "Proof"), a.proof) == D_ERR) return "bad Proof";
  if (dec_bool(d, d.field(root, "Anonymous"), a.anonymous) == D_ERR) return "bad Anonymous";
  return check_metadata(d, d.field(root, "Metadata"));
}

std::string dec_token(const uint8_t* p, size_t n, ElemRef& data, std::vector<uint8_t>& pool) {
  data = ElemRef{D_NIL, 0, 0};
  std::string err;
  bool is_null;
  JDoc& d = tl_doc;
  if (!top_object(d, p, n, err, is_null)) return err;
  if (is_null) return "";
  uint32_t root = d.root();
  std::vector<uint8_t> tmp;
  if (dec_bytes(d, d.field(root, "Owner"), tmp) == D_ERR) return "bad Owner";
  if (dec_g1(d, d.field(root, "Data"), data, pool) == D_ERR) return "bad Data";
  if (data.st == D_OK && data.bad) return "bad Data";
  return "";
}

}  // namespace ftsh

// ---------------------------------------------------------------- validation
namespace ftsh {

namespace {

struct ReqState {
  bool failed = false;  // request-level failure (decode): code set
  int32_t code = FTZ_OK;
  std::vector<IssueAct> is;
  std::vector<TransferAct> tr;
  std::vector<uint8_t> pool;               // element slots of the actions (64 B each)
  std::vector<std::vector<ElemRef>> ins;   // per transfer: ledger input Data elements
  std::vector<int32_t> tr_pre;             // per transfer: code decided before the ZK check (0 = none)
  std::vector<int32_t> is_pre;
};

// element slots a request's unmarshal decodes (ActionOut data, InputCommitments)
template <class F>
void for_unmarshal_elems(const ReqState& s, F f) {
  for (const IssueAct& a : s.is)
    for (const ElemRef& e : a.out.data) f(e);
  for (const TransferAct& a : s.tr) {
    for (const ElemRef& e : a.in_coms) f(e);
    for (const ElemRef& e : a.out.data) f(e);
  }
}

}  // namespace

int verify_token_requests(size_t n, const ftz_bytes* reqs, const RequestHooks& h, int32_t* codes, int32_t* failed,
                          std::string& err) {
  std::vector<ReqState> st(n);
  // 1. decode: ASN.1, then every issue action, then every transfer action
  //    (validator.go unmarshalIssueActions / unmarshalTransferActions)
  for (size_t r = 0; r < n; r++) {
    ReqState& s = st[r];
    std::vector<Slice> f[4];
    std::string e = der_token_request(reqs[r].p, reqs[r].len, f);
    if (e.empty()) {
      s.is.resize(f[0].size());
      for (size_t k = 0; k < f[0].size() && e.empty(); k++) e = dec_issue_action(f[0][k].p, f[0][k].len, s.is[k], s.pool);
      s.tr.resize(f[1].size());
      for (size_t k = 0; k < f[1].size() && e.empty(); k++)
        e = dec_transfer_action(f[1][k].p, f[1][k].len, s.tr[k], s.pool);
    }
    if (!e.empty()) {
      s.failed = true;
      s.code = FTZ_ERR_PARSE;
    }
  }
  // 2. curve checks of the elements decoded at unmarshal (math.G1 UnmarshalJSON
  //    -> gnark SetBytes), one device pass over every request
  {
    std::vector<uint8_t> slots;
    std::vector<std::pair<size_t, size_t>> who;  // (request, slot offset)
    for (size_t r = 0; r < n; r++) {
      if (st[r].failed) continue;
      for_unmarshal_elems(st[r], [&](const ElemRef& e) {
        if (e.st != D_OK) return;
        slots.insert(slots.end(), st[r].pool.begin() + e.off, st[r].pool.begin() + e.off + 64);
        who.push_back({r, e.off});
      });
    }
    if (!who.empty()) {
      std::vector<uint8_t> ok(who.size());
      int rc = h.check(who.size(), slots.data(), ok.data());
      if (rc != FTZ_SUCCESS) {
        err = "element check failed";
        return rc;
      }
      for (size_t k = 0; k < who.size(); k++)
        if (!ok[k]) {
          st[who[k].first].failed = true;
          st[who[k].first].code = FTZ_ERR_PARSE;
        }
    }
  }
  // 3. ledger inputs of every transfer (TransferSignatureValidate's loads,
  //    validator_transfer.go:42-81), then their Data elements' curve checks
  std::vector<uint8_t> lslots;
  std::vector<std::pair<size_t, size_t>> lwho;  // (request, transfer)
  for (size_t r = 0; r < n; r++) {
    ReqState& s = st[r];
    if (s.failed) continue;
    s.ins.resize(s.tr.size());
    s.tr_pre.assign(s.tr.size(), 0);
    s.is_pre.assign(s.is.size(), 0);
    for (size_t t = 0; t < s.tr.size(); t++) {
      for (const std::string& key : s.tr[t].inputs) {
        const uint8_t* val = nullptr;
        size_t vlen = 0;
        if (!h.get_state || h.get_state(h.user, key.data(), key.size(), &val, &vlen) != 0 || vlen == 0) {
          s.tr_pre[t] = FTZ_ERR_INPUT;  // "failed to retrieve input" / "does not exists"
          break;
        }
        ElemRef d;
        if (!dec_token(val, vlen, d, s.pool).empty()) {
          s.tr_pre[t] = FTZ_ERR_INPUT;  // "failed to deserialize input to spend"
          break;
        }
        s.ins[t].push_back(d);
      }
      if (s.tr_pre[t]) continue;
      for (const ElemRef& d : s.ins[t])
        if (d.st == D_OK) {
          lslots.insert(lslots.end(), s.pool.begin() + d.off, s.pool.begin() + d.off + 64);
          lwho.push_back({r, t});
        }
    }
  }
  if (!lwho.empty()) {
    std::vector<uint8_t> ok(lwho.size());
    int rc = h.check(lwho.size(), lslots.data(), ok.data());
    if (rc != FTZ_SUCCESS) {
      err = "element check failed";
      return rc;
    }
    for (size_t k = 0; k < lwho.size(); k++)
      if (!ok[k]) st[lwho[k].first].tr_pre[lwho[k].second] = FTZ_ERR_INPUT;
  }
  // 4. the ZK checks of every action still open, in shared device batches.
  //    A nil or foreign-curve commitment reaches the verifier and the reference
  //    panics on it (G1 use / driver type assertion); a nil issue output fails
  //    GetCommitments ("failed to verify issue", validator.go verifyIssue).
  std::vector<uint8_t> coms;  // contiguous 64-byte commitments per action
  struct TRef { size_t r, t, in_off, out_off; };
  struct IRef { size_t r, k, out_off; };
  std::vector<TRef> trefs;
  std::vector<IRef> irefs;
  auto put = [&](const ReqState& s, const ElemRef& e) {
    size_t o = coms.size();
    coms.resize(o + 64, 0);
    memcpy(coms.data() + o, s.pool.data() + e.off, 64);
  };
  for (size_t r = 0; r < n; r++) {
    ReqState& s = st[r];
    if (s.failed) continue;
    for (size_t k = 0; k < s.is.size(); k++) {
      const IssueAct& a = s.is[k];
      if (a.out.nil_token) {
        s.is_pre[k] = FTZ_ERR_MALFORMED;
        continue;
      }
      bool bad = false;
      for (const ElemRef& e : a.out.data) bad |= e.st != D_OK;
      if (bad) {
        s.is_pre[k] = FTZ_ERR_PANIC;
        continue;
      }
      size_t o = coms.size();
      for (const ElemRef& e : a.out.data) put(s, e);
      irefs.push_back({r, k, o});
    }
    for (size_t t = 0; t < s.tr.size(); t++) {
      if (s.tr_pre[t]) continue;
      const TransferAct& a = s.tr[t];
      bool bad = a.out.nil_token;
      for (const ElemRef& e : a.out.data) bad |= e.st != D_OK;
      for (const ElemRef& e : s.ins[t]) bad |= e.st != D_OK;
      if (bad) {
        s.tr_pre[t] = FTZ_ERR_PANIC;
        continue;
      }
      size_t io = coms.size();
      for (const ElemRef& e : s.ins[t]) put(s, e);
      size_t oo = coms.size();
      for (const ElemRef& e : a.out.data) put(s, e);
      trefs.push_back({r, t, io, oo});
    }
  }
  std::vector<ftz_issue> iv(irefs.size());
  for (size_t k = 0; k < irefs.size(); k++) {
    const IssueAct& a = st[irefs[k].r].is[irefs[k].k];
    iv[k] = ftz_issue{coms.data() + irefs[k].out_off, (uint32_t)a.out.data.size(), a.proof.data(), a.proof.size(),
                      (uint8_t)(a.anonymous ? 1 : 0)};
  }
  std::vector<ftz_transfer> tv(trefs.size());
  for (size_t k = 0; k < trefs.size(); k++) {
    const ReqState& s = st[trefs[k].r];
    const TransferAct& a = s.tr[trefs[k].t];
    tv[k] = ftz_transfer{coms.data() + trefs[k].in_off, (uint32_t)s.ins[trefs[k].t].size(),
                         coms.data() + trefs[k].out_off, (uint32_t)a.out.data.size(), a.proof.data(), a.proof.size()};
  }
  std::vector<int32_t> icodes(iv.size()), tcodes(tv.size());
  // issues on a helper thread while the transfers go in from this one: the job
  // engine coalesces both into the same device batches
  int irc = FTZ_SUCCESS, trc = FTZ_SUCCESS;
  std::thread ith;
  if (!iv.empty()) {
    if (tv.empty())
      irc = h.verify_issues(iv.size(), iv.data(), icodes.data());
    else
      ith = std::thread([&] { irc = h.verify_issues(iv.size(), iv.data(), icodes.data()); });
  }
  if (!tv.empty()) trc = h.verify_transfers(tv.size(), tv.data(), tcodes.data());
  if (ith.joinable()) ith.join();
  if (irc != FTZ_SUCCESS || trc != FTZ_SUCCESS) {
    err = irc != FTZ_SUCCESS ? "issue verification failed" : "transfer verification failed";
    return irc != FTZ_SUCCESS ? irc : trc;
  }
  for (size_t k = 0; k < irefs.size(); k++) st[irefs[k].r].is_pre[irefs[k].k] = icodes[k];
  for (size_t k = 0; k < trefs.size(); k++) st[trefs[k].r].tr_pre[trefs[k].t] = tcodes[k];
  // 5. first failure in the reference's order: issues, then transfers
  for (size_t r = 0; r < n; r++) {
    const ReqState& s = st[r];
    int32_t code = s.failed ? s.code : FTZ_OK, at = -1;
    if (!s.failed) {
      for (size_t k = 0; k < s.is.size() && code == FTZ_OK; k++)
        if (s.is_pre[k]) code = s.is_pre[k], at = (int32_t)k;
      for (size_t t = 0; t < s.tr.size() && code == FTZ_OK; t++)
        if (s.tr_pre[t]) code = s.tr_pre[t], at = (int32_t)(s.is.size() + t);
    }
    codes[r] = code;
    if (failed) failed[r] = at;
  }
  return FTZ_SUCCESS;
}

}  // namespace ftsh

// Host decoding of raw token requests (request.h).
#include "request.h"

#include <string.h>

#include <algorithm>
#include <chrono>
#include <deque>
#include <memory>
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

// header at off: identifier byte must be `want`; on success (nullptr) body =
// [off, off+len), else the reason
const char* der_header(const Der& d, size_t& off, uint8_t want, size_t& len) {
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
  return nullptr;
}

// SEQUENCE OF OCTET STRING at off (advances off past it)
const char* der_seq_of_octets(const Der& d, size_t& off, std::vector<Slice>& out) {
  size_t len;
  const char* e = der_header(d, off, 0x30, len);
  if (e) return e;
  Der inner{d.b + off, len};
  size_t k = 0;
  out.clear();
  while (k < inner.n) {
    size_t el;
    e = der_header(inner, k, 0x04, el);
    if (e) return strcmp(e, "tags don't match") == 0 ? "sequence tag mismatch" : e;
    out.push_back(Slice{inner.b + k, el});
    k += el;
  }
  off += len;
  return nullptr;
}

}  // namespace

std::string der_token_request(const uint8_t* raw, size_t len, std::vector<Slice> out[4]) {
  for (int f = 0; f < 4; f++) out[f].clear();
  if (len == 0) return "empty token request";
  Der d{raw, len};
  size_t off = 0, body;
  const char* e = der_header(d, off, 0x30, body);
  if (e) return std::string("failed to unmarshal token request: ") + e;
  Der inner{raw + off, body};
  size_t k = 0;
  for (int f = 0; f < 4; f++) {
    e = der_seq_of_octets(inner, k, out[f]);
    if (e) return std::string("failed to unmarshal token request: ") + e;
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
  const size_t off = pool.size();
  const DecStatus st = dec_elem_append(d, node, pool);  // the bytes land at off
  r.st = st;
  r.bad = 0;
  r.off = 0;
  if (st != D_OK && st != D_PANIC) return st;
  size_t L = pool.size() - off;
  uint8_t m = L ? (pool[off] & 0xC0) : 0;
  if (L < 32 || (m == 0x00 && L < 64)) r.bad = 1;
  r.off = off;
  pool.resize(off + 64, 0);  // the slot: the first 64 bytes, zero-padded
  return st;
}

// OutputTokens: []*token.Token, each {"Owner": []byte, "Data": *math.G1}
std::string dec_outputs(const JDoc& d, int64_t node, ActionOut& o, std::vector<uint8_t>& pool) {
  o.data.clear();
  o.nil_token = false;
  if (node < 0 || d.at((uint32_t)node).type == J_NULL) return "";
  if (d.at((uint32_t)node).type != J_ARR) return "cannot unmarshal into []*token.Token";
  uint32_t cnt = d.len((uint32_t)node);
  static thread_local std::vector<uint8_t> tmp;  // Owner: checked, not kept
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
  static thread_local std::vector<uint8_t> tmp;
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
  static thread_local std::vector<uint8_t> tmp;
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
  static thread_local std::vector<uint8_t> tmp;
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

namespace {

struct TRef {
  size_t r, t, in_off, out_off;
};
struct IRef {
  size_t r, k, out_off;
};

// One pipeline step: requests [r0, r1) from decode to the engine's verdicts.
struct Chunk {
  size_t r0 = 0, r1 = 0;
  std::vector<ReqState> st;
  std::vector<uint8_t> coms;  // contiguous 64-byte commitments per action
  std::vector<TRef> trefs;
  std::vector<IRef> irefs;
  std::vector<ftz_transfer> tv;
  std::vector<ftz_issue> iv;
  std::vector<int32_t> tcodes, icodes;
  int trc = FTZ_SUCCESS, irc = FTZ_SUCCESS;
  std::thread th_t, th_i;
  void join() {
    if (th_t.joinable()) th_t.join();
    if (th_i.joinable()) th_i.join();
  }
};

// accumulates the calling thread's time since the last mark into one stage
struct StageClock {
  RequestStats* st;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void mark(double RequestStats::*field) {
    auto now = std::chrono::steady_clock::now();
    if (st) st->*field += std::chrono::duration<double, std::milli>(now - t).count();
    t = now;
  }
};

void run_par(const RequestHooks& h, size_t k, const std::function<void(size_t)>& f) {
  if (h.par && k > 1) {
    h.par(k, f);
  } else {
    for (size_t i = 0; i < k; i++) f(i);
  }
}

// exclusive prefix sums in place: v[0] = 0, v[i + 1] = v[i] + (count of item i)
void prefix(std::vector<size_t>& v) {
  v[0] = 0;
  for (size_t i = 1; i < v.size(); i++) v[i] += v[i - 1];
}

// Steps 1-4 of a chunk and the start of its ZK verification: decode_chunk
// (steps 1-2, decoding and the unmarshal checks), then ledger_chunk (the
// ledger callbacks on the calling thread, token decoding, checks, the
// verification hand-off).  Every per-request stage runs on h.par (a request's
// state is written by one thread).  Decoding chunk k+1 on a thread of its own
// beside chunk k's ledger phase measured the same (674k against 675k
// transfers/s, six alternating runs, profiles/r06/req_decode.txt): the leg is
// bound by the device work and the planning threads, not the calling thread.
void par_each(const RequestHooks& h, size_t m, const std::function<void(size_t)>& f) {
  constexpr size_t PIECE = 32;
  run_par(h, (m + PIECE - 1) / PIECE, [&](size_t p) {
    for (size_t r = p * PIECE; r < m && r < (p + 1) * PIECE; r++) f(r);
  });
}

int decode_chunk(const ftz_bytes* reqs, const RequestHooks& h, Chunk& c, RequestStats* stats, std::string& err) {
  const size_t m = c.r1 - c.r0;
  StageClock clk{stats};
  c.st.resize(m);
  auto each = [&](const std::function<void(size_t)>& f) { par_each(h, m, f); };
  std::vector<size_t> cnt(m + 1, 0);
  // 1. decode: ASN.1, then every issue action, then every transfer action
  //    (validator.go unmarshalIssueActions / unmarshalTransferActions);
  //    cnt = the request's elements decoded at unmarshal
  each([&](size_t i) {
    ReqState& s = c.st[i];
    const ftz_bytes& q = reqs[c.r0 + i];
    static thread_local std::vector<Slice> f[4];  // cleared by der_token_request
    std::string e = der_token_request(q.p, q.len, f);
    if (e.empty()) {
      s.is.resize(f[0].size());
      for (size_t k = 0; k < f[0].size() && e.empty(); k++) e = dec_issue_action(f[0][k].p, f[0][k].len, s.is[k], s.pool);
      s.tr.resize(f[1].size());
      for (size_t k = 0; k < f[1].size() && e.empty(); k++) e = dec_transfer_action(f[1][k].p, f[1][k].len, s.tr[k], s.pool);
    }
    if (!e.empty()) {
      s.failed = true;
      s.code = FTZ_ERR_PARSE;
      return;
    }
    size_t k = 0;
    for_unmarshal_elems(s, [&](const ElemRef& x) { k += x.st == D_OK; });
    cnt[i + 1] = k;
  });
  clk.mark(&RequestStats::decode);
  // 2. curve checks of the elements decoded at unmarshal (math.G1 UnmarshalJSON
  //    -> gnark SetBytes), one device pass over the chunk
  prefix(cnt);
  if (cnt[m]) {
    std::vector<uint8_t> slots(64 * cnt[m]), ok(cnt[m]);
    each([&](size_t r) {
      size_t o = cnt[r];
      if (c.st[r].failed) return;  // a request that failed to decode counted none
      for_unmarshal_elems(c.st[r], [&](const ElemRef& x) {
        if (x.st == D_OK) memcpy(slots.data() + 64 * o++, c.st[r].pool.data() + x.off, 64);
      });
    });
    int rc = h.check(cnt[m], slots.data(), ok.data());
    if (rc != FTZ_SUCCESS) {
      err = "element check failed";
      return rc;
    }
    each([&](size_t r) {
      for (size_t k = cnt[r]; k < cnt[r + 1]; k++)
        if (!ok[k]) {
          c.st[r].failed = true;
          c.st[r].code = FTZ_ERR_PARSE;
        }
    });
  }
  clk.mark(&RequestStats::check);
  return FTZ_SUCCESS;
}

int ledger_chunk(const RequestHooks& h, Chunk& c, std::string& err) {
  const size_t m = c.r1 - c.r0;
  StageClock clk{h.stats};
  auto each = [&](const std::function<void(size_t)>& f) { par_each(h, m, f); };
  std::vector<size_t> cnt(m + 1, 0);
  // 3. ledger inputs of every transfer (TransferSignatureValidate's loads,
  //    validator_transfer.go:42-81) through the callbacks on the calling thread
  std::vector<size_t> kat(m + 1, 0);  // the request's first key index
  each([&](size_t r) {
    ReqState& s = c.st[r];
    if (s.failed) return;
    s.ins.resize(s.tr.size());
    s.tr_pre.assign(s.tr.size(), 0);
    s.is_pre.assign(s.is.size(), 0);
    size_t k = 0;
    for (const TransferAct& t : s.tr) k += t.inputs.size();
    kat[r + 1] = k;
  });
  prefix(kat);
  std::vector<ftz_bytes> keys(kat[m]);
  each([&](size_t r) {
    size_t k = kat[r];
    if (c.st[r].failed) return;
    for (const TransferAct& t : c.st[r].tr)
      for (const std::string& key : t.inputs) keys[k++] = ftz_bytes{reinterpret_cast<const uint8_t*>(key.data()), key.size()};
  });
  std::vector<ftz_bytes> vals(keys.size(), ftz_bytes{nullptr, 0});  // {NULL, 0}: missing / not read
  std::vector<uint8_t> vbuf;  // the one-key form's values, copied (each is valid until the next call)
  if (!keys.empty()) {
    if (h.get_states) {
      // values valid until the next get_states call: the tokens are decoded below, before it
      if (h.get_states(h.user, keys.size(), keys.data(), vals.data()) != 0)
        for (ftz_bytes& v : vals) v = ftz_bytes{nullptr, 0};
    } else {
      std::vector<std::pair<size_t, size_t>> at(keys.size(), {0, 0});
      for (size_t r = 0; r < m; r++) {
        const ReqState& s = c.st[r];
        if (s.failed) continue;
        size_t k = kat[r];
        for (const TransferAct& t : s.tr) {
          size_t k1 = k + t.inputs.size();
          for (; k < k1; k++) {
            const uint8_t* val = nullptr;
            size_t vlen = 0;
            if (!h.get_state ||
                h.get_state(h.user, reinterpret_cast<const char*>(keys[k].p), keys[k].len, &val, &vlen) != 0 ||
                vlen == 0)
              break;  // "failed to retrieve input" / "does not exists": the transfer's later inputs are not read
            at[k] = {vbuf.size(), vlen};
            vbuf.insert(vbuf.end(), val, val + vlen);
          }
          k = k1;
        }
      }
      for (size_t k = 0; k < keys.size(); k++)
        if (at[k].second) vals[k] = ftz_bytes{vbuf.data() + at[k].first, at[k].second};
    }
  }
  clk.mark(&RequestStats::lookup);
  // token decoding per request; cnt = the request's ledger Data elements to check
  std::fill(cnt.begin(), cnt.end(), 0);
  each([&](size_t r) {
    ReqState& s = c.st[r];
    if (s.failed) return;
    size_t k = kat[r], nd = 0;
    for (size_t t = 0; t < s.tr.size(); t++) {
      size_t k1 = k + s.tr[t].inputs.size();
      for (; k < k1; k++) {
        if (!vals[k].p || !vals[k].len) {
          s.tr_pre[t] = FTZ_ERR_INPUT;  // "failed to retrieve input" / "does not exists"
          break;
        }
        ElemRef d;
        if (!dec_token(vals[k].p, vals[k].len, d, s.pool).empty()) {
          s.tr_pre[t] = FTZ_ERR_INPUT;  // "failed to deserialize input to spend"
          break;
        }
        s.ins[t].push_back(d);
      }
      k = k1;
      if (!s.tr_pre[t])
        for (const ElemRef& d : s.ins[t]) nd += d.st == D_OK;
    }
    cnt[r + 1] = nd;
  });
  clk.mark(&RequestStats::tokens);
  prefix(cnt);
  if (cnt[m]) {
    std::vector<uint8_t> slots(64 * cnt[m]), ok(cnt[m]);
    std::vector<uint32_t> tr_of(cnt[m]);
    each([&](size_t r) {
      const ReqState& s = c.st[r];
      size_t o = cnt[r];
      if (s.failed) return;
      for (size_t t = 0; t < s.tr.size(); t++) {
        if (s.tr_pre[t]) continue;
        for (const ElemRef& d : s.ins[t])
          if (d.st == D_OK) {
            memcpy(slots.data() + 64 * o, s.pool.data() + d.off, 64);
            tr_of[o++] = (uint32_t)t;
          }
      }
    });
    int rc = h.check(cnt[m], slots.data(), ok.data());
    if (rc != FTZ_SUCCESS) {
      err = "element check failed";
      return rc;
    }
    each([&](size_t r) {
      for (size_t k = cnt[r]; k < cnt[r + 1]; k++)
        if (!ok[k]) c.st[r].tr_pre[tr_of[k]] = FTZ_ERR_INPUT;
    });
  }
  clk.mark(&RequestStats::check);
  // 4. the ZK checks of every action still open, through the job engine.
  //    A nil or foreign-curve commitment reaches the verifier and the reference
  //    panics on it (G1 use / driver type assertion); a nil issue output fails
  //    GetCommitments ("failed to verify issue", validator.go verifyIssue).
  //    Per request: the pre-verifier codes and the counts, then prefix sums,
  //    then every request fills its commitments / jobs in place.
  std::vector<size_t> ncom(m + 1, 0), nis(m + 1, 0), ntr(m + 1, 0);
  each([&](size_t r) {
    ReqState& s = c.st[r];
    if (s.failed) return;
    size_t nc = 0, ni = 0, nt = 0;
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
      nc += a.out.data.size();
      ni++;
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
      nc += s.ins[t].size() + a.out.data.size();
      nt++;
    }
    ncom[r + 1] = nc;
    nis[r + 1] = ni;
    ntr[r + 1] = nt;
  });
  prefix(ncom);
  prefix(nis);
  prefix(ntr);
  c.coms.resize(64 * ncom[m]);
  c.irefs.resize(nis[m]);
  c.trefs.resize(ntr[m]);
  c.iv.resize(nis[m]);
  c.tv.resize(ntr[m]);
  each([&](size_t r) {
    const ReqState& s = c.st[r];
    if (s.failed) return;
    size_t o = 64 * ncom[r], ki = nis[r], kt = ntr[r];
    auto put = [&](const ElemRef& e) {
      memcpy(c.coms.data() + o, s.pool.data() + e.off, 64);
      o += 64;
    };
    for (size_t k = 0; k < s.is.size(); k++) {
      if (s.is_pre[k]) continue;
      const IssueAct& a = s.is[k];
      size_t oo = o;
      for (const ElemRef& e : a.out.data) put(e);
      c.irefs[ki] = {r, k, oo};
      c.iv[ki++] = ftz_issue{c.coms.data() + oo, (uint32_t)a.out.data.size(), a.proof.data(), a.proof.size(),
                             (uint8_t)(a.anonymous ? 1 : 0)};
    }
    for (size_t t = 0; t < s.tr.size(); t++) {
      if (s.tr_pre[t]) continue;
      const TransferAct& a = s.tr[t];
      size_t io = o;
      for (const ElemRef& e : s.ins[t]) put(e);
      size_t oo = o;
      for (const ElemRef& e : a.out.data) put(e);
      c.trefs[kt] = {r, t, io, oo};
      c.tv[kt++] = ftz_transfer{c.coms.data() + io, (uint32_t)s.ins[t].size(), c.coms.data() + oo,
                                (uint32_t)a.out.data.size(), a.proof.data(), a.proof.size()};
    }
  });
  c.icodes.resize(c.iv.size());
  c.tcodes.resize(c.tv.size());
  clk.mark(&RequestStats::build);
  // issues and transfers on helper threads: the job engine coalesces them (and
  // the other chunks in flight) into shared device batches
  Chunk* cp = &c;
  if (!c.iv.empty())
    c.th_i = std::thread([&h, cp] { cp->irc = h.verify_issues(cp->iv.size(), cp->iv.data(), cp->icodes.data()); });
  if (!c.tv.empty())
    c.th_t = std::thread([&h, cp] { cp->trc = h.verify_transfers(cp->tv.size(), cp->tv.data(), cp->tcodes.data()); });
  return FTZ_SUCCESS;
}

// 5. the chunk's verdicts: first failure in the reference's order, issues then transfers
int finish_chunk(Chunk& c, int32_t* codes, int32_t* failed, std::string& err) {
  c.join();
  if (c.irc != FTZ_SUCCESS || c.trc != FTZ_SUCCESS) {
    err = c.irc != FTZ_SUCCESS ? "issue verification failed" : "transfer verification failed";
    return c.irc != FTZ_SUCCESS ? c.irc : c.trc;
  }
  for (size_t k = 0; k < c.irefs.size(); k++) c.st[c.irefs[k].r].is_pre[c.irefs[k].k] = c.icodes[k];
  for (size_t k = 0; k < c.trefs.size(); k++) c.st[c.trefs[k].r].tr_pre[c.trefs[k].t] = c.tcodes[k];
  for (size_t i = 0; i < c.st.size(); i++) {
    const ReqState& s = c.st[i];
    int32_t code = s.failed ? s.code : FTZ_OK, at = -1;
    if (!s.failed) {
      for (size_t k = 0; k < s.is.size() && code == FTZ_OK; k++)
        if (s.is_pre[k]) code = s.is_pre[k], at = (int32_t)k;
      for (size_t t = 0; t < s.tr.size() && code == FTZ_OK; t++)
        if (s.tr_pre[t]) code = s.tr_pre[t], at = (int32_t)(s.is.size() + t);
    }
    codes[c.r0 + i] = code;
    if (failed) failed[c.r0 + i] = at;
  }
  return FTZ_SUCCESS;
}

}  // namespace

int verify_token_requests(size_t n, const ftz_bytes* reqs, const RequestHooks& h, int32_t* codes, int32_t* failed,
                          std::string& err) {
  const size_t CH = h.chunk ? h.chunk : 8192, IN = h.inflight ? h.inflight : 1;
  std::deque<std::unique_ptr<Chunk>> fly;
  int rc = FTZ_SUCCESS;
  // the first chunks are smaller (CH/8, CH/4, CH/2, then CH): the device gets
  // its first verification work after an eighth of a chunk's decoding
#ifndef FTS_REQ_RAMP
#define FTS_REQ_RAMP 8
#endif
  size_t ch = std::max<size_t>(CH / FTS_REQ_RAMP, 1), r0 = 0;
  auto make = [&]() {
    std::unique_ptr<Chunk> c(new Chunk());
    c->r0 = r0;
    c->r1 = std::min(n, r0 + ch);
    r0 = c->r1;
    ch = std::min(CH, 2 * ch);
    return c;
  };
  for (; r0 < n && rc == FTZ_SUCCESS;) {
    StageClock clk{h.stats};
    while (fly.size() >= IN) {  // bound the memory held by chunks in flight
      rc = finish_chunk(*fly.front(), codes, failed, err);
      fly.pop_front();
      if (rc != FTZ_SUCCESS) break;
    }
    clk.mark(&RequestStats::drain);
    if (rc != FTZ_SUCCESS) break;
    fly.push_back(make());
    rc = decode_chunk(reqs, h, *fly.back(), h.stats, err);
    if (rc == FTZ_SUCCESS) rc = ledger_chunk(h, *fly.back(), err);
  }
  // drain (also after an error: every helper thread is joined before returning)
  StageClock clk{h.stats};
  while (!fly.empty()) {
    std::string e2;
    int r2 = finish_chunk(*fly.front(), codes, failed, e2);
    if (rc == FTZ_SUCCESS && r2 != FTZ_SUCCESS) {
      rc = r2;
      err = e2;
    }
    fly.pop_front();
  }
  clk.mark(&RequestStats::drain);
  return rc;
}

}  // namespace ftsh

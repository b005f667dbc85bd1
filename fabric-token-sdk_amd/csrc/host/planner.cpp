// Host planner: restates the *control flow* of the reference verifiers (which
// checks run, in which order, and which error class each failure produces) and
// compiles the arithmetic into GPU jobs.  Reference (paths under
// token/core/zkatdlog/crypto/):
//   transfer.Verifier.Verify             transfer/transfer.go:124-154
//   WellFormednessVerifier.Verify        transfer/wellformedness.go:157-240
//   rangeproof.Verifier.Verify           range/proof.go:211-284, 393-444
//   MembershipVerifier.Verify            sigproof/membership.go:162-180, 260-305
//   POKVerifier.recomputeCommitment      sigproof/pok.go:160-204
//   issue.Verifier.Verify                issue/issue.go:202-223
//   issue WellFormednessVerifier.Verify  issue/wellformedness.go:206-265
// No group, field or hash arithmetic happens here: every value is produced on
// the GPU.  The planner only parses bytes (JSON, base64) and lays out jobs.
#include "planner.h"

#include <math.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <type_traits>

#include "gojson.h"

namespace ftsh {

// struct-pointer / slice-of-struct-pointer fields, whose duplicate keys merge
// (go_merge): range/proof.go:25-57 RangeProof -> EqualityProofs,
// MembershipProof -> sigproof/membership.go:19-33 MembershipProof ->
// pssign.Signature; setup.go:25-54 PublicParams -> RangeProofParams ->
// SignedValues []*pssign.Signature
static const JField LEAVES_F[] = {{nullptr, JF_STRUCT, nullptr}};
static const JField SIGPROOF_F[] = {{"Signature", JF_STRUCT, LEAVES_F}, {nullptr, JF_STRUCT, nullptr}};
static const JField MP_F[] = {{"SignatureProofs", JF_SLICE, SIGPROOF_F}, {nullptr, JF_STRUCT, nullptr}};
static const JField RANGE_F[] = {{"EqualityProofs", JF_STRUCT, LEAVES_F},
                                 {"MembershipProofs", JF_SLICE, MP_F},
                                 {nullptr, JF_STRUCT, nullptr}};
static const JField RPP_F[] = {{"SignedValues", JF_SLICE, LEAVES_F}, {nullptr, JF_STRUCT, nullptr}};
static const JField PP_F[] = {{"RangeProofParams", JF_STRUCT, RPP_F}, {nullptr, JF_STRUCT, nullptr}};

void Plan::clear() {
  rnd.clear();
  sc1.clear();
  sc_post.clear();
  emit.clear();
  b64.clear();
  cp.clear();
  cp2.clear();
  out.clear();
  out_off.clear();
  item_off.clear();
  dev_pools = false;
  arena_len = out_len = 0;
  wire.clear();
  arena.clear();
  dec.clear();
  zr.clear();
  sc.clear();
  sclist.clear();
  vt.clear();
  g1.clear();
  g1p.clear();
  g2.clear();
  pr.clear();
  seg.clear();
  hpre.clear();
  hmain.clear();
  ck.clear();
  tx.clear();
  n_pts = n_scal = n_g1out = n_g2out = 0;
}

namespace {

struct Ref {
  int64_t off = -1;  // offset into plan.wire (-1: nil pointer)
  uint32_t len = 0;
  bool nil() const { return off < 0; }
};

// Typed decoding of one JSON document with json.Unmarshal semantics:
// syntax errors are reported before any element is decoded; an element whose
// UnmarshalJSON would panic (foreign curve) marks `panic`; element / type
// errors mark `err` (the reference's Unmarshal returns the first error).
// The JDoc is borrowed from the builder so its buffers are reused.
struct Doc {
  JDoc& d;
  bool ok = false;
  bool panic = false;
  bool err = false;
  Plan* pl;

  Doc(Plan* p, JDoc& jd) : d(jd), pl(p) {}

  bool parse(const std::vector<uint8_t>& b, bool nil, const JField* schema = nullptr) {
    if (nil) return ok = false;  // json.Unmarshal(nil) -> "unexpected end of JSON input"
    ok = d.parse(b.data(), b.size());
    if (ok && schema) go_merge(d, schema);
    return ok;
  }

  Ref elem(int64_t node) {
    Ref r;
    if (node < 0 || d.at((uint32_t)node).type == J_NULL) return r;
    size_t off = 0;
    uint32_t len = 0;
    // element bytes land 16-byte aligned in the wire pool (device vector loads)
    DecStatus st = dec_elem_into(d, node, pl->wire, off, len);
    if (st == D_ERR) {
      err = true;
      return r;
    }
    if (st == D_PANIC) {
      panic = true;
      return r;
    }
    if (len > ZR_MAX_LEN) {  // beyond the device decoder's range
      pl->wire.resize(off);
      err = true;
      return r;
    }
    r.off = (int64_t)off;
    r.len = len;
    return r;
  }

  // []*Elem: null -> nil (empty), non-array -> error
  std::vector<Ref> list(int64_t node) {
    std::vector<Ref> out;
    if (node < 0 || d.at((uint32_t)node).type == J_NULL) return out;
    if (d.at((uint32_t)node).type != J_ARR) {
      err = true;
      return out;
    }
    uint32_t n = d.len((uint32_t)node);
    out.reserve(n);
    for (uint32_t k = 0; k < n; k++) out.push_back(elem(d.elem((uint32_t)node, k)));
    return out;
  }

  // struct-typed node: null/missing -> nil pointer (returns -1 and sets isnil),
  // non-object -> error
  int64_t obj(int64_t node, bool& isnil) {
    isnil = false;
    if (node < 0 || d.at((uint32_t)node).type == J_NULL) {
      isnil = true;
      return -1;
    }
    if (d.at((uint32_t)node).type != J_OBJ) {
      err = true;
      isnil = true;
      return -1;
    }
    return node;
  }

  int64_t f(int64_t obj, const char* name) { return obj < 0 ? -1 : d.field((uint32_t)obj, name); }

  // top-level value decoded into a struct: null -> zero struct, object -> ok,
  // anything else -> type error
  int64_t top() {
    uint32_t r = d.root();
    if (d.at(r).type == J_NULL) return -1;
    if (d.at(r).type != J_OBJ) {
      err = true;
      return -1;
    }
    return r;
  }
};

// Reader for the canonical json.Marshal bytes of the proof structs: fields in
// declaration order, no whitespace, elements as {"curve":1,"element":"<b64>"},
// pointers / slices null or present.  A document that matches this grammar
// exactly decodes to the same values under Go's rules as under the general
// path (Doc), which it skips: no DOM, element bytes decoded straight from the
// source into the wire pool.  Anything else -- whitespace, case-folded,
// duplicate or unknown keys, escapes, another curve id, bad base64 -- makes a
// reader call return false; the caller then rolls the wire pool back and
// re-parses the document with the general path, which owns every error.
struct Canon {
  const uint8_t* s;
  size_t n, i;
  Plan* pl;

  Canon(const uint8_t* p, size_t len, Plan* plan) : s(p), n(len), i(0), pl(plan) {}

  bool lit(const char* L, size_t len) {
    if (i + len > n || memcmp(s + i, L, len) != 0) return false;
    i += len;
    return true;
  }
  template <size_t N>
  bool lit(const char (&L)[N]) {
    return lit(L, N - 1);
  }
  bool at(char c) const { return i < n && s[i] == (uint8_t)c; }
  bool end() const { return i == n; }

  // string body up to the closing quote (validated by the strict base64
  // decoder, which rejects anything but the alphabet and final padding)
  bool b64span(size_t& a, size_t& b) {
    a = i;
    const void* q = memchr(s + i, '"', n - i);
    if (!q) return false;
    b = (size_t)((const uint8_t*)q - s);
    i = b + 1;
    return true;
  }

  // *Elem: null or {"curve":1,"element":"<b64>"}
  bool elem(Ref& r) {
    r = Ref();
    if (at('n')) return lit("null");
    if (!lit("{\"curve\":1,\"element\":\"")) return false;
    size_t a, b;
    if (!b64span(a, b)) return false;
    std::vector<uint8_t>& w = pl->wire;
    size_t off = (w.size() + 15) & ~(size_t)15;  // 16-byte aligned element (device vector loads)
    w.resize(off, 0);
    if (!b64_decode_strict_append((const char*)s + a, b - a, w) || w.size() - off > ZR_MAX_LEN) return false;
    r.off = (int64_t)off;
    r.len = (uint32_t)(w.size() - off);
    return lit("}");
  }

  // []*Elem: null or [E,...]
  bool list(std::vector<Ref>& out) {
    out.clear();
    if (at('n')) return lit("null");
    if (!lit("[")) return false;
    if (lit("]")) return true;
    while (true) {
      Ref r;
      if (!elem(r)) return false;
      out.push_back(r);
      if (lit(",")) continue;
      return lit("]");
    }
  }

  // []byte: null (nil) or "<b64>" decoded into out
  bool bytes(std::vector<uint8_t>& out, bool& nil) {
    out.clear();
    nil = at('n');
    if (nil) return lit("null");
    if (!lit("\"")) return false;
    size_t a, b;
    if (!b64span(a, b)) return false;
    return b64_decode_strict_append((const char*)s + a, b - a, out);
  }

  // string without escapes or non-ASCII bytes
  bool plain_string(std::string& out) {
    if (!lit("\"")) return false;
    size_t a = i;
    while (i < n && s[i] != '"') {
      if (s[i] == '\\' || s[i] < 0x20 || s[i] >= 0x80) return false;
      i++;
    }
    if (i >= n) return false;
    out.assign((const char*)s + a, i - a);
    i++;
    return true;
  }
};

struct Membership {
  bool nil = true;
  Ref chal, value, combf, sigbf, hash;
  bool sig_nil = true;
  Ref R, S, commitment;
};
struct MP {
  bool nil = true;
  std::vector<Ref> coms;
  std::vector<Membership> sps;
};
struct RangeDoc {
  Ref chal;
  bool eq_nil = true;
  Ref eq_type;
  std::vector<Ref> eq_val, eq_tbf, eq_cbf;
  std::vector<MP> mps;
};

class Builder {
 public:
  Builder(Plan& p, const PPInfo& pp) : pl(p), pp(pp) {}

  void transfer(const TransferIn& t);
  void issue(const IssueIn& t);
  void opening(const OpeningIn& o);

 private:
  Plan& pl;
  const PPInfo& pp;
  JDoc jtop, jwf, jrc;                 // parse buffers, reused across proofs
  std::vector<uint8_t> wfb, rcb;       // base64-decoded inner documents
  TxChecks tc;
  int part = 0;  // 0: WF part, 1: range part
  uint32_t ncheck[2];

  void check(uint8_t kind, uint8_t code, uint32_t a = 0, uint32_t b = 0) {
    Check c;
    c.kind = kind;
    c.code = code;
    c.pad = 0;
    c.a = a;
    c.b = b;
    pl.ck.push_back(c);
    ncheck[part]++;
  }
  void fail(uint8_t code) { check(CK_STATIC, code); }

  // 16-byte aligned (the device SHA-256 streams aligned whole blocks)
  uint32_t arena_alloc(uint32_t n) {
    uint32_t off = (uint32_t)((pl.arena.size() + 15) & ~(size_t)15);
    pl.arena.resize(off + n, 0);
    return off;
  }
  uint32_t scalar(const Ref& r) {
    ZrJob j;
    j.raw = (uint32_t)r.off;
    j.len = r.len;
    j.out = pl.n_scal++;
    pl.zr.push_back(j);
    return j.out;
  }
  uint32_t point(uint32_t raw, uint32_t len, uint32_t bytes, uint32_t b64) {
    DecodeJob j;
    j.raw = raw;
    j.len = len;
    j.out = pl.n_pts++;
    j.bytes = bytes;
    j.b64 = b64;
    pl.dec.push_back(j);
    return j.out;
  }
  uint32_t point(const Ref& r, uint32_t bytes = NONE, uint32_t b64 = NONE) {
    return point((uint32_t)r.off, r.len, bytes, b64);
  }
  uint32_t seg(uint32_t off, uint32_t len) {
    pl.seg.push_back({off, len});
    return (uint32_t)pl.seg.size() - 1;
  }
  uint32_t g1job(std::initializer_list<std::pair<uint8_t, uint32_t>> fixed, const std::vector<VTerm>& var,
                 uint32_t vscal, uint32_t bytes, bool feeds_pairing = false) {
    G1Job j;
    memset(&j, 0, sizeof(j));
    j.nfix = 0;
    for (auto& f : fixed) {
      j.fbase[j.nfix] = f.first;
      j.fscal[j.nfix] = f.second;
      j.nfix++;
    }
    j.vstart = (uint32_t)pl.vt.size();
    j.vcount = (uint32_t)var.size();
    pl.vt.insert(pl.vt.end(), var.begin(), var.end());
    j.vscal = vscal;
    j.vneg = 1;
    j.out = pl.n_g1out++;
    j.bytes = bytes;
    j.b64 = NONE;
    (feeds_pairing ? pl.g1p : pl.g1).push_back(j);
    return j.out;
  }
  // a verification transcript's HashToZr slot (debug_challenges plans only)
  uint32_t dbg_scal() { return pp.debug_challenges ? pl.n_scal++ : NONE; }
  static VTerm vterm(uint32_t pt, uint64_t w = 1) {
    VTerm v;
    v.pt = pt;
    v.w_lo = (uint32_t)w;
    v.w_hi = (uint32_t)(w >> 32);
    v.flags = 0;
    return v;
  }

  void begin_tx(uint8_t mode) {
    tc.wf_start = (uint32_t)pl.ck.size();
    ncheck[0] = ncheck[1] = 0;
    part = 0;
    tc.mode = mode;
  }
  void begin_range() {
    tc.wf_count = ncheck[0];
    tc.rg_start = (uint32_t)pl.ck.size();
    part = 1;
  }
  void end_tx() {
    if (part == 0) {
      tc.wf_count = ncheck[0];
      tc.rg_start = (uint32_t)pl.ck.size();
    }
    tc.rg_count = ncheck[1];
    pl.tx.push_back(tc);
  }

  uint32_t tokens(const uint8_t* p, uint32_t n, uint32_t& bytes_off);
  bool wf_side(uint32_t tok_pt, uint32_t n, const std::vector<Ref>& vals, const std::vector<Ref>& bfs,
               const Ref& type, const Ref& sum, const Ref& chal, uint32_t& s_type, uint32_t& s_sum,
               uint32_t& s_chal, uint32_t wfout_bytes);
  void range_part(const std::vector<uint8_t>& rc, bool rc_nil, uint32_t out_pt, uint32_t out_bytes, uint32_t n);
  static void decode_range(Doc& doc, RangeDoc& r);
  bool fast_range(const std::vector<uint8_t>& rc, RangeDoc& r);
};

// RangeProof (range/proof.go:25-57) in canonical form
bool Builder::fast_range(const std::vector<uint8_t>& rc, RangeDoc& r) {
  Canon c(rc.data(), rc.size(), &pl);
  if (!c.lit("{\"Challenge\":") || !c.elem(r.chal) || !c.lit(",\"EqualityProofs\":")) return false;
  r.eq_nil = c.at('n');
  if (r.eq_nil) {
    if (!c.lit("null")) return false;
  } else if (!c.lit("{\"Type\":") || !c.elem(r.eq_type) || !c.lit(",\"Value\":") || !c.list(r.eq_val) ||
             !c.lit(",\"TokenBlindingFactor\":") || !c.list(r.eq_tbf) || !c.lit(",\"CommitmentBlindingFactor\":") ||
             !c.list(r.eq_cbf) || !c.lit("}")) {
    return false;
  }
  if (!c.lit(",\"MembershipProofs\":")) return false;
  r.mps.clear();
  if (c.at('n')) {
    if (!c.lit("null")) return false;
  } else {
    if (!c.lit("[")) return false;
    if (!c.lit("]")) {
      while (true) {
        r.mps.emplace_back();
        MP& mp = r.mps.back();
        mp.nil = c.at('n');
        if (mp.nil) {
          if (!c.lit("null")) return false;
        } else {
          if (!c.lit("{\"Commitments\":") || !c.list(mp.coms) || !c.lit(",\"SignatureProofs\":")) return false;
          if (c.at('n')) {
            if (!c.lit("null")) return false;
          } else {
            if (!c.lit("[")) return false;
            if (!c.lit("]")) {
              while (true) {
                mp.sps.emplace_back();
                Membership& m = mp.sps.back();
                m.nil = c.at('n');
                if (m.nil) {
                  if (!c.lit("null")) return false;
                } else {
                  if (!c.lit("{\"Challenge\":") || !c.elem(m.chal) || !c.lit(",\"Signature\":")) return false;
                  m.sig_nil = c.at('n');
                  if (m.sig_nil) {
                    if (!c.lit("null")) return false;
                  } else if (!c.lit("{\"R\":") || !c.elem(m.R) || !c.lit(",\"S\":") || !c.elem(m.S) || !c.lit("}")) {
                    return false;
                  }
                  if (!c.lit(",\"Value\":") || !c.elem(m.value) || !c.lit(",\"ComBlindingFactor\":") ||
                      !c.elem(m.combf) || !c.lit(",\"SigBlindingFactor\":") || !c.elem(m.sigbf) ||
                      !c.lit(",\"Hash\":") || !c.elem(m.hash) || !c.lit(",\"Commitment\":") || !c.elem(m.commitment) ||
                      !c.lit("}")) {
                    return false;
                  }
                }
                if (c.lit(",")) continue;
                if (!c.lit("]")) return false;
                break;
              }
            }
          }
          if (!c.lit("}")) return false;
        }
        if (c.lit(",")) continue;
        if (!c.lit("]")) return false;
        break;
      }
    }
  }
  return c.lit("}") && c.end();
}

uint32_t Builder::tokens(const uint8_t* p, uint32_t n, uint32_t& bytes_off) {
  bytes_off = arena_alloc(64 * n);
  uint32_t first = pl.n_pts;
  for (uint32_t k = 0; k < n; k++) {
    pl.wire.resize((pl.wire.size() + 15) & ~(size_t)15, 0);
    uint32_t raw = (uint32_t)pl.wire.size();
    pl.wire.insert(pl.wire.end(), p + 64 * k, p + 64 * k + 64);
    point(raw, 64, bytes_off + 64 * k, NONE);
  }
  return first;
}

// One side (inputs or outputs) of transfer WF verification:
// parseProof (wellformedness.go:200-240) + RecomputeCommitments (common/schnorr.go:106-118).
bool Builder::wf_side(uint32_t tok_pt, uint32_t n, const std::vector<Ref>& vals, const std::vector<Ref>& bfs,
                      const Ref& type, const Ref& sum, const Ref& chal, uint32_t& s_type, uint32_t& s_sum,
                      uint32_t& s_chal, uint32_t wfout_bytes) {
  if (vals.size() != n || bfs.size() != n) {
    fail(E_MALFORMED);
    return false;
  }
  if (type.nil()) {  // ModMul(ttype, n) dereferences nil (wellformedness.go:227)
    fail(E_PANIC);
    return false;
  }
  for (auto& b : bfs)
    if (b.nil()) {  // crypto.Sum: "invalid value to be summed"
      fail(E_MALFORMED);
      return false;
    }
  if (chal.nil()) {
    fail(E_MALFORMED);
    return false;
  }
  for (auto& v : vals)
    if (v.nil()) {
      fail(E_MALFORMED);
      return false;
    }
  if (sum.nil()) {
    fail(E_MALFORMED);
    return false;
  }
  if (s_type == NONE) s_type = scalar(type);
  if (s_sum == NONE) s_sum = scalar(sum);
  if (s_chal == NONE) s_chal = scalar(chal);
  // derived scalars: type * n, sum of blinding factors
  uint32_t s_tn = pl.n_scal++;
  pl.sc.push_back({SOP_MULK, s_type, n, s_tn});
  uint32_t s_bf[64];
  std::vector<uint32_t> bfi(n), vai(n);
  for (uint32_t i = 0; i < n; i++) {
    vai[i] = scalar(vals[i]);
    bfi[i] = scalar(bfs[i]);
  }
  (void)s_bf;
  uint32_t s_bfsum = pl.n_scal++;
  pl.sc.push_back({SOP_SUM, (uint32_t)pl.sclist.size(), n, s_bfsum});
  pl.sclist.insert(pl.sclist.end(), bfi.begin(), bfi.end());
  std::vector<VTerm> all;
  for (uint32_t i = 0; i < n; i++) {
    g1job({{G1B_PED0, s_type}, {G1B_PED1, vai[i]}, {G1B_PED2, bfi[i]}}, {vterm(tok_pt + i)}, s_chal,
          wfout_bytes + 64 * i);
    all.push_back(vterm(tok_pt + i));
  }
  g1job({{G1B_PED0, s_tn}, {G1B_PED1, s_sum}, {G1B_PED2, s_bfsum}}, all, s_chal, wfout_bytes + 64 * n);
  return true;
}

void Builder::decode_range(Doc& doc, RangeDoc& r) {
  int64_t top = doc.top();
  r.chal = doc.elem(doc.f(top, "Challenge"));
  bool isnil;
  int64_t eq = doc.obj(doc.f(top, "EqualityProofs"), isnil);
  r.eq_nil = isnil;
  if (!isnil) {
    r.eq_type = doc.elem(doc.f(eq, "Type"));
    r.eq_val = doc.list(doc.f(eq, "Value"));
    r.eq_tbf = doc.list(doc.f(eq, "TokenBlindingFactor"));
    r.eq_cbf = doc.list(doc.f(eq, "CommitmentBlindingFactor"));
  }
  int64_t mps = doc.f(top, "MembershipProofs");
  if (mps >= 0 && doc.d.at((uint32_t)mps).type != J_NULL) {
    if (doc.d.at((uint32_t)mps).type != J_ARR) {
      doc.err = true;
      return;
    }
    uint32_t n = doc.d.len((uint32_t)mps);
    r.mps.resize(n);
    for (uint32_t k = 0; k < n; k++) {
      MP& mp = r.mps[k];
      int64_t o = doc.obj(doc.d.elem((uint32_t)mps, k), isnil);
      mp.nil = isnil;
      if (isnil) continue;
      mp.coms = doc.list(doc.f(o, "Commitments"));
      int64_t sps = doc.f(o, "SignatureProofs");
      if (sps >= 0 && doc.d.at((uint32_t)sps).type != J_NULL) {
        if (doc.d.at((uint32_t)sps).type != J_ARR) {
          doc.err = true;
          continue;
        }
        uint32_t m = doc.d.len((uint32_t)sps);
        mp.sps.resize(m);
        for (uint32_t i = 0; i < m; i++) {
          Membership& s = mp.sps[i];
          int64_t so = doc.obj(doc.d.elem((uint32_t)sps, i), isnil);
          s.nil = isnil;
          if (isnil) continue;
          s.chal = doc.elem(doc.f(so, "Challenge"));
          int64_t sig = doc.obj(doc.f(so, "Signature"), isnil);
          s.sig_nil = isnil;
          if (!isnil) {
            s.R = doc.elem(doc.f(sig, "R"));
            s.S = doc.elem(doc.f(sig, "S"));
          }
          s.value = doc.elem(doc.f(so, "Value"));
          s.combf = doc.elem(doc.f(so, "ComBlindingFactor"));
          s.sigbf = doc.elem(doc.f(so, "SigBlindingFactor"));
          s.hash = doc.elem(doc.f(so, "Hash"));
          s.commitment = doc.elem(doc.f(so, "Commitment"));
        }
      }
    }
  }
}

static const char SIG_JSON_R[] = "{\"R\":{\"curve\":1,\"element\":\"";  // 27
static const char SIG_JSON_S[] = "\"},\"S\":{\"curve\":1,\"element\":\"";  // 29
static const char SIG_JSON_E[] = "\"}}";                                   // 3
static constexpr uint32_t SIG_JSON_LEN = 27 + 88 + 29 + 88 + 3;            // 235
static constexpr uint32_t DIGIT_SLOT = 64 + 64 + 384 + SIG_JSON_LEN;       // 747

// rangeproof.Verifier.Verify (range/proof.go:211-284)
void Builder::range_part(const std::vector<uint8_t>& rc, bool rc_nil, uint32_t out_pt, uint32_t out_bytes,
                         uint32_t n) {
  begin_range();
  RangeDoc r;
  size_t wire_mark = pl.wire.size();
  if (rc_nil || !fast_range(rc, r)) {
    pl.wire.resize(wire_mark);
    r = RangeDoc();
    Doc doc(&pl, jrc);
    if (!doc.parse(rc, rc_nil, RANGE_F)) {
      fail(E_PARSE);
      return;
    }
    decode_range(doc, r);
    if (doc.panic) {
      fail(E_PANIC);
      return;
    }
    if (doc.err) {
      pl.wire.resize(wire_mark);
      fail(E_PARSE);
      return;
    }
  }
  // decode every G1 of the document (json.Unmarshal -> mathlib NewG1FromBytes)
  uint32_t e = (uint32_t)pp.exponent;
  // commitments rows (hashed in the range transcript) -- laid out contiguously
  uint32_t ncoms = 0;
  for (auto& mp : r.mps)
    if (!mp.nil) ncoms += (uint32_t)mp.coms.size();
  uint32_t coms_bytes = arena_alloc(64 * ncoms);
  uint32_t pts_first = pl.n_pts;
  std::vector<std::vector<uint32_t>> com_pt(r.mps.size());
  uint32_t cb = coms_bytes;
  for (size_t k = 0; k < r.mps.size(); k++) {
    if (r.mps[k].nil) continue;
    for (auto& c : r.mps[k].coms) {
      if (c.nil()) {
        com_pt[k].push_back(NONE);
      } else {
        com_pt[k].push_back(point(c, cb));
      }
      cb += 64;
    }
  }
  // membership proof points and their arena slots
  struct DigitPts {
    uint32_t R = NONE, S = NONE, C = NONE, slot = 0;
  };
  std::vector<std::vector<DigitPts>> dp(r.mps.size());
  for (size_t k = 0; k < r.mps.size(); k++) {
    if (r.mps[k].nil) continue;
    for (auto& s : r.mps[k].sps) {
      DigitPts d;
      if (!s.nil) {
        d.slot = arena_alloc(DIGIT_SLOT);
        uint8_t* js = &pl.arena[d.slot + 512];
        memcpy(js, SIG_JSON_R, 27);
        memcpy(js + 27 + 88, SIG_JSON_S, 29);
        memcpy(js + 27 + 88 + 29 + 88, SIG_JSON_E, 3);
        if (!s.sig_nil && !s.R.nil()) d.R = point(s.R, NONE, d.slot + 512 + 27);
        if (!s.sig_nil && !s.S.nil()) d.S = point(s.S, NONE, d.slot + 512 + 27 + 88 + 29);
        if (!s.commitment.nil()) d.C = point(s.commitment, d.slot);
      }
      dp[k].push_back(d);
    }
  }
  if (pl.n_pts > pts_first) check(CK_PTS, E_PARSE, pts_first, pl.n_pts - pts_first);

  if (r.mps.size() != n) {
    fail(E_MALFORMED);
    return;
  }
  for (auto& mp : r.mps) {
    if (mp.nil || mp.coms.size() != mp.sps.size()) {
      fail(E_MALFORMED);
      return;
    }
  }
  for (auto& mp : r.mps)
    for (auto& s : mp.sps)
      if (s.nil) {  // MembershipVerifier.Verify(nil) dereferences nil in a goroutine
        fail(E_PANIC);
        return;
      }
  // membership verifications (sigproof/membership.go:162-180)
  for (size_t k = 0; k < r.mps.size(); k++) {
    for (size_t i = 0; i < r.mps[k].sps.size(); i++) {
      const Membership& s = r.mps[k].sps[i];
      const DigitPts& d = dp[k][i];
      // POKVerifier.recomputeCommitment (pok.go:160-204)
      if (s.value.nil() || s.hash.nil() || s.sig_nil || s.R.nil() || s.S.nil() || s.chal.nil() ||
          s.sigbf.nil()) {
        fail(E_MALFORMED);
        return;
      }
      // Schnorr on Commitments[k][i] (membership.go:297-299)
      if (com_pt[k][i] == NONE || s.combf.nil()) {
        fail(E_MALFORMED);
        return;
      }
      // computeChallenge marshals proof.Commitment (membership.go:261)
      if (d.C == NONE) {
        fail(E_MALFORMED);
        return;
      }
      uint32_t sc_ch = scalar(s.chal), sc_v = scalar(s.value), sc_cb = scalar(s.combf);
      uint32_t sc_sb = scalar(s.sigbf), sc_h = scalar(s.hash);
      // G1 commitment: v*Ped0 + cb*Ped1 - c*Commitments[k][i]
      g1job({{G1B_PED0, sc_v}, {G1B_PED1, sc_cb}}, {vterm(com_pt[k][i])}, sc_ch, d.slot + 64);
      // P1 = sigbf*P - c*S   (pairs with Q)
      uint32_t p1 = g1job({{G1B_PEDGEN, sc_sb}}, {vterm(d.S)}, sc_ch, NONE, true);
      // t' = c*PK0 + v*PK1 + h*PK2   (pairs with R)
      G2Job g2;
      memset(&g2, 0, sizeof(g2));
      g2.nfix = 3;
      g2.fbase[0] = G2B_PK0;
      g2.fscal[0] = sc_ch;
      g2.fbase[1] = G2B_PK1;
      g2.fscal[1] = sc_v;
      g2.fbase[2] = G2B_PK2;
      g2.fscal[2] = sc_h;
      g2.out = pl.n_g2out++;
      pl.g2.push_back(g2);
      pl.pr.push_back({p1, d.R, g2.out, d.slot + 128, NONE});
      HashJob h;
      h.seg_start = (uint32_t)pl.seg.size();
      seg(CONST_FLAG | C_PED0, 128);
      seg(d.slot, 128);
      seg(CONST_FLAG | C_PEDGEN, 64);
      seg(CONST_FLAG | C_PK_Q, 512);
      seg(d.slot + 128, 384 + SIG_JSON_LEN);
      h.seg_count = 5;
      h.expect = sc_ch;
      h.out_scal = dbg_scal();
      pl.hmain.push_back(h);
      check(CK_HASH, E_MEMBERSHIP, (uint32_t)pl.hmain.size() - 1);
    }
  }
  // recomputeCommitments (range/proof.go:393-444)
  if (r.eq_nil || r.eq_val.size() != n || r.eq_tbf.size() != n || r.eq_cbf.size() != n) {
    fail(E_MALFORMED);
    return;
  }
  if (r.chal.nil() || r.eq_type.nil()) {
    fail(E_MALFORMED);
    return;
  }
  for (uint32_t j = 0; j < n; j++)
    if (r.eq_val[j].nil() || r.eq_tbf[j].nil()) {
      fail(E_MALFORMED);
      return;
    }
  for (uint32_t j = 0; j < n; j++)
    if (pp.exponent <= 0 || r.mps[j].coms.size() != e || r.eq_cbf[j].nil()) {
      fail(E_MALFORMED);
      return;
    }
  uint32_t sc_rc = scalar(r.chal), sc_t = scalar(r.eq_type);
  uint32_t rg_bytes = arena_alloc(128 * n);
  std::vector<uint32_t> sv(n);
  for (uint32_t j = 0; j < n; j++) {
    sv[j] = scalar(r.eq_val[j]);
    uint32_t stb = scalar(r.eq_tbf[j]);
    g1job({{G1B_PED0, sc_t}, {G1B_PED1, sv[j]}, {G1B_PED2, stb}}, {vterm(out_pt + j)}, sc_rc, rg_bytes + 64 * j);
  }
  for (uint32_t j = 0; j < n; j++) {
    uint32_t scb = scalar(r.eq_cbf[j]);
    std::vector<VTerm> terms;
    if (pp.pow_exact && e > 1) {  // sum_i b^i com_i in Horner order (VT_HORNER): same point
      for (uint32_t i = e; i-- > 0;) terms.push_back(vterm(com_pt[j][i], pp.base));
      terms[0].flags = VT_HORNER;
    } else {
      // int64 weights; only -2^63 (math.Pow >= 2^63) is negative: weight 2^63, subtracted
      for (uint32_t i = 0; i < e; i++) {
        const int64_t w = (int64_t)pp.pow[i];
        terms.push_back(vterm(com_pt[j][i], w < 0 ? 0 - (uint64_t)w : (uint64_t)w));
        if (w < 0) terms.back().flags = VT_NEG;
      }
    }
    g1job({{G1B_PED0, sv[j]}, {G1B_PED1, scb}}, terms, sc_rc, rg_bytes + 64 * (n + j));
  }
  HashJob h;
  h.seg_start = (uint32_t)pl.seg.size();
  seg(CONST_FLAG | C_PEDGEN, 64);
  seg(out_bytes, 64 * n);
  seg(rg_bytes, 128 * n);
  seg(CONST_FLAG | C_PED0, 192);
  seg(CONST_FLAG | C_Q_PK, 512);
  seg(coms_bytes, 64 * ncoms);
  h.seg_count = 6;
  h.expect = sc_rc;
  h.out_scal = dbg_scal();
  pl.hmain.push_back(h);
  check(CK_HASH, E_RANGE, (uint32_t)pl.hmain.size() - 1);
}

void Builder::transfer(const TransferIn& t) {
  begin_tx(0);
  uint32_t tok_bytes;
  uint32_t tok_pt = tokens(t.inputs, t.n_in, tok_bytes);
  tokens(t.outputs, t.n_out, tok_bytes), (void)0;
  // tokens() allocated inputs then outputs contiguously
  uint32_t in_bytes = tok_bytes - 64 * t.n_in;
  if (t.n_in + t.n_out) check(CK_PTS, E_PARSE, tok_pt, t.n_in + t.n_out);

  // transfer.Proof JSON (transfer.go:125-129)
  bool wf_nil = true, rc_nil = true;
  Canon oc(t.proof, t.proof_len, &pl);
  bool outer_fast = oc.lit("{\"WellFormedness\":") && oc.bytes(wfb, wf_nil) && oc.lit(",\"RangeCorrectness\":") &&
                    oc.bytes(rcb, rc_nil) && oc.lit("}") && oc.end();
  if (!outer_fast) {
    JDoc& top = jtop;
    if (!top.parse(t.proof, t.proof_len)) {
      fail(E_PARSE);
      end_tx();
      return;
    }
    uint32_t root = top.root();
    bool bad = false;
    if (top.at(root).type == J_OBJ) {
      DecStatus a = dec_bytes(top, top.field(root, "WellFormedness"), wfb);
      DecStatus b = dec_bytes(top, top.field(root, "RangeCorrectness"), rcb);
      bad = (a == D_ERR || b == D_ERR);
      wf_nil = (a != D_OK);
      rc_nil = (b != D_OK);
    } else if (top.at(root).type != J_NULL) {
      bad = true;
    }
    if (bad) {
      fail(E_PARSE);
      end_tx();
      return;
    }
  }
  // WellFormednessVerifier.Verify (wellformedness.go:157-197, parseProof :200-240)
  {
    Doc doc(&pl, jwf);
    size_t mark = pl.wire.size();
    std::vector<Ref> ibf, obf, ivl, ovl;
    Ref type, sum, chal;
    Canon c(wfb.data(), wfb.size(), &pl);
    bool fast = !wf_nil && c.lit("{\"InputBlindingFactors\":") && c.list(ibf) &&
                c.lit(",\"OutputBlindingFactors\":") && c.list(obf) && c.lit(",\"InputValues\":") && c.list(ivl) &&
                c.lit(",\"OutputValues\":") && c.list(ovl) && c.lit(",\"Type\":") && c.elem(type) &&
                c.lit(",\"Sum\":") && c.elem(sum) && c.lit(",\"Challenge\":") && c.elem(chal) && c.lit("}") && c.end();
    if (!fast) pl.wire.resize(mark);
    if (!fast && !doc.parse(wfb, wf_nil)) {
      fail(E_PARSE);
    } else {
      if (!fast) {
        int64_t top = doc.top();
        ibf = doc.list(doc.f(top, "InputBlindingFactors"));
        obf = doc.list(doc.f(top, "OutputBlindingFactors"));
        ivl = doc.list(doc.f(top, "InputValues"));
        ovl = doc.list(doc.f(top, "OutputValues"));
        type = doc.elem(doc.f(top, "Type"));
        sum = doc.elem(doc.f(top, "Sum"));
        chal = doc.elem(doc.f(top, "Challenge"));
      }
      if (doc.panic) {
        fail(E_PANIC);
      } else if (doc.err) {
        pl.wire.resize(mark);
        fail(E_PARSE);
      } else {
        uint32_t s_type = NONE, s_sum = NONE, s_chal = NONE;
        uint32_t nwf = t.n_in + 1 + t.n_out + 1;
        uint32_t wfout = arena_alloc(64 * nwf);
        if (wf_side(tok_pt, t.n_in, ivl, ibf, type, sum, chal, s_type, s_sum, s_chal, wfout) &&
            wf_side(tok_pt + t.n_in, t.n_out, ovl, obf, type, sum, chal, s_type, s_sum, s_chal,
                    wfout + 64 * (t.n_in + 1))) {
          HashJob h;
          h.seg_start = (uint32_t)pl.seg.size();
          seg(wfout, 64 * nwf);
          seg(in_bytes, 64 * (t.n_in + t.n_out));
          h.seg_count = 2;
          h.expect = s_chal;
          h.out_scal = dbg_scal();
          pl.hmain.push_back(h);
          check(CK_HASH, E_WF, (uint32_t)pl.hmain.size() - 1);
        }
      }
    }
  }
  // ownership transfer (1-in/1-out) skips the range proof (transfer.go:70-72)
  if (!(t.n_in == 1 && t.n_out == 1)) range_part(rcb, rc_nil, tok_pt + t.n_in, in_bytes + 64 * t.n_in, t.n_out);
  end_tx();
}

// Token commitment H(type)*Ped0 + value*Ped1 + bf*Ped2 (token/token.go:64-76,
// common/schnorr.go:59-76); with a commitment given, the auditor's opening check
// (audit/auditor.go:208-234): its canonical RawBytes land next to the
// recomputed ones and the host compares them (G1 Equals on affine points).
void Builder::opening(const OpeningIn& o) {
  begin_tx(1);
  uint32_t res = arena_alloc(128);
  pl.item_off.push_back(res);
  if (o.commitment) {
    pl.wire.resize((pl.wire.size() + 15) & ~(size_t)15, 0);
    uint32_t raw = (uint32_t)pl.wire.size();
    pl.wire.insert(pl.wire.end(), o.commitment, o.commitment + 64);
    uint32_t pt = point(raw, 64, res + 64, NONE);
    check(CK_PTS, E_PARSE, pt, 1);
  }
  uint32_t str_off = arena_alloc((uint32_t)o.type_len);
  if (o.type_len) memcpy(pl.arena.data() + str_off, o.type, o.type_len);
  uint32_t s_h = pl.n_scal++;
  HashJob h;
  h.seg_start = (uint32_t)pl.seg.size();
  seg(str_off, (uint32_t)o.type_len);
  h.seg_count = 1;
  h.expect = NONE;
  h.out_scal = s_h;
  pl.hpre.push_back(h);
  Ref v, b;
  for (int k = 0; k < 2; k++) {
    pl.wire.resize((pl.wire.size() + 15) & ~(size_t)15, 0);
    Ref& r = k ? b : v;
    r.off = (int64_t)pl.wire.size();
    r.len = 32;
    const uint8_t* src = k ? o.bf : o.value;
    pl.wire.insert(pl.wire.end(), src, src + 32);
  }
  uint32_t s_v = scalar(v), s_b = scalar(b);
  g1job({{G1B_PED0, s_h}, {G1B_PED1, s_v}, {G1B_PED2, s_b}}, {}, NONE, res);
  end_tx();
}

void Builder::issue(const IssueIn& t) {
  begin_tx(1);
  uint32_t tok_bytes;
  uint32_t tok_pt = tokens(t.outputs, t.n_out, tok_bytes);
  if (t.n_out) check(CK_PTS, E_PARSE, tok_pt, t.n_out);
  uint32_t n = t.n_out;
  bool wf_nil = true, rc_nil = true;
  Canon oc(t.proof, t.proof_len, &pl);
  bool outer_fast = oc.lit("{\"WellFormedness\":") && oc.bytes(wfb, wf_nil) && oc.lit(",\"RangeCorrectness\":") &&
                    oc.bytes(rcb, rc_nil) && oc.lit("}") && oc.end();
  if (!outer_fast) {
    JDoc& top = jtop;
    if (!top.parse(t.proof, t.proof_len)) {
      fail(E_PARSE);
      end_tx();
      return;
    }
    uint32_t root = top.root();
    bool bad = false;
    if (top.at(root).type == J_OBJ) {
      DecStatus a = dec_bytes(top, top.field(root, "WellFormedness"), wfb);
      DecStatus b = dec_bytes(top, top.field(root, "RangeCorrectness"), rcb);
      bad = (a == D_ERR || b == D_ERR);
      wf_nil = (a != D_OK);
      rc_nil = (b != D_OK);
    } else if (top.at(root).type != J_NULL) {
      bad = true;
    }
    if (bad) {
      fail(E_PARSE);
      end_tx();
      return;
    }
  }
  // issue WellFormednessVerifier.Verify (issue/wellformedness.go:206-236, parseProof :239-265)
  Doc doc(&pl, jwf);
  size_t mark = pl.wire.size();
  Ref type, chal;
  std::vector<Ref> vals, bfs;
  std::string clear;
  Canon c(wfb.data(), wfb.size(), &pl);
  bool fast = !wf_nil && c.lit("{\"Type\":") && c.elem(type) && c.lit(",\"Values\":") && c.list(vals) &&
              c.lit(",\"BlindingFactors\":") && c.list(bfs) && c.lit(",\"TypeInTheClear\":") &&
              c.plain_string(clear) && c.lit(",\"Challenge\":") && c.elem(chal) && c.lit("}") && c.end();
  if (!fast) {
    pl.wire.resize(mark);
    clear.clear();
    if (!doc.parse(wfb, wf_nil)) {
      fail(E_PARSE);
      end_tx();
      return;
    }
    int64_t top = doc.top();
    type = doc.elem(doc.f(top, "Type"));
    vals = doc.list(doc.f(top, "Values"));
    bfs = doc.list(doc.f(top, "BlindingFactors"));
    DecStatus cs = dec_string(doc.d, doc.f(top, "TypeInTheClear"), clear);
    if (cs == D_ERR) doc.err = true;
    chal = doc.elem(doc.f(top, "Challenge"));
  }
  if (doc.panic) {
    fail(E_PANIC);
    end_tx();
    return;
  }
  if (doc.err) {
    pl.wire.resize(mark);
    fail(E_PARSE);
    end_tx();
    return;
  }
  if (chal.nil()) {
    fail(E_MALFORMED);
    end_tx();
    return;
  }
  uint32_t s_chal = scalar(chal);
  uint32_t s_type = NONE;
  if (!t.anonymous) {
    // Type := c * HashToZr(TypeInTheClear)  (issue/wellformedness.go:243-245)
    uint32_t str_off = arena_alloc((uint32_t)clear.size());
    memcpy(pl.arena.data() + str_off, clear.data(), clear.size());
    uint32_t s_h = pl.n_scal++;
    HashJob h;
    h.seg_start = (uint32_t)pl.seg.size();
    seg(str_off, (uint32_t)clear.size());
    h.seg_count = 1;
    h.expect = NONE;
    h.out_scal = s_h;
    pl.hpre.push_back(h);
    s_type = pl.n_scal++;
    pl.sc.push_back({SOP_MUL, s_chal, s_h, s_type});
  }
  if (vals.size() != n || bfs.size() != n) {
    fail(E_MALFORMED);
    end_tx();
    return;
  }
  if (t.anonymous && type.nil() && n > 0) {
    fail(E_MALFORMED);
    end_tx();
    return;
  }
  for (uint32_t i = 0; i < n; i++)
    if (vals[i].nil() || bfs[i].nil()) {
      fail(E_MALFORMED);
      end_tx();
      return;
    }
  if (t.anonymous && n > 0) s_type = scalar(type);
  uint32_t wfout = arena_alloc(64 * n);
  for (uint32_t i = 0; i < n; i++) {
    uint32_t sv = scalar(vals[i]), sb = scalar(bfs[i]);
    g1job({{G1B_PED0, s_type}, {G1B_PED1, sv}, {G1B_PED2, sb}}, {vterm(tok_pt + i)}, s_chal, wfout + 64 * i);
  }
  HashJob h;
  h.seg_start = (uint32_t)pl.seg.size();
  seg(wfout, 64 * n);
  seg(tok_bytes, 64 * n);
  h.seg_count = 2;
  h.expect = s_chal;
  h.out_scal = dbg_scal();
  pl.hmain.push_back(h);
  check(CK_HASH, E_WF, (uint32_t)pl.hmain.size() - 1);
  range_part(rcb, rc_nil, tok_pt, tok_bytes, n);
  end_tx();
}

}  // namespace

// ------------------------------------------------------------------ work pool
struct WorkPool::State {
  std::mutex run_mu;  // one run() at a time
  std::mutex mu;
  std::condition_variable cv, done_cv;
  const std::function<void(size_t)>* fn = nullptr;
  size_t n = 0;
  std::atomic<size_t> next{0};
  size_t gen = 0, active = 0;
  bool stop = false;
  std::vector<std::thread> th;
};

WorkPool::WorkPool(int threads) : st_(new State()), nthreads_(std::max(0, threads - 1)) {
  for (int t = 0; t < nthreads_; t++) {
    st_->th.emplace_back([this]() {
      State& s = *st_;
      size_t seen = 0;
      while (true) {
        std::unique_lock<std::mutex> lk(s.mu);
        s.cv.wait(lk, [&]() { return s.stop || s.gen != seen; });
        if (s.stop) return;
        seen = s.gen;
        const std::function<void(size_t)>* f = s.fn;
        size_t n = s.n;
        lk.unlock();
        for (size_t i; (i = s.next.fetch_add(1)) < n;) (*f)(i);
        lk.lock();
        if (--s.active == 0) s.done_cv.notify_all();
      }
    });
  }
}

WorkPool::~WorkPool() {
  {
    std::lock_guard<std::mutex> lk(st_->mu);
    st_->stop = true;
  }
  st_->cv.notify_all();
  for (auto& t : st_->th) t.join();
  delete st_;
}

void WorkPool::run(size_t n, const std::function<void(size_t)>& f) {
  if (n == 0) return;
  State& s = *st_;
  std::lock_guard<std::mutex> rl(s.run_mu);
  if (nthreads_ == 0 || n == 1) {
    for (size_t i = 0; i < n; i++) f(i);
    return;
  }
  {
    std::lock_guard<std::mutex> lk(s.mu);
    s.fn = &f;
    s.n = n;
    s.next.store(0);
    s.active = (size_t)nthreads_;
    s.gen++;
  }
  s.cv.notify_all();
  for (size_t i; (i = s.next.fetch_add(1)) < n;) f(i);
  std::unique_lock<std::mutex> lk(s.mu);
  s.done_cv.wait(lk, [&]() { return s.active == 0; });
}

// ------------------------------------------------------------------ flat plans
namespace {

constexpr size_t SEC_ALIGN = 256;
constexpr size_t IDX_LIMIT = (size_t)1 << 31;  // Seg.off uses bit 31 (CONST_FLAG); NONE is 2^32 - 1

size_t elem_size(int s) {
  switch (s) {
    case PS_WIRE: case PS_ARENA: case PS_OUT: return 1;
    case PS_DEC: return sizeof(DecodeJob);
    case PS_ZR: return sizeof(ZrJob);
    case PS_SC: case PS_SC1: case PS_SCPOST: return sizeof(ScalJob);
    case PS_SCLIST: return sizeof(uint32_t);
    case PS_VT: return sizeof(VTerm);
    case PS_G1: case PS_G1P: return sizeof(G1Job);
    case PS_G2: return sizeof(G2Job);
    case PS_PR: return sizeof(PairJob);
    case PS_SEG: return sizeof(Seg);
    case PS_HPRE: case PS_HMAIN: return sizeof(HashJob);
    case PS_CK: return sizeof(Check);
    case PS_TX: return sizeof(TxChecks);
    case PS_RND: return sizeof(RandJob);
    case PS_EMIT: return sizeof(EmitJob);
    case PS_B64: return sizeof(B64Job);
    case PS_CP: case PS_CP2: return sizeof(CopyJob);
  }
  return 1;
}

size_t piece_count(const Plan& p, int s) {
  switch (s) {
    case PS_WIRE: return p.wire.size();
    case PS_ARENA: return p.dev_pools ? p.arena_len : p.arena.size();
    case PS_DEC: return p.dec.size();
    case PS_ZR: return p.zr.size();
    case PS_SC: return p.sc.size();
    case PS_SCLIST: return p.sclist.size();
    case PS_VT: return p.vt.size();
    case PS_G1: return p.g1.size();
    case PS_G1P: return p.g1p.size();
    case PS_G2: return p.g2.size();
    case PS_PR: return p.pr.size();
    case PS_SEG: return p.seg.size();
    case PS_HPRE: return p.hpre.size();
    case PS_HMAIN: return p.hmain.size();
    case PS_CK: return p.ck.size();
    case PS_TX: return p.tx.size();
    case PS_RND: return p.rnd.size();
    case PS_SC1: return p.sc1.size();
    case PS_SCPOST: return p.sc_post.size();
    case PS_EMIT: return p.emit.size();
    case PS_B64: return p.b64.size();
    case PS_CP: return p.cp.size();
    case PS_CP2: return p.cp2.size();
    case PS_OUT: return p.dev_pools ? p.out_len : p.out.size();
  }
  return 0;
}

// Piece `b` (indices local to b) written at base `o` of the sections dst[s]
// (element 0 of each) with every index relocated: the flat plan's blob, or the
// tail of another Plan (plan_append; const-region segments keep their flag).
void relocate_into(const Plan& b, const PieceBase& o, bool p2_g1out, bool keep_const, uint8_t* const* dst,
                   bool copy_pools = true) {
  const uint32_t o_wire = (uint32_t)o.sec[PS_WIRE], o_arena = (uint32_t)o.sec[PS_ARENA];
  const uint32_t o_pts = o.pts, o_scal = o.scal, o_g1 = o.g1out, o_g2 = o.g2out;
  const uint32_t o_list = (uint32_t)o.sec[PS_SCLIST], o_vt = (uint32_t)o.sec[PS_VT], o_seg = (uint32_t)o.sec[PS_SEG];
  const uint32_t o_hmain = (uint32_t)o.sec[PS_HMAIN], o_ck = (uint32_t)o.sec[PS_CK], o_out = (uint32_t)o.sec[PS_OUT];
  auto rel = [](uint32_t v, uint32_t off) { return v == NONE ? NONE : v + off; };
  if (!b.wire.empty()) memcpy(dst[PS_WIRE] + o_wire, b.wire.data(), b.wire.size());
  if (copy_pools && !b.arena.empty()) memcpy(dst[PS_ARENA] + o_arena, b.arena.data(), b.arena.size());
  if (copy_pools && !b.out.empty()) memcpy(dst[PS_OUT] + o_out, b.out.data(), b.out.size());
  DecodeJob* dec = reinterpret_cast<DecodeJob*>(dst[PS_DEC]) + o.sec[PS_DEC];
  for (DecodeJob j : b.dec) {
    j.raw += o_wire;
    j.out += o_pts;
    j.bytes = rel(j.bytes, o_arena);
    j.b64 = rel(j.b64, o_arena);
    *dec++ = j;
  }
  ZrJob* zr = reinterpret_cast<ZrJob*>(dst[PS_ZR]) + o.sec[PS_ZR];
  for (ZrJob j : b.zr) {
    j.raw += o_wire;
    j.out += o_scal;
    *zr++ = j;
  }
  auto rel_sc = [&](ScalJob j) {
    if (j.op == SOP_SUM) {
      j.a += o_list;
    } else {
      j.a += o_scal;
      if (j.op == SOP_MUL || j.op == SOP_MADD) j.b += o_scal;
      if (j.op == SOP_MADD) j.c += o_scal;
    }
    j.out += o_scal;
    return j;
  };
  const int scs[3] = {PS_SC, PS_SC1, PS_SCPOST};
  const std::vector<ScalJob>* scv[3] = {&b.sc, &b.sc1, &b.sc_post};
  for (int k = 0; k < 3; k++) {
    ScalJob* d = reinterpret_cast<ScalJob*>(dst[scs[k]]) + o.sec[scs[k]];
    for (const ScalJob& j : *scv[k]) *d++ = rel_sc(j);
  }
  uint32_t* sl = reinterpret_cast<uint32_t*>(dst[PS_SCLIST]) + o.sec[PS_SCLIST];
  for (uint32_t v : b.sclist) *sl++ = v + o_scal;
  VTerm* vt = reinterpret_cast<VTerm*>(dst[PS_VT]) + o.sec[PS_VT];
  for (VTerm v : b.vt) {
    v.pt += o_pts;
    *vt++ = v;
  }
  for (int side = 0; side < 2; side++) {
    int sec = side ? PS_G1P : PS_G1;
    G1Job* d = reinterpret_cast<G1Job*>(dst[sec]) + o.sec[sec];
    for (G1Job j : (side ? b.g1p : b.g1)) {
      for (int k = 0; k < j.nfix; k++) j.fscal[k] += o_scal;
      j.vstart += o_vt;
      j.vscal = rel(j.vscal, o_scal);
      j.out += o_g1;
      j.bytes = rel(j.bytes, o_arena);
      j.b64 = rel(j.b64, o_arena);
      *d++ = j;
    }
  }
  G2Job* g2 = reinterpret_cast<G2Job*>(dst[PS_G2]) + o.sec[PS_G2];
  for (G2Job j : b.g2) {
    for (int k = 0; k < j.nfix; k++) j.fscal[k] += o_scal;
    j.out += o_g2;
    *g2++ = j;
  }
  PairJob* pr = reinterpret_cast<PairJob*>(dst[PS_PR]) + o.sec[PS_PR];
  for (PairJob j : b.pr) {
    j.p1 += o_g1;
    j.p2 += p2_g1out ? o_g1 : o_pts;
    j.q2 = rel(j.q2, o_g2);
    j.p3 = rel(j.p3, o_g1);
    j.bytes += o_arena;
    *pr++ = j;
  }
  Seg* sg = reinterpret_cast<Seg*>(dst[PS_SEG]) + o.sec[PS_SEG];
  for (Seg s : b.seg) {
    if (s.off & CONST_FLAG) {
      if (!keep_const) s.off &= ~CONST_FLAG;  // const region sits at absolute offset 0
    } else {
      s.off += o_arena;
    }
    *sg++ = s;
  }
  const int hs[2] = {PS_HPRE, PS_HMAIN};
  const std::vector<HashJob>* hv[2] = {&b.hpre, &b.hmain};
  for (int k = 0; k < 2; k++) {
    HashJob* d = reinterpret_cast<HashJob*>(dst[hs[k]]) + o.sec[hs[k]];
    for (HashJob h : *hv[k]) {
      h.seg_start += o_seg;
      h.expect = rel(h.expect, o_scal);
      h.out_scal = rel(h.out_scal, o_scal);
      *d++ = h;
    }
  }
  Check* ck = reinterpret_cast<Check*>(dst[PS_CK]) + o.sec[PS_CK];
  for (Check c : b.ck) {
    if (c.kind == CK_PTS) c.a += o_pts;
    if (c.kind == CK_HASH) c.a += o_hmain;
    *ck++ = c;
  }
  TxChecks* tx = reinterpret_cast<TxChecks*>(dst[PS_TX]) + o.sec[PS_TX];
  for (TxChecks t : b.tx) {
    t.wf_start += o_ck;
    t.rg_start += o_ck;
    *tx++ = t;
  }
  RandJob* rnd = reinterpret_cast<RandJob*>(dst[PS_RND]) + o.sec[PS_RND];
  for (RandJob j : b.rnd) {
    j.seed += o_arena;
    j.tag += o_arena;
    j.out += o_scal;
    *rnd++ = j;
  }
  EmitJob* em = reinterpret_cast<EmitJob*>(dst[PS_EMIT]) + o.sec[PS_EMIT];
  for (EmitJob j : b.emit) {
    j.dst += o_arena;
    j.src += j.kind == EM_ZR ? o_scal : o_arena;
    *em++ = j;
  }
  B64Job* bj = reinterpret_cast<B64Job*>(dst[PS_B64]) + o.sec[PS_B64];
  for (B64Job j : b.b64) {
    j.src += o_arena;
    j.dst += o_out;
    *bj++ = j;
  }
  const int cps[2] = {PS_CP, PS_CP2};
  const std::vector<CopyJob>* cpv[2] = {&b.cp, &b.cp2};
  for (int k = 0; k < 2; k++) {
    CopyJob* d = reinterpret_cast<CopyJob*>(dst[cps[k]]) + o.sec[cps[k]];
    for (CopyJob j : *cpv[k]) {
      j.src += o_wire;
      j.dst += j.to_out ? o_out : o_arena;
      *d++ = j;
    }
  }
}

void relocate_piece(const Plan& b, const PieceBase& o, const FlatPlan& fp, uint8_t* blob) {
  uint8_t* dst[PS_COUNT];
  for (int s = 0; s < PS_COUNT; s++) dst[s] = blob + fp.off[s];
  relocate_into(b, o, fp.p2_g1out, false, dst);
}

}  // namespace

std::string flat_layout(const PlanWork& w, bool p2_g1out, FlatPlan& fp) {
  fp.p2_g1out = p2_g1out;
  fp.base.assign(w.used, PieceBase{});
  fp.out_off.clear();
  fp.item_off.clear();
  fp.n_items = 0;
  size_t cur[PS_COUNT] = {};
  cur[PS_ARENA] = C_SIZE;
  uint64_t pts = 0, scal = 0, g1 = 0, g2 = 0;
  for (size_t k = 0; k < w.used; k++) {
    const Plan& p = w.pieces[k];
    PieceBase& b = fp.base[k];
    cur[PS_WIRE] = (cur[PS_WIRE] + 15) & ~(size_t)15;  // keep the pieces' 16-byte alignment
    cur[PS_ARENA] = (cur[PS_ARENA] + 15) & ~(size_t)15;
    for (int s = 0; s < PS_COUNT; s++) {
      b.sec[s] = cur[s];
      cur[s] += piece_count(p, s);
    }
    b.pts = (uint32_t)pts;
    b.scal = (uint32_t)scal;
    b.g1out = (uint32_t)g1;
    b.g2out = (uint32_t)g2;
    pts += p.n_pts;
    scal += p.n_scal;
    g1 += p.n_g1out;
    g2 += p.n_g2out;
    for (uint32_t v : p.out_off) fp.out_off.push_back((uint32_t)(v + b.sec[PS_OUT]));
    for (uint32_t v : p.item_off) fp.item_off.push_back((uint32_t)(v + b.sec[PS_ARENA]));
    fp.n_items += p.tx.size();
  }
  if (!fp.out_off.empty() || cur[PS_OUT]) fp.out_off.push_back((uint32_t)cur[PS_OUT]);
  for (int s = 0; s < PS_COUNT; s++)
    if (cur[s] >= IDX_LIMIT) return "batch too large for 32-bit job indices (split it into smaller batches)";
  if (pts >= IDX_LIMIT || scal >= IDX_LIMIT || g1 >= IDX_LIMIT || g2 >= IDX_LIMIT)
    return "batch too large for 32-bit job indices (split it into smaller batches)";
  fp.n_pts = (uint32_t)pts;
  fp.n_scal = (uint32_t)scal;
  fp.n_g1out = (uint32_t)g1;
  fp.n_g2out = (uint32_t)g2;
  // device-initialised pools: ARENA and OUT go last, after the uploaded sections
  fp.dev_pools = w.used > 0;
  for (size_t k = 0; k < w.used; k++) fp.dev_pools = fp.dev_pools && w.pieces[k].dev_pools;
  int order[PS_COUNT], no = 0;
  for (int s = 0; s < PS_COUNT; s++)
    if (!fp.dev_pools || (s != PS_ARENA && s != PS_OUT)) order[no++] = s;
  if (fp.dev_pools) {
    order[no++] = PS_ARENA;
    order[no++] = PS_OUT;
  }
  size_t off = 0;
  for (int q = 0; q < PS_COUNT; q++) {
    int s = order[q];
    if (fp.dev_pools && s == PS_ARENA) fp.upload = off;
    fp.cnt[s] = cur[s];
    fp.off[s] = off;
    size_t bytes = cur[s] * elem_size(s) + (s == PS_WIRE ? WIRE_TAIL : 0);
    off = (off + bytes + SEC_ALIGN - 1) & ~(SEC_ALIGN - 1);
  }
  fp.bytes = std::max<size_t>(off, SEC_ALIGN);
  if (!fp.dev_pools) fp.upload = fp.bytes;
  return "";
}

void flat_write(const PlanWork& w, const FlatPlan& fp, uint8_t* blob, const uint8_t* const_bytes, WorkPool& pool) {
  memcpy(blob + fp.off[PS_ARENA], const_bytes, C_SIZE);
  memset(blob + fp.off[PS_WIRE] + fp.cnt[PS_WIRE], 0, WIRE_TAIL);
  pool.run(w.used, [&](size_t k) {
    const Plan& p = w.pieces[k];
    const PieceBase& b = fp.base[k];
    // zero the alignment gap in front of the piece's byte pools
    size_t prev_w = k ? fp.base[k - 1].sec[PS_WIRE] + w.pieces[k - 1].wire.size() : 0;
    size_t prev_a = k ? fp.base[k - 1].sec[PS_ARENA] + piece_count(w.pieces[k - 1], PS_ARENA) : C_SIZE;
    memset(blob + fp.off[PS_WIRE] + prev_w, 0, b.sec[PS_WIRE] - prev_w);
    memset(blob + fp.off[PS_ARENA] + prev_a, 0, b.sec[PS_ARENA] - prev_a);
    relocate_piece(p, b, fp, blob);
  });
}

PieceBase plan_append(Plan& d, const Plan& b) {
  d.wire.resize((d.wire.size() + 15) & ~(size_t)15, 0);  // the pieces' 16-byte alignment
  if (d.dev_pools)
    d.arena_len = (d.arena_len + 15) & ~(size_t)15;
  else
    d.arena.resize((d.arena.size() + 15) & ~(size_t)15, 0);
  PieceBase o;
  for (int s = 0; s < PS_COUNT; s++) o.sec[s] = piece_count(d, s);
  o.pts = d.n_pts;
  o.scal = d.n_scal;
  o.g1out = d.n_g1out;
  o.g2out = d.n_g2out;
  d.wire.resize(d.wire.size() + b.wire.size());
  if (d.dev_pools) {
    d.arena_len += b.arena.size();
    d.out_len += b.out.size();
  } else {
    d.arena.resize(d.arena.size() + b.arena.size());
    d.out.resize(d.out.size() + b.out.size());
  }
  d.dec.resize(d.dec.size() + b.dec.size());
  d.zr.resize(d.zr.size() + b.zr.size());
  d.sc.resize(d.sc.size() + b.sc.size());
  d.sclist.resize(d.sclist.size() + b.sclist.size());
  d.vt.resize(d.vt.size() + b.vt.size());
  d.g1.resize(d.g1.size() + b.g1.size());
  d.g1p.resize(d.g1p.size() + b.g1p.size());
  d.g2.resize(d.g2.size() + b.g2.size());
  d.pr.resize(d.pr.size() + b.pr.size());
  d.seg.resize(d.seg.size() + b.seg.size());
  d.hpre.resize(d.hpre.size() + b.hpre.size());
  d.hmain.resize(d.hmain.size() + b.hmain.size());
  d.ck.resize(d.ck.size() + b.ck.size());
  d.tx.resize(d.tx.size() + b.tx.size());
  d.rnd.resize(d.rnd.size() + b.rnd.size());
  d.sc1.resize(d.sc1.size() + b.sc1.size());
  d.sc_post.resize(d.sc_post.size() + b.sc_post.size());
  d.emit.resize(d.emit.size() + b.emit.size());
  d.b64.resize(d.b64.size() + b.b64.size());
  d.cp.resize(d.cp.size() + b.cp.size());
  d.cp2.resize(d.cp2.size() + b.cp2.size());
  uint8_t* dst[PS_COUNT] = {
      d.wire.data(), d.arena.data(), (uint8_t*)d.dec.data(), (uint8_t*)d.zr.data(), (uint8_t*)d.sc.data(),
      (uint8_t*)d.sclist.data(), (uint8_t*)d.vt.data(), (uint8_t*)d.g1.data(), (uint8_t*)d.g1p.data(),
      (uint8_t*)d.g2.data(), (uint8_t*)d.pr.data(), (uint8_t*)d.seg.data(), (uint8_t*)d.hpre.data(),
      (uint8_t*)d.hmain.data(), (uint8_t*)d.ck.data(), (uint8_t*)d.tx.data(), (uint8_t*)d.rnd.data(),
      (uint8_t*)d.sc1.data(), (uint8_t*)d.sc_post.data(), (uint8_t*)d.emit.data(), (uint8_t*)d.b64.data(),
      (uint8_t*)d.cp.data(), (uint8_t*)d.cp2.data(), d.out.data()};
  relocate_into(b, o, b.p2_g1out, true, dst, !d.dev_pools);
  for (uint32_t v : b.out_off) d.out_off.push_back((uint32_t)(v + o.sec[PS_OUT]));
  for (uint32_t v : b.item_off) d.item_off.push_back((uint32_t)(v + o.sec[PS_ARENA]));
  d.n_pts += b.n_pts;
  d.n_scal += b.n_scal;
  d.n_g1out += b.n_g1out;
  d.n_g2out += b.n_g2out;
  return o;
}

void plan_unflatten(const FlatPlan& fp, const uint8_t* blob, Plan& out) {
  out.clear();
  auto take = [&](auto& v, PlanSec s) {
    using T = typename std::remove_reference<decltype(v)>::type::value_type;
    const T* p = reinterpret_cast<const T*>(blob + fp.off[s]);
    v.assign(p, p + fp.cnt[s]);
  };
  take(out.wire, PS_WIRE);
  out.wire.insert(out.wire.end(), blob + fp.off[PS_WIRE] + fp.cnt[PS_WIRE],
                  blob + fp.off[PS_WIRE] + fp.cnt[PS_WIRE] + WIRE_TAIL);
  take(out.arena, PS_ARENA);
  take(out.dec, PS_DEC);
  take(out.zr, PS_ZR);
  take(out.sc, PS_SC);
  take(out.sclist, PS_SCLIST);
  take(out.vt, PS_VT);
  take(out.g1, PS_G1);
  take(out.g1p, PS_G1P);
  take(out.g2, PS_G2);
  take(out.pr, PS_PR);
  take(out.seg, PS_SEG);
  take(out.hpre, PS_HPRE);
  take(out.hmain, PS_HMAIN);
  take(out.ck, PS_CK);
  take(out.tx, PS_TX);
  take(out.rnd, PS_RND);
  take(out.sc1, PS_SC1);
  take(out.sc_post, PS_SCPOST);
  take(out.emit, PS_EMIT);
  take(out.b64, PS_B64);
  take(out.cp, PS_CP);
  take(out.cp2, PS_CP2);
  take(out.out, PS_OUT);
  out.out_off = fp.out_off;
  out.item_off = fp.item_off;
  out.p2_g1out = fp.p2_g1out;
  out.n_pts = fp.n_pts;
  out.n_scal = fp.n_scal;
  out.n_g1out = fp.n_g1out;
  out.n_g2out = fp.n_g2out;
}

// items per piece: at least 32, at most one piece per pool thread
size_t plan_piece_count(size_t n, int threads) {
  return std::max<size_t>(1, std::min<size_t>((size_t)std::max(1, threads), n / 32));
}

void plan_items(const PPInfo& pp, size_t n, const PlanItem* items, PlanWork& w, WorkPool& pool) {
  size_t np = plan_piece_count(n, pool.size());
  if (w.pieces.size() < np) w.pieces.resize(np);
  w.used = np;
  pool.run(np, [&](size_t c) {
    Plan& p = w.pieces[c];
    p.clear();
    size_t lo = n * c / np, hi = n * (c + 1) / np;
    Builder b(p, pp);
    for (size_t i = lo; i < hi; i++) {
      if (items[i].kind == 0)
        b.transfer(items[i].t);
      else if (items[i].kind == 1)
        b.issue(items[i].i);
      else
        b.opening(items[i].o);
    }
  });
}

void plan_items_merged(const PPInfo& pp, size_t n, const PlanItem* items, Plan& out, int threads) {
  WorkPool pool(threads);
  PlanWork w;
  plan_items(pp, n, items, w, pool);
  FlatPlan fp;
  flat_layout(w, false, fp);
  std::vector<uint8_t> blob(fp.bytes);
  flat_write(w, fp, blob.data(), std::vector<uint8_t>(C_SIZE, 0).data(), pool);
  plan_unflatten(fp, blob.data(), out);
}

namespace {

template <class In>
void plan_merged(const PPInfo& pp, size_t n, const In* in, Plan& out, int threads, uint8_t kind) {
  std::vector<PlanItem> items(n);
  for (size_t i = 0; i < n; i++) {
    memset(&items[i], 0, sizeof(PlanItem));
    items[i].kind = kind;
    if constexpr (std::is_same<In, TransferIn>::value)
      items[i].t = in[i];
    else
      items[i].i = in[i];
  }
  WorkPool pool(threads);
  PlanWork w;
  plan_items(pp, n, items.data(), w, pool);
  FlatPlan fp;
  flat_layout(w, false, fp);
  std::vector<uint8_t> blob(fp.bytes);
  flat_write(w, fp, blob.data(), std::vector<uint8_t>(C_SIZE, 0).data(), pool);
  plan_unflatten(fp, blob.data(), out);
}

}  // namespace

void plan_transfers(const PPInfo& pp, size_t n, const TransferIn* tx, Plan& out, int threads) {
  plan_merged(pp, n, tx, out, threads, 0);
}

void plan_issues(const PPInfo& pp, size_t n, const IssueIn* is, Plan& out, int threads) {
  plan_merged(pp, n, is, out, threads, 1);
}

// ------------------------------------------------------------------ public params
// crypto.PublicParams.Validate (setup.go:238-273, RangeProofParams.Validate
// :56-80) after Deserialize (:134-151), on the serialized bytes: "" or the
// reference's error text.  Point encodings are checked by ftz_ctx_create.
static constexpr int64_t MATHLIB_CURVES = 3;  // [EXT] len(math.Curves) at IBM/mathlib 0a7378db6912

std::string validate_pp(const uint8_t* p, size_t n, const char* label) {
  JDoc outer;
  if (!outer.parse(p, n) || outer.at(outer.root()).type != J_OBJ) return "invalid public parameters json";
  std::string ident;
  if (dec_string(outer, outer.field(outer.root(), "Identifier"), ident) == D_ERR) return "invalid identifier";
  if (ident != label) return "invalid identifier, expecting [" + std::string(label) + "], got [" + ident + "]";
  std::vector<uint8_t> raw;
  if (dec_bytes(outer, outer.field(outer.root(), "Raw"), raw) == D_ERR) return "invalid Raw";
  JDoc d;
  if (!d.parse(raw.data(), raw.size())) return "failed unmarshalling public parameters";
  go_merge(d, PP_F);
  uint32_t r = d.root();
  if (d.at(r).type == J_NULL) r = NONE;
  else if (d.at(r).type != J_OBJ) return "failed unmarshalling public parameters";
  auto fld = [&](uint32_t o, const char* k) -> int64_t { return o == NONE ? -1 : d.field(o, k); };
  auto isnull = [&](int64_t x) { return x < 0 || d.at((uint32_t)x).type == J_NULL; };
  auto arrlen = [&](int64_t x) -> int64_t {
    if (isnull(x)) return 0;
    return d.at((uint32_t)x).type == J_ARR ? (int64_t)d.len((uint32_t)x) : -1;
  };
  int64_t curve = 0, icurve = 0, prec = 0;
  std::vector<uint8_t> ipk;
  if (dec_int(d, fld(r, "Curve"), curve) == D_ERR || dec_int(d, fld(r, "IdemixCurveID"), icurve) == D_ERR ||
      dec_int(d, fld(r, "QuantityPrecision"), prec) == D_ERR || prec < 0 ||
      dec_bytes(d, fld(r, "IdemixIssuerPK"), ipk) == D_ERR)
    return "failed unmarshalling public parameters";
  const std::string P = "invalid public parameters: ", W = P + "invalid range proof parameters: ";
  if (curve > MATHLIB_CURVES - 1)
    return P + "invalid curveID [" + std::to_string(curve) + " > " + std::to_string(MATHLIB_CURVES - 1) + "]";
  if (icurve > MATHLIB_CURVES - 1)  // the reference prints pp.Curve here
    return P + "invalid idemix curveID [" + std::to_string(curve) + " > " + std::to_string(MATHLIB_CURVES - 1) + "]";
  if (isnull(fld(r, "PedGen"))) return P + "nil Pedersen generator";
  int64_t ped = fld(r, "PedParams"), np = arrlen(ped);
  if (np < 0) return "failed unmarshalling public parameters";
  if (np != 3) return P + "length mismatch in Pedersen parameters [" + std::to_string(np) + " vs. 3]";
  for (uint32_t i = 0; i < 3; i++)
    if (isnull(d.elem((uint32_t)ped, i))) return P + "nil Pedersen parameter at index " + std::to_string(i);
  int64_t rpp = fld(r, "RangeProofParams");
  if (isnull(rpp)) return P + "nil range proof parameters";
  if (d.at((uint32_t)rpp).type != J_OBJ) return "failed unmarshalling public parameters";
  int64_t spk = d.field((uint32_t)rpp, "SignPK"), sv = d.field((uint32_t)rpp, "SignedValues");
  int64_t nspk = arrlen(spk), nsv = arrlen(sv), e = 0;
  if (nspk < 0 || nsv < 0 || dec_int(d, d.field((uint32_t)rpp, "Exponent"), e) == D_ERR)
    return "failed unmarshalling public parameters";
  if (nspk != 3) return W + "signature public key should be 3, instead it is " + std::to_string(nspk);
  if (nsv < 2) return W + "signed values should be > 2";
  if (isnull(d.field((uint32_t)rpp, "Q"))) return W + "generator Q is nil";
  if (e == 0) return W + "exponent is 0";
  for (int64_t i = 0; i < nsv; i++)
    if (isnull(d.elem((uint32_t)sv, (uint32_t)i))) return W + "signed value at index " + std::to_string(i) + " is nil";
  for (int64_t i = 0; i < nspk; i++)
    if (isnull(d.elem((uint32_t)spk, (uint32_t)i))) return W + "public key at index " + std::to_string(i) + " is nil";
  if (prec != 64) return P + "quantity precision should be 64 instead it is " + std::to_string(prec);
  if (ipk.empty()) return P + "empty idemix issuer";
  return "";
}

// crypto.PublicParams.Deserialize (setup.go:134-151) + the structural subset
// of Validate (setup.go:238-273) the verifier relies on.
// every Miller line of the fixed G2 point has r0 != 0 (the normalised-line
// Miller kernels divide by it); false for a point that does not decode
static bool g2_lines_normalisable(const std::vector<uint8_t>& raw) {
  std::vector<uint8_t> b = raw;
  b.resize(std::max<size_t>(b.size(), 128) + 64, 0);
  G2Dev d;
  if (!decode_g2(b.data(), 128, d, nullptr)) return false;
  g2a q = g2_load(d);
  if (q.inf) return false;
  std::vector<LineCoef> l(MILLER_LINES);
  int n = precompute_lines(l.data(), q);
  for (int i = 0; i < n; i++)
    if (f2_is_zero(l[i].r0)) return false;
  return n == MILLER_LINES;
}

bool pp_sig_tables(const PPInfo& pp) {
  if (pp.no_sigtab || pp.base == 0 || pp.base > G1B_SIG_MAX_DIGITS || pp.sig_r.size() != pp.base || pp.sig_s.size() != pp.base)
    return false;
  auto zero = [](const std::vector<uint8_t>& v) {
    for (uint8_t b : v)
      if (b) return false;
    return true;
  };
  for (uint32_t d = 0; d < pp.base; d++)
    if (zero(pp.sig_r[d]) || zero(pp.sig_s[d])) return false;
  return true;
}

size_t proof_challenge_slots(const TxChecks& t, const Check* ck, const HashJob* hmain, int32_t* kinds,
                             uint32_t* slots, size_t cap) {
  size_t m = 0;
  auto part = [&](uint32_t start, uint32_t count) {
    for (uint32_t k = 0; k < count; k++) {
      const Check& c = ck[start + k];
      if (c.kind != CK_HASH) continue;
      if (m < cap) {
        kinds[m] = c.code;
        slots[m] = hmain[c.a].out_scal;
      }
      m++;
    }
  };
  part(t.wf_start, t.wf_count);
  part(t.rg_start, t.rg_count);
  return m;
}

// Go math.Pow (src/math/pow.go, go1.18; amd64 runs this pure-Go path) for an
// integer exponent: yf = 0, so ans = Ldexp(a1, ae) with a1 the product of the
// mantissas x1^(2^k) of the set bits of n, each squared mantissa renormalised
// to [0.5, 1).  Each step is one IEEE multiply or add; contraction into an FMA
// would change the rounding, so it is off here.
double go_pow_int(double x, int64_t n) {
#pragma clang fp contract(off)
  if (n == 0 || x == 1.0) return 1.0;
  if (n == 1) return x;
  double a1 = 1.0;
  int64_t ae = 0;
  int xe_i = 0;
  double x1 = frexp(x, &xe_i);
  int64_t xe = xe_i;
  for (int64_t i = n; i != 0; i >>= 1) {
    if (xe < -(1 << 12) || (1 << 12) < xe) {  // catastrophic overflow: Ldexp handles it
      ae += xe;
      break;
    }
    if (i & 1) {
      a1 *= x1;
      ae += xe;
    }
    x1 *= x1;
    xe <<= 1;
    if (x1 < .5) {
      x1 += x1;
      xe--;
    }
  }
  if (ae > 4096) return HUGE_VAL;  // Go's Ldexp overflows to +Inf (a1 in (0, 1])
  return ldexp(a1, (int)ae);
}

// int64(f) on amd64 (CVTTSD2SQ): truncation when representable, else the
// "integer indefinite" 0x8000000000000000.  [EXT] the Go spec leaves the
// out-of-range result implementation-defined.
int64_t go_int64(double f) {
  if (!(f >= -9223372036854775808.0 && f < 9223372036854775808.0)) return INT64_MIN;
  return (int64_t)f;
}

int64_t digit_weight(uint32_t base, int64_t i) { return go_int64(go_pow_int((double)base, i)); }

int prover_digits(const PPInfo& pp, const uint8_t* be32, uint32_t* digits) {
  const int64_t e = pp.exponent;
  const uint32_t b = pp.base;
  if (e <= 0 || b < 2 || pp.pow.size() != (size_t)e) return 1;
  for (int k = 0; k < 24; k++)
    if (be32[k]) return 1;
  uint64_t u = 0;
  for (int k = 24; k < 32; k++) u = (u << 8) | be32[k];
  if (pp.pow_top == INT64_MIN) {
    // [EXT] the reference refuses every value here; exact digits of v < b^e,
    // valid for its verifier when every weight below e is b^i
    if (!pp.pow_exact) return 1;
    unsigned __int128 bound = 1;
    for (int64_t i = 0; i < e && bound <= ((unsigned __int128)1 << 64); i++) bound *= b;
    if ((unsigned __int128)u >= bound) return 1;
    for (int64_t i = 0; i < e; i++) {
      digits[i] = (uint32_t)(u % b);
      u /= b;
    }
    return 0;
  }
  // Value.Int() (range/proof.go:299) fails above int64; then v >= int64(math.Pow(b, e)) (:303)
  if (u >> 63 || (int64_t)u >= pp.pow_top) return 1;
  int64_t v = (int64_t)u;
  digits[0] = (uint32_t)(v % (int64_t)b);  // values[0] = v % Base on the original v (:307)
  for (int64_t i = 0; i < e - 1; i++) {    // quotient / remainder by w_(e-1-i) (:308-311)
    const int64_t w = (int64_t)pp.pow[e - 1 - i];
    const int64_t q = v / w;
    v = v % w;
    if (q < 0 || q >= (int64_t)b) return 2;  // Signatures[values[i]] out of range (:326)
    digits[e - 1 - i] = (uint32_t)q;
  }
  return 0;
}

std::string parse_pp(const uint8_t* p, size_t n, const char* label, PPInfo& out) {
  JDoc outer;
  if (!outer.parse(p, n)) return "invalid public parameters json";
  uint32_t root = outer.root();
  if (outer.at(root).type != J_OBJ) return "invalid public parameters json";
  std::string ident;
  if (dec_string(outer, outer.field(root, "Identifier"), ident) == D_ERR) return "invalid identifier";
  if (ident != label) return "invalid identifier, expecting [" + std::string(label) + "], got [" + ident + "]";
  std::vector<uint8_t> raw;
  if (dec_bytes(outer, outer.field(root, "Raw"), raw) != D_OK) return "missing Raw";
  JDoc d;
  if (!d.parse(raw.data(), raw.size())) return "failed unmarshalling public parameters";
  go_merge(d, PP_F);
  uint32_t r = d.root();
  if (d.at(r).type != J_OBJ) return "failed unmarshalling public parameters";
  out.label = ident;
  if (dec_int(d, d.field(r, "Curve"), out.curve) == D_ERR) return "bad Curve";
  if (out.curve != 1) return "zkatdlog public parameters must use BN254 (curve 1)";
  auto el = [&](int64_t node, std::vector<uint8_t>& o) -> bool {
    ElemBytes e = dec_elem(d, node);
    if (e.st != D_OK) return false;
    o = e.raw;
    return true;
  };
  if (!el(d.field(r, "PedGen"), out.pedgen)) return "invalid public parameters: nil Pedersen generator";
  int64_t pedp = d.field(r, "PedParams");
  if (pedp < 0 || d.at((uint32_t)pedp).type != J_ARR || d.len((uint32_t)pedp) != 3)
    return "invalid public parameters: length mismatch in Pedersen parameters";
  for (int k = 0; k < 3; k++)
    if (!el(d.elem((uint32_t)pedp, k), out.ped[k])) return "invalid public parameters: nil Pedersen parameter";
  int64_t rpp = d.field(r, "RangeProofParams");
  if (rpp < 0 || d.at((uint32_t)rpp).type != J_OBJ) return "invalid public parameters: nil range proof parameters";
  int64_t spk = d.field((uint32_t)rpp, "SignPK");
  if (spk < 0 || d.at((uint32_t)spk).type != J_ARR || d.len((uint32_t)spk) != 3)
    return "invalid range proof parameters: signature public key should be 3";
  for (int k = 0; k < 3; k++)
    if (!el(d.elem((uint32_t)spk, k), out.pk[k])) return "invalid range proof parameters: nil public key";
  if (!el(d.field((uint32_t)rpp, "Q"), out.q)) return "invalid range proof parameters: generator Q is nil";
  // RangeProofParams.Validate (setup.go:66-68) refuses only 0; a negative
  // exponent is a PP on which every range proof is "not well formed"
  // (range/proof.go:424-426).  Above MAX_EXPONENT the context is refused.
  if (dec_int(d, d.field((uint32_t)rpp, "Exponent"), out.exponent) != D_OK || out.exponent == 0 ||
      out.exponent > MAX_EXPONENT)
    return "invalid range proof parameters: exponent";
  int64_t sv = d.field((uint32_t)rpp, "SignedValues");
  if (sv < 0 || d.at((uint32_t)sv).type != J_ARR || d.len((uint32_t)sv) < 2)
    return "invalid range proof parameters: signed values should be > 2";
  out.base = d.len((uint32_t)sv);
  out.sig_r.resize(out.base);
  out.sig_s.resize(out.base);
  for (uint32_t k = 0; k < out.base; k++) {
    uint32_t s = d.elem((uint32_t)sv, k);
    if (d.at(s).type != J_OBJ) return "invalid range proof parameters: signed value is nil";
    if (!el(d.field(s, "R"), out.sig_r[k]) || !el(d.field(s, "S"), out.sig_s[k]))
      return "invalid range proof parameters: signed value is nil";
  }
  // digit weights int64(math.Pow(float64(Base), float64(i))) (range/proof.go:428)
  out.pow.clear();
  for (int64_t i = 0; i < out.exponent; i++) out.pow.push_back((uint64_t)digit_weight(out.base, i));
  out.pow_top = digit_weight(out.base, out.exponent > 0 ? out.exponent : 0);
  // the Horner form of sum_i pow[i] com_i needs pow[i] == base^i exactly
  out.pow_exact = out.exponent > 0;
  unsigned __int128 bi = 1;
  for (size_t i = 0; i < out.pow.size(); i++) {
    if (i) bi *= out.base;
    if (bi >> 63 || (uint64_t)bi != out.pow[i]) out.pow_exact = false;
    if (bi >> 63) break;
  }
  out.fixed_pairs = pp_sig_tables(out) && g2_lines_normalisable(out.q) && g2_lines_normalisable(out.pk[1]) &&
                    g2_lines_normalisable(out.pk[2]);
  return "";
}

}  // namespace ftsh

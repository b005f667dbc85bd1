// Host planner: restates the *control flow* of the reference verifiers (which
// checks run, in which order, and which error class each failure produces) and
// compiles the arithmetic into GPU jobs.  Reference (paths under
// token/core/zkatdlog/crypto/):
//   transfer.Verifier.Verify             transfer/transfer.go:124-154
//   WellFormednessVerifier.Verify        transfer/wellformedness.go:311-394
//   rangeproof.Verifier.Verify           range/proof.go:211-284, 393-444
//   MembershipVerifier.Verify            sigproof/membership.go:162-180, 260-305
//   POKVerifier.recomputeCommitment      sigproof/pok.go:160-204
//   issue.Verifier.Verify                issue/issue.go:202-223
//   issue WellFormednessVerifier.Verify  issue/wellformedness.go:206-265
// No group, field or hash arithmetic happens here: every value is produced on
// the GPU.  The planner only parses bytes (JSON, base64) and lays out jobs.
#include "planner.h"

#include <string.h>

#include <algorithm>
#include <thread>

#include "gojson.h"

namespace ftsh {

void Plan::clear() {
  rnd.clear();
  sc1.clear();
  sc_post.clear();
  emit.clear();
  b64.clear();
  out.clear();
  out_off.clear();
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
struct Doc {
  JDoc d;
  bool ok = false;
  bool panic = false;
  bool err = false;
  Plan* pl;

  explicit Doc(Plan* p) : pl(p) {}

  bool parse(const std::vector<uint8_t>& b, bool nil) {
    if (nil) return ok = false;  // json.Unmarshal(nil) -> "unexpected end of JSON input"
    ok = d.parse(b.data(), b.size());
    return ok;
  }

  Ref elem(int64_t node) {
    Ref r;
    if (node < 0 || d.at((uint32_t)node).type == J_NULL) return r;
    ElemBytes e = dec_elem(d, node);
    if (e.st == D_ERR) {
      err = true;
      return r;
    }
    if (e.st == D_PANIC) {
      panic = true;
      return r;
    }
    if (e.raw.size() > ZR_MAX_LEN) {  // beyond the device decoder's range
      err = true;
      return r;
    }
    pl->wire.resize((pl->wire.size() + 15) & ~(size_t)15, 0);  // 16-byte aligned element (vector loads)
    r.off = (int64_t)pl->wire.size();
    r.len = (uint32_t)e.raw.size();
    pl->wire.insert(pl->wire.end(), e.raw.begin(), e.raw.end());
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

 private:
  Plan& pl;
  const PPInfo& pp;
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
  static VTerm vterm(uint32_t pt, uint64_t w = 1) {
    VTerm v;
    v.pt = pt;
    v.w_lo = (uint32_t)w;
    v.w_hi = (uint32_t)(w >> 32);
    v.pad = 0;
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
};

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
// parseProof (wellformedness.go:354-394) + RecomputeCommitments (common/schnorr.go:106-118).
bool Builder::wf_side(uint32_t tok_pt, uint32_t n, const std::vector<Ref>& vals, const std::vector<Ref>& bfs,
                      const Ref& type, const Ref& sum, const Ref& chal, uint32_t& s_type, uint32_t& s_sum,
                      uint32_t& s_chal, uint32_t wfout_bytes) {
  if (vals.size() != n || bfs.size() != n) {
    fail(E_MALFORMED);
    return false;
  }
  if (type.nil()) {  // ModMul(ttype, n) dereferences nil (wellformedness.go:381)
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
  Doc doc(&pl);
  if (!doc.parse(rc, rc_nil)) {
    fail(E_PARSE);
    return;
  }
  RangeDoc r;
  size_t wire_mark = pl.wire.size();
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
      // POKVerifier.recomputeCommitment (pok.go:465-509)
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
      pl.pr.push_back({p1, d.R, g2.out, d.slot + 128});
      HashJob h;
      h.seg_start = (uint32_t)pl.seg.size();
      seg(CONST_FLAG | C_PED0, 128);
      seg(d.slot, 128);
      seg(CONST_FLAG | C_PEDGEN, 64);
      seg(CONST_FLAG | C_PK_Q, 512);
      seg(d.slot + 128, 384 + SIG_JSON_LEN);
      h.seg_count = 5;
      h.expect = sc_ch;
      h.out_scal = NONE;
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
    if (r.mps[j].coms.size() != e || r.eq_cbf[j].nil()) {
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
    for (uint32_t i = 0; i < e; i++) terms.push_back(vterm(com_pt[j][i], pp.pow[i]));
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
  h.out_scal = NONE;
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
  std::vector<uint8_t> wfb, rcb;
  bool wf_nil = true, rc_nil = true;
  {
    JDoc top;
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
  // WellFormednessVerifier.Verify (wellformedness.go:311-351)
  {
    Doc doc(&pl);
    if (!doc.parse(wfb, wf_nil)) {
      fail(E_PARSE);
    } else {
      size_t mark = pl.wire.size();
      int64_t top = doc.top();
      std::vector<Ref> ibf = doc.list(doc.f(top, "InputBlindingFactors"));
      std::vector<Ref> obf = doc.list(doc.f(top, "OutputBlindingFactors"));
      std::vector<Ref> ivl = doc.list(doc.f(top, "InputValues"));
      std::vector<Ref> ovl = doc.list(doc.f(top, "OutputValues"));
      Ref type = doc.elem(doc.f(top, "Type"));
      Ref sum = doc.elem(doc.f(top, "Sum"));
      Ref chal = doc.elem(doc.f(top, "Challenge"));
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
          h.out_scal = NONE;
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

void Builder::issue(const IssueIn& t) {
  begin_tx(1);
  uint32_t tok_bytes;
  uint32_t tok_pt = tokens(t.outputs, t.n_out, tok_bytes);
  if (t.n_out) check(CK_PTS, E_PARSE, tok_pt, t.n_out);
  uint32_t n = t.n_out;
  std::vector<uint8_t> wfb, rcb;
  bool wf_nil = true, rc_nil = true;
  {
    JDoc top;
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
  // issue WellFormednessVerifier.Verify (issue/wellformedness.go:206-265)
  Doc doc(&pl);
  if (!doc.parse(wfb, wf_nil)) {
    fail(E_PARSE);
    end_tx();
    return;
  }
  size_t mark = pl.wire.size();
  int64_t top = doc.top();
  Ref type = doc.elem(doc.f(top, "Type"));
  std::vector<Ref> vals = doc.list(doc.f(top, "Values"));
  std::vector<Ref> bfs = doc.list(doc.f(top, "BlindingFactors"));
  std::string clear;
  DecStatus cs = dec_string(doc.d, doc.f(top, "TypeInTheClear"), clear);
  if (cs == D_ERR) doc.err = true;
  Ref chal = doc.elem(doc.f(top, "Challenge"));
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
  h.out_scal = NONE;
  pl.hmain.push_back(h);
  check(CK_HASH, E_WF, (uint32_t)pl.hmain.size() - 1);
  range_part(rcb, rc_nil, tok_pt, tok_bytes, n);
  end_tx();
}

}  // namespace

// Append piece `b` (local indices) to plan `a`, relocating every index.
void plan_merge(Plan& a, const Plan& b) {
  a.arena.resize((a.arena.size() + 15) & ~(size_t)15, 0);  // keep the pieces' 16-byte alignment
  a.wire.resize((a.wire.size() + 15) & ~(size_t)15, 0);
  uint32_t o_wire = (uint32_t)a.wire.size(), o_arena = (uint32_t)a.arena.size();
  uint32_t o_pts = a.n_pts, o_scal = a.n_scal, o_g1 = a.n_g1out, o_g2 = a.n_g2out;
  uint32_t o_list = (uint32_t)a.sclist.size(), o_vt = (uint32_t)a.vt.size(), o_seg = (uint32_t)a.seg.size();
  uint32_t o_hmain = (uint32_t)a.hmain.size(), o_ck = (uint32_t)a.ck.size();
  auto rel = [](uint32_t v, uint32_t o) { return v == NONE ? NONE : v + o; };
  a.wire.insert(a.wire.end(), b.wire.begin(), b.wire.end());
  a.arena.insert(a.arena.end(), b.arena.begin(), b.arena.end());
  for (DecodeJob j : b.dec) {
    j.raw += o_wire;
    j.out += o_pts;
    j.bytes = rel(j.bytes, o_arena);
    j.b64 = rel(j.b64, o_arena);
    a.dec.push_back(j);
  }
  for (ZrJob j : b.zr) {
    j.raw += o_wire;
    j.out += o_scal;
    a.zr.push_back(j);
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
  for (const ScalJob& j : b.sc) a.sc.push_back(rel_sc(j));
  for (const ScalJob& j : b.sc1) a.sc1.push_back(rel_sc(j));
  for (const ScalJob& j : b.sc_post) a.sc_post.push_back(rel_sc(j));
  for (uint32_t v : b.sclist) a.sclist.push_back(v + o_scal);
  for (VTerm v : b.vt) {
    v.pt += o_pts;
    a.vt.push_back(v);
  }
  for (int side = 0; side < 2; side++) {
    for (G1Job j : (side ? b.g1p : b.g1)) {
      for (int k = 0; k < j.nfix; k++) j.fscal[k] += o_scal;
      j.vstart += o_vt;
      j.vscal = rel(j.vscal, o_scal);
      j.out += o_g1;
      j.bytes = rel(j.bytes, o_arena);
      j.b64 = rel(j.b64, o_arena);
      (side ? a.g1p : a.g1).push_back(j);
    }
  }
  for (G2Job j : b.g2) {
    for (int k = 0; k < j.nfix; k++) j.fscal[k] += o_scal;
    j.out += o_g2;
    a.g2.push_back(j);
  }
  for (PairJob j : b.pr) {
    j.p1 += o_g1;
    j.p2 += a.p2_g1out ? o_g1 : o_pts;
    j.q2 += o_g2;
    j.bytes += o_arena;
    a.pr.push_back(j);
  }
  for (Seg s : b.seg) {
    if (s.off & CONST_FLAG)
      s.off &= ~CONST_FLAG;  // const region sits at absolute offset 0
    else
      s.off += o_arena;
    a.seg.push_back(s);
  }
  for (HashJob h : b.hpre) {
    h.seg_start += o_seg;
    h.expect = rel(h.expect, o_scal);
    h.out_scal = rel(h.out_scal, o_scal);
    a.hpre.push_back(h);
  }
  for (HashJob h : b.hmain) {
    h.seg_start += o_seg;
    h.expect = rel(h.expect, o_scal);
    h.out_scal = rel(h.out_scal, o_scal);
    a.hmain.push_back(h);
  }
  for (Check c : b.ck) {
    if (c.kind == CK_PTS) c.a += o_pts;
    if (c.kind == CK_HASH) c.a += o_hmain;
    a.ck.push_back(c);
  }
  for (TxChecks t : b.tx) {
    t.wf_start += o_ck;
    t.rg_start += o_ck;
    a.tx.push_back(t);
  }
  // prover pieces
  for (RandJob j : b.rnd) {
    j.seed += o_arena;
    j.tag += o_arena;
    j.out += o_scal;
    a.rnd.push_back(j);
  }
  for (EmitJob j : b.emit) {
    j.dst += o_arena;
    j.src += j.kind == EM_ZR ? o_scal : o_arena;
    a.emit.push_back(j);
  }
  uint32_t o_out = (uint32_t)a.out.size();
  for (B64Job j : b.b64) {
    j.src += o_arena;
    j.dst += o_out;
    a.b64.push_back(j);
  }
  a.out.insert(a.out.end(), b.out.begin(), b.out.end());
  for (uint32_t v : b.out_off) a.out_off.push_back(v + o_out);
  a.n_pts += b.n_pts;
  a.n_scal += b.n_scal;
  a.n_g1out += b.n_g1out;
  a.n_g2out += b.n_g2out;
}

namespace {

template <class In, class Fn>
void plan_batch(const PPInfo& pp, size_t n, const In* in, Plan& out, int threads, Fn fn) {
  out.clear();
  out.arena.resize(C_SIZE, 0);
  if (threads < 1) threads = 1;
  size_t chunks = std::min<size_t>((size_t)threads, std::max<size_t>(1, n / 64));
  std::vector<Plan> pieces(chunks);
  std::vector<std::thread> th;
  for (size_t c = 0; c < chunks; c++) {
    size_t lo = n * c / chunks, hi = n * (c + 1) / chunks;
    th.emplace_back([&, c, lo, hi]() {
      Builder b(pieces[c], pp);
      for (size_t i = lo; i < hi; i++) fn(b, in[i]);
    });
  }
  for (auto& t : th) t.join();
  for (auto& p : pieces) plan_merge(out, p);
}

}  // namespace

void plan_transfers(const PPInfo& pp, size_t n, const TransferIn* tx, Plan& out, int threads) {
  plan_batch(pp, n, tx, out, threads, [](Builder& b, const TransferIn& t) { b.transfer(t); });
}

void plan_issues(const PPInfo& pp, size_t n, const IssueIn* is, Plan& out, int threads) {
  plan_batch(pp, n, is, out, threads, [](Builder& b, const IssueIn& t) { b.issue(t); });
}

// ------------------------------------------------------------------ public params
// crypto.PublicParams.Deserialize (setup.go:350-367) + the structural subset
// of Validate (setup.go:454-489) the verifier relies on.
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
  if (dec_int(d, d.field((uint32_t)rpp, "Exponent"), out.exponent) != D_OK || out.exponent <= 0 ||
      out.exponent > 64)
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
  // digit weights base^i (range/proof.go:428: int64(math.Pow(float64(base), i)))
  out.pow.clear();
  long double acc = 1;
  for (int64_t i = 0; i < out.exponent; i++) {
    double pw = 1.0;
    for (int64_t k = 0; k < i; k++) pw *= (double)out.base;  // float64 math.Pow is exact below 2^53
    (void)acc;
    if (pw >= 9223372036854775808.0) return "range proof exponent overflows int64";
    out.pow.push_back((uint64_t)(int64_t)pw);
  }
  return "";
}

}  // namespace ftsh

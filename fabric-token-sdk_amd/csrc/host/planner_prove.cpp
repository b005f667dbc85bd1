// Host planner of the batch PROVER: lays out, per transfer / issue, the GPU
// jobs that compute a zkatdlog proof and the JSON templates the device fills.
// Reference (paths under token/core/zkatdlog/crypto/):
//   transfer.Prover.Prove                 transfer/transfer.go:89-121
//   transfer WellFormednessProver         transfer/wellformedness.go:131-154, 243-378
//   rangeproof.Prover.Prove               range/proof.go:141-209, preProcess :288-337,
//                                         computeCommitment :340-368
//   MembershipProver.Prove                sigproof/membership.go:112-158,
//                                         obfuscateSignature :196-222, computeCommitment :225-257
//   issue.Prover.Prove / WF prover        issue/issue.go:151-184; issue/wellformedness.go:74-184
//   token commitments                     token/token.go:64-98
// Randomness: the reference draws every blinding value from crypto/rand.  The
// batch prover derives them from a per-proof 32-byte seed and a tag naming the
// value, rand(tag) = SHA-256(seed||tag||0) || SHA-256(seed||tag||1) mod r, the
// same derivation as the oracle's prover (ftsoracle/zkat.py Rand), so proofs
// are reproducible and checkable byte for byte.  The Go shim passes 32 bytes
// of crypto/rand per proof as the seed.
//
// No arithmetic happens here: the planner writes tag strings, witness bytes and
// JSON templates into the arena and emits jobs; every scalar, point, GT element,
// hash and base64 character of the proof is produced on the GPU.
#include <stdio.h>
#include <string.h>

#include <string>
#include <thread>
#include <vector>

#include "planner.h"

namespace ftsh {
namespace {

static const char ZR_PRE[] = "{\"curve\":1,\"element\":\"";  // mathlib curveElement JSON, BN254
static const char EL_END[] = "\"}";
static constexpr uint32_t SIG_JSON_LEN = 27 + 88 + 29 + 88 + 3;
static const char SIG_JSON_R[] = "{\"R\":{\"curve\":1,\"element\":\"";
static const char SIG_JSON_S[] = "\"},\"S\":{\"curve\":1,\"element\":\"";
static const char SIG_JSON_E[] = "\"}}";

// Go encoding/json string encoding (HTML-safe escaping of <, >, &, U+2028/9).
std::string go_json_str(const char* s, size_t n) {
  std::string o = "\"";
  static const char* hex = "0123456789abcdef";
  for (size_t i = 0; i < n; i++) {
    unsigned char c = (unsigned char)s[i];
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      case '\b': o += "\\b"; break;
      case '\f': o += "\\f"; break;
      case '<': o += "\\u003c"; break;
      case '>': o += "\\u003e"; break;
      case '&': o += "\\u0026"; break;
      default:
        if (c < 0x20) {
          o += "\\u00";
          o += hex[c >> 4];
          o += hex[c & 15];
        } else if (c == 0xE2 && i + 2 < n && (unsigned char)s[i + 1] == 0x80 &&
                   ((unsigned char)s[i + 2] == 0xA8 || (unsigned char)s[i + 2] == 0xA9)) {
          o += (unsigned char)s[i + 2] == 0xA8 ? "\\u2028" : "\\u2029";
          i += 2;
        } else {
          o += (char)c;
        }
    }
  }
  return o + "\"";
}

// Witness-dependent bytes of a planned proof (ProofTpl): everything else a
// proof's plan holds -- jobs, tags, JSON templates, arena layout -- depends only
// on its shape.  Digit sources index k * e + i (token k, digit i).
enum SrcKind : uint8_t {
  SRC_SEED, SRC_IN_PT, SRC_OUT_PT, SRC_IN_VAL, SRC_IN_BF, SRC_OUT_VAL, SRC_OUT_BF, SRC_TYPE,
  SRC_SIG_R, SRC_SIG_S, SRC_DIGIT, SRC_NONE = 0xFF
};
struct Patch {
  uint8_t arena;  // 1: arena byte offset, 0: wire
  uint8_t kind;   // SrcKind
  uint16_t k;
  uint32_t off, len;
};
// ... and the digit-dependent fixed base of a G1 job (the signature point
// table of digit k: R_d for s == 0, S_d for s == 1)
struct BasePatch {
  uint8_t g1p;   // 1: pl.g1p, 0: pl.g1
  uint8_t slot;  // fbase slot
  uint8_t s;
  uint16_t k;
  uint32_t job;  // template-local job index
};

struct PB {
  Plan& pl;
  const PPInfo& pp;
  uint32_t seed_off = 0;
  std::string tagp;  // tag prefix
  std::string err;
  std::vector<Patch>* rec = nullptr;  // template build: where the witness bytes go
  std::vector<BasePatch>* brec = nullptr;
  const bool sigtab;                   // digit signature points through fixed-base tables
  PB(Plan& p, const PPInfo& q) : pl(p), pp(q), sigtab(pp_sig_tables(q)) {}
  void note_base(bool g1p, uint8_t slot, uint8_t s, uint32_t k) {
    if (brec) brec->push_back({(uint8_t)(g1p ? 1 : 0), slot, s, (uint16_t)k, (uint32_t)((g1p ? pl.g1p : pl.g1).size() - 1)});
  }
  void note(bool arena, uint8_t kind, uint32_t k, uint32_t off, uint32_t len) {
    if (rec && kind != SRC_NONE) rec->push_back({(uint8_t)(arena ? 1 : 0), kind, (uint16_t)k, off, len});
  }
  uint32_t arena_data(const void* p, size_t n, uint8_t kind, uint32_t k = 0) {
    uint32_t off = arena_put(p, n);
    note(true, kind, k, off, (uint32_t)n);
    return off;
  }

  // 16-byte aligned allocations (the device SHA-256 streams aligned whole blocks)
  uint32_t arena_alloc(uint32_t n) {
    uint32_t off = (uint32_t)((pl.arena.size() + 15) & ~(size_t)15);
    pl.arena.resize(off + n, 0);
    return off;
  }
  uint32_t arena_put(const void* p, size_t n) {
    uint32_t off = arena_alloc((uint32_t)n);
    if (n) memcpy(pl.arena.data() + off, p, n);
    return off;
  }
  uint32_t seg(uint32_t off, uint32_t len) {
    pl.seg.push_back({off, len});
    return (uint32_t)pl.seg.size() - 1;
  }
  uint32_t rnd(const std::string& tag) {
    RandJob j;
    j.seed = seed_off;
    j.tag = arena_alloc((uint32_t)(tagp.size() + tag.size()));
    memcpy(pl.arena.data() + j.tag, tagp.data(), tagp.size());
    memcpy(pl.arena.data() + j.tag + tagp.size(), tag.data(), tag.size());
    j.len = (uint32_t)(tagp.size() + tag.size());
    j.out = pl.n_scal++;
    pl.rnd.push_back(j);
    return j.out;
  }
  // 32-byte big-endian scalar from the wire (mod r)
  uint32_t zr32(const uint8_t* b, uint8_t kind = SRC_NONE, uint32_t k = 0) {
    ZrJob j;
    pl.wire.resize((pl.wire.size() + 15) & ~(size_t)15, 0);
    j.raw = (uint32_t)pl.wire.size();
    note(false, kind, k, j.raw, 32);
    pl.wire.insert(pl.wire.end(), b, b + 32);
    j.len = 32;
    j.out = pl.n_scal++;
    pl.zr.push_back(j);
    return j.out;
  }
  uint32_t zr_u64(uint64_t v, uint8_t kind = SRC_NONE, uint32_t k = 0) {
    uint8_t b[32] = {0};
    for (int q = 0; q < 8; q++) b[31 - q] = (uint8_t)(v >> (8 * q));
    return zr32(b, kind, k);
  }
  // HashToZr of an arena range (before the group work)
  uint32_t hash_pre(uint32_t off, uint32_t len) {
    HashJob h;
    h.seg_start = (uint32_t)pl.seg.size();
    seg(off, len);
    h.seg_count = 1;
    h.expect = NONE;
    h.out_scal = pl.n_scal++;
    pl.hpre.push_back(h);
    return h.out_scal;
  }
  uint32_t challenge(std::initializer_list<std::pair<uint32_t, uint32_t>> segs) {
    HashJob h;
    h.seg_start = (uint32_t)pl.seg.size();
    for (auto& s : segs) seg(s.first, s.second);
    h.seg_count = (uint32_t)segs.size();
    h.expect = NONE;
    h.out_scal = pl.n_scal++;
    pl.hmain.push_back(h);
    return h.out_scal;
  }
  uint32_t sc(uint32_t op, uint32_t a, uint32_t b, uint32_t c = 0) {
    uint32_t o = pl.n_scal++;
    pl.sc.push_back({op, a, b, o, c});
    return o;
  }
  // level 1: the summands are outputs of level-0 scalar jobs (k_scalar runs
  // one lane per job, so dependent jobs go to a second launch)
  uint32_t sum(const std::vector<uint32_t>& v, bool level1 = false) {
    uint32_t o = pl.n_scal++;
    (level1 ? pl.sc1 : pl.sc).push_back({SOP_SUM, (uint32_t)pl.sclist.size(), (uint32_t)v.size(), o, 0});
    pl.sclist.insert(pl.sclist.end(), v.begin(), v.end());
    return o;
  }
  // response r + c*w (after the challenge hash)
  uint32_t resp(uint32_t r, uint32_t c, uint32_t w) {
    uint32_t o = pl.n_scal++;
    pl.sc_post.push_back({SOP_MADD, r, c, o, w});
    return o;
  }
  uint32_t point(const uint8_t* raw, uint32_t len, uint32_t bytes, uint8_t kind = SRC_NONE, uint32_t k = 0) {
    DecodeJob j;
    pl.wire.resize((pl.wire.size() + 15) & ~(size_t)15, 0);
    j.raw = (uint32_t)pl.wire.size();
    note(false, kind, k, j.raw, len);
    pl.wire.insert(pl.wire.end(), raw, raw + len);
    j.len = len;
    j.out = pl.n_pts++;
    j.bytes = bytes;
    j.b64 = NONE;
    pl.dec.push_back(j);
    return j.out;
  }
  uint32_t g1job(std::initializer_list<std::pair<uint8_t, uint32_t>> fixed, uint32_t var_pt, uint32_t vscal,
                 uint32_t bytes, uint32_t b64, bool feeds_pairing) {
    G1Job j;
    memset(&j, 0, sizeof(j));
    for (auto& f : fixed) {
      j.fbase[j.nfix] = f.first;
      j.fscal[j.nfix] = f.second;
      j.nfix++;
    }
    j.vstart = (uint32_t)pl.vt.size();
    j.vcount = 0;
    j.vscal = NONE;
    if (var_pt != NONE) {
      VTerm v;
      v.pt = var_pt;
      v.w_lo = 1;
      v.w_hi = 0;
      v.flags = 0;
      pl.vt.push_back(v);
      j.vcount = 1;
      j.vscal = vscal;
    }
    j.vneg = 0;
    j.out = pl.n_g1out++;
    j.bytes = bytes;
    j.b64 = b64;
    (feeds_pairing ? pl.g1p : pl.g1).push_back(j);
    return j.out;
  }

  // ---- JSON template writer: literal text plus fixed-length base64 holes
  std::string doc;
  struct Hole {
    uint32_t pos, kind, src;
  };
  std::vector<Hole> holes;
  void lit(const char* s) { doc += s; }
  void zr(uint32_t scal) {
    doc += ZR_PRE;
    holes.push_back({(uint32_t)doc.size(), EM_ZR, scal});
    doc.append(44, '=');
    doc += EL_END;
  }
  void g1(uint32_t bytes_off) {
    doc += ZR_PRE;
    holes.push_back({(uint32_t)doc.size(), EM_G1, bytes_off});
    doc.append(88, '=');
    doc += EL_END;
  }
  void zr_list(const std::vector<uint32_t>& v) {
    lit("[");
    for (size_t i = 0; i < v.size(); i++) {
      if (i) lit(",");
      zr(v[i]);
    }
    lit("]");
  }
  // move the document into the arena; returns (offset, length)
  std::pair<uint32_t, uint32_t> flush_doc() {
    uint32_t off = arena_put(doc.data(), doc.size());
    for (auto& h : holes) pl.emit.push_back({off + h.pos, h.kind, h.src});
    std::pair<uint32_t, uint32_t> r(off, (uint32_t)doc.size());
    doc.clear();
    holes.clear();
    return r;
  }

  // outer proof {"WellFormedness":b64,"RangeCorrectness":b64|null}
  void outer(std::pair<uint32_t, uint32_t> wf, bool has_rc, std::pair<uint32_t, uint32_t> rc) {
    pl.out_off.push_back((uint32_t)pl.out.size());
    auto put = [&](const char* s) { pl.out.insert(pl.out.end(), s, s + strlen(s)); };
    auto b64 = [&](std::pair<uint32_t, uint32_t> d) {
      put("\"");
      pl.b64.push_back({d.first, d.second, (uint32_t)pl.out.size()});
      pl.out.resize(pl.out.size() + 4 * ((d.second + 2) / 3), '=');
      put("\"");
    };
    put("{\"WellFormedness\":");
    b64(wf);
    put(",\"RangeCorrectness\":");
    if (has_rc)
      b64(rc);
    else
      put("null");
    put("}");
  }

  // rangeproof.Prover.Prove over tokens (output commitments at tok_bytes);
  // v[k], bf[k] witness scalars, vals[k] the integer values, h_type HashToZr(type)
  std::pair<uint32_t, uint32_t> range(uint32_t tok_bytes, uint32_t n, const std::vector<uint32_t>& v,
                                      const std::vector<uint32_t>& bf, const std::vector<uint32_t>& digs,
                                      uint32_t h_type, const std::string& tag);
  void transfer(const TransferWit& w, size_t idx);
  void issue(const IssueWit& w, size_t idx);
  void begin(const uint8_t* seed) { seed_off = arena_data(seed, 32, SRC_SEED); }
  void checks(uint32_t first_pt) {
    TxChecks t;
    t.wf_start = (uint32_t)pl.ck.size();
    t.wf_count = 0;
    if (pl.n_pts > first_pt) {
      Check c;
      c.kind = CK_PTS;
      c.code = E_PARSE;
      c.pad = 0;
      c.a = first_pt;
      c.b = pl.n_pts - first_pt;
      pl.ck.push_back(c);
      t.wf_count = 1;
    }
    t.rg_start = (uint32_t)pl.ck.size();
    t.rg_count = 0;
    t.mode = 0;
    pl.tx.push_back(t);
  }
};

// PB's value checks (transfer.go:100-107 / issue.go via range.Prover): every
// output's digits (prover_digits), zero digits for a refused value; "" or the
// error text of the first refused value
static std::string range_digits(const PPInfo& pp, const uint8_t* vals, uint32_t n, size_t idx, uint32_t* digs) {
  const uint32_t e = pp.exponent > 0 ? (uint32_t)pp.exponent : 0;
  std::string err;
  for (uint32_t k = 0; k < n; k++) {
    int r = prover_digits(pp, vals + 32 * k, digs + (size_t)k * e);
    if (r) {
      memset(digs + (size_t)k * e, 0, sizeof(uint32_t) * e);
      if (err.empty())
        err = "proof " + std::to_string(idx) +
              (r == 1 ? ": can't compute range proof: value of token outside authorized range"
                      : ": can't compute range proof: digit index out of range (the reference panics)");
    }
  }
  return err;
}

std::pair<uint32_t, uint32_t> PB::range(uint32_t tok_bytes, uint32_t n, const std::vector<uint32_t>& v,
                                        const std::vector<uint32_t>& bf, const std::vector<uint32_t>& digs,
                                        uint32_t h_type, const std::string& tag) {
  const uint32_t e = (uint32_t)pp.exponent, base = pp.base;
  uint32_t coms = arena_alloc(64 * n * e);
  uint32_t rg = arena_alloc(128 * n);
  struct Dig {
    uint32_t com, rp, obfs, chal, val, cbf, sbf, hash;
  };
  std::vector<std::vector<Dig>> dg(n, std::vector<Dig>(e));
  std::vector<uint32_t> cbf(n);
  (void)base;
  for (uint32_t k = 0; k < n; k++) {
    std::vector<uint32_t> parts;
    for (uint32_t i = 0; i < e; i++) {
      uint32_t d = digs[k * e + i];  // prover_digits: preProcess's values[i] (range/proof.go:297-311)
      std::string mt = tag + "/mp/" + std::to_string(k) + "/" + std::to_string(i);
      uint32_t dbf = rnd(tag + "/digit/" + std::to_string(k) + "/" + std::to_string(i) + "/bf");
      uint32_t sd = zr_u64(d, SRC_DIGIT, k * e + i);
      // Commitments[k][i] = d*Ped0 + dbf*Ped1   (range/proof.go:340-368)
      uint32_t com_off = coms + 64 * (k * e + i);
      g1job({{G1B_PED0, sd}, {G1B_PED1, dbf}}, NONE, NONE, com_off, NONE, false);
      // membership proof of d on the PS signature of d (sigproof/membership.go:112-158)
      uint32_t blinding = rnd(mt + "/sigbf"), rr = rnd(mt + "/randomize");
      // slot: [g1c 64 | GT 384 | sig JSON 235 | R' 64 | S'' 64]
      uint32_t slot = arena_alloc(64 + 384 + SIG_JSON_LEN + 128);
      uint8_t* js = &pl.arena[slot + 448];
      memcpy(js, SIG_JSON_R, 27);
      memcpy(js + 27 + 88, SIG_JSON_S, 29);
      memcpy(js + 27 + 88 + 29 + 88, SIG_JSON_E, 3);
      uint32_t rp_bytes = slot + 448 + SIG_JSON_LEN, obfs_bytes = rp_bytes + 64;
      // R' = rr*R, S'' = rr*S + blinding*P  (obfuscateSignature, :196-222)
      uint32_t Rp;
      if (sigtab) {  // (R, S) = SignedValues[d]: fixed bases of the prover's table set
        // with fixed pairs R' feeds no pairing (below), only the proof bytes
        Rp = g1job({{(uint8_t)(G1B_SIG0 + 2 * d), rr}}, NONE, NONE, rp_bytes, slot + 448 + 27, !pp.fixed_pairs);
        note_base(!pp.fixed_pairs, 0, 0, k * e + i);
        g1job({{G1B_PEDGEN, blinding}, {(uint8_t)(G1B_SIG0 + 2 * d + 1), rr}}, NONE, NONE, obfs_bytes,
              slot + 448 + 27 + 88 + 29, false);
        note_base(false, 1, 1, k * e + i);
      } else {
        uint32_t Rd = point(pp.sig_r[d].data(), (uint32_t)pp.sig_r[d].size(), NONE, SRC_SIG_R, k * e + i);
        uint32_t Sd = point(pp.sig_s[d].data(), (uint32_t)pp.sig_s[d].size(), NONE, SRC_SIG_S, k * e + i);
        Rp = g1job({}, Rd, rr, rp_bytes, slot + 448 + 27, true);
        g1job({{G1B_PEDGEN, blinding}}, Sd, rr, obfs_bytes, slot + 448 + 27 + 88 + 29, false);
      }
      // h = HashToZr(d.Bytes())
      uint8_t db[32] = {0};
      db[28] = (uint8_t)(d >> 24);
      db[29] = (uint8_t)(d >> 16);
      db[30] = (uint8_t)(d >> 8);
      db[31] = (uint8_t)d;
      uint32_t h = hash_pre(arena_data(db, 32, SRC_DIGIT, k * e + i), 32);
      uint32_t rv = rnd(mt + "/r_value"), rh = rnd(mt + "/r_hash"), rsbf = rnd(mt + "/r_sigbf");
      // GT = FExp(e(R', rv*PK1 + rh*PK2) * e(rsbf*P, Q))   (computeCommitment, :225-257)
      uint32_t p1 = g1job({{G1B_PEDGEN, rsbf}}, NONE, NONE, NONE, NONE, true);
      if (sigtab && pp.fixed_pairs) {
        // bilinearity: e(R', rv PK1 + rh PK2) = e((rv rr) R_d, PK1) e((rh rr) R_d, PK2), the
        // same GT element with every G2 argument fixed (precomputed lines, no G2 work)
        // and both G1 arguments fixed-base products of R_d
        uint32_t a = g1job({{(uint8_t)(G1B_SIG0 + 2 * d), sc(SOP_MUL, rv, rr)}}, NONE, NONE, NONE, NONE, true);
        note_base(true, 0, 0, k * e + i);
        uint32_t b = g1job({{(uint8_t)(G1B_SIG0 + 2 * d), sc(SOP_MUL, rh, rr)}}, NONE, NONE, NONE, NONE, true);
        note_base(true, 0, 0, k * e + i);
        pl.pr.push_back({p1, a, NONE, slot + 64, b});
      } else {
        G2Job g2;
        memset(&g2, 0, sizeof(g2));
        g2.nfix = 2;
        g2.fbase[0] = G2B_PK1;
        g2.fscal[0] = rv;
        g2.fbase[1] = G2B_PK2;
        g2.fscal[1] = rh;
        g2.out = pl.n_g2out++;
        pl.g2.push_back(g2);
        pl.pr.push_back({p1, Rp, g2.out, slot + 64, NONE});
      }
      uint32_t rcb = rnd(mt + "/r_combf");
      g1job({{G1B_PED0, rv}, {G1B_PED1, rcb}}, NONE, NONE, slot, NONE, false);
      // challenge (computeChallenge, membership.go:260-277)
      uint32_t c = challenge({{CONST_FLAG | C_PED0, 128},
                              {com_off, 64},
                              {slot, 64},
                              {CONST_FLAG | C_PEDGEN, 64},
                              {CONST_FLAG | C_PK_Q, 512},
                              {slot + 64, 384 + SIG_JSON_LEN}});
      Dig& D = dg[k][i];
      D.com = com_off;
      D.rp = rp_bytes;
      D.obfs = obfs_bytes;
      D.chal = c;
      D.val = resp(rv, c, sd);
      D.cbf = resp(rcb, c, dbf);
      D.sbf = resp(rsbf, c, blinding);
      D.hash = resp(rh, c, h);
      // commitment blinding factor of the token: sum_i dbf_i base^i
      uint64_t w = pp.pow[i];
      parts.push_back(sc(SOP_MULK64, dbf, (uint32_t)w, (uint32_t)(w >> 32)));
    }
    cbf[k] = sum(parts, true);
  }
  // equality proofs (range/proof.go:141-209)
  uint32_t rtype = rnd(tag + "/r_type");
  std::vector<uint32_t> rv(n), rcbf(n), rtbf(n);
  for (uint32_t k = 0; k < n; k++) {
    rv[k] = rnd(tag + "/r_value/" + std::to_string(k));
    rcbf[k] = rnd(tag + "/r_combf/" + std::to_string(k));
    rtbf[k] = rnd(tag + "/r_tokbf/" + std::to_string(k));
  }
  for (uint32_t k = 0; k < n; k++)
    g1job({{G1B_PED0, rtype}, {G1B_PED1, rv[k]}, {G1B_PED2, rtbf[k]}}, NONE, NONE, rg + 64 * k, NONE, false);
  for (uint32_t k = 0; k < n; k++)
    g1job({{G1B_PED0, rv[k]}, {G1B_PED1, rcbf[k]}}, NONE, NONE, rg + 64 * (n + k), NONE, false);
  uint32_t c = challenge({{CONST_FLAG | C_PEDGEN, 64},
                          {tok_bytes, 64 * n},
                          {rg, 128 * n},
                          {CONST_FLAG | C_PED0, 192},
                          {CONST_FLAG | C_Q_PK, 512},
                          {coms, 64 * n * e}});
  std::vector<uint32_t> ev(n), etb(n), ecb(n);
  for (uint32_t k = 0; k < n; k++) {
    ev[k] = resp(rv[k], c, v[k]);
    etb[k] = resp(rtbf[k], c, bf[k]);
    ecb[k] = resp(rcbf[k], c, cbf[k]);
  }
  uint32_t et = resp(rtype, c, h_type);
  // RangeProof JSON (range/proof.go:25-57)
  lit("{\"Challenge\":");
  zr(c);
  lit(",\"EqualityProofs\":{\"Type\":");
  zr(et);
  lit(",\"Value\":");
  zr_list(ev);
  lit(",\"TokenBlindingFactor\":");
  zr_list(etb);
  lit(",\"CommitmentBlindingFactor\":");
  zr_list(ecb);
  lit("},\"MembershipProofs\":[");
  for (uint32_t k = 0; k < n; k++) {
    if (k) lit(",");
    lit("{\"Commitments\":[");
    for (uint32_t i = 0; i < e; i++) {
      if (i) lit(",");
      g1(dg[k][i].com);
    }
    lit("],\"SignatureProofs\":[");
    for (uint32_t i = 0; i < e; i++) {
      const Dig& D = dg[k][i];
      if (i) lit(",");
      lit("{\"Challenge\":");
      zr(D.chal);
      lit(",\"Signature\":{\"R\":");
      g1(D.rp);
      lit(",\"S\":");
      g1(D.obfs);
      lit("},\"Value\":");
      zr(D.val);
      lit(",\"ComBlindingFactor\":");
      zr(D.cbf);
      lit(",\"SigBlindingFactor\":");
      zr(D.sbf);
      lit(",\"Hash\":");
      zr(D.hash);
      lit(",\"Commitment\":");
      g1(D.com);
      lit("}");
    }
    lit("]}");
  }
  lit("]}");
  return flush_doc();
}

void PB::transfer(const TransferWit& w, size_t idx) {
  const uint32_t ni = w.n_in, no = w.n_out;
  bool need_range = !(ni == 1 && no == 1);
  std::vector<uint32_t> ov;
  if (need_range) {
    ov.assign((size_t)no * (pp.exponent > 0 ? (size_t)pp.exponent : 0), 0);
    std::string e = range_digits(pp, w.out_values, no, idx, ov.data());
    if (err.empty()) err = e;
  }
  begin(w.seed);
  uint32_t first_pt = pl.n_pts;
  // tokens: inputs then outputs, canonical RawBytes (hashed by both transcripts)
  uint32_t tok = arena_alloc(64 * (ni + no));
  for (uint32_t i = 0; i < ni; i++) point(w.inputs + 64 * i, 64, tok + 64 * i, SRC_IN_PT, i);
  for (uint32_t k = 0; k < no; k++) point(w.outputs + 64 * k, 64, tok + 64 * (ni + k), SRC_OUT_PT, k);
  std::vector<uint32_t> iv(ni), ibf(ni), ovs(no), obf(no);
  for (uint32_t i = 0; i < ni; i++) {
    iv[i] = zr32(w.in_values + 32 * i, SRC_IN_VAL, i);
    ibf[i] = zr32(w.in_bfs + 32 * i, SRC_IN_BF, i);
  }
  for (uint32_t k = 0; k < no; k++) {
    ovs[k] = zr32(w.out_values + 32 * k, SRC_OUT_VAL, k);
    obf[k] = zr32(w.out_bfs + 32 * k, SRC_OUT_BF, k);
  }
  uint32_t h_type = hash_pre(arena_data(w.type, w.type_len, SRC_TYPE), (uint32_t)w.type_len);
  // range proof first (transfer.go:100-107), then well-formedness
  std::pair<uint32_t, uint32_t> rc(0, 0);
  if (need_range) {
    tagp = "";
    rc = range(tok + 64 * ni, no, ovs, obf, ov, h_type, "tx/range");
  }
  // WellFormednessProver (transfer/wellformedness.go:243-378)
  const std::string t = "tx/wf";
  uint32_t rt = rnd(t + "/r_type");
  std::vector<uint32_t> riv(ni), ribf(ni), rov(no), robf(no);
  for (uint32_t i = 0; i < ni; i++) {
    riv[i] = rnd(t + "/r_inv/" + std::to_string(i));
    ribf[i] = rnd(t + "/r_inbf/" + std::to_string(i));
  }
  uint32_t rs = rnd(t + "/r_sum");
  for (uint32_t k = 0; k < no; k++) {
    rov[k] = rnd(t + "/r_outv/" + std::to_string(k));
    robf[k] = rnd(t + "/r_outbf/" + std::to_string(k));
  }
  uint32_t nwf = ni + 1 + no + 1;
  uint32_t wf = arena_alloc(64 * nwf);
  // in_i = rv_i Ped1 + rt Ped0 + rbf_i Ped2; InputSum = (sum rbf) Ped2 + rs Ped1 + n_in rt Ped0
  for (uint32_t i = 0; i < ni; i++)
    g1job({{G1B_PED0, rt}, {G1B_PED1, riv[i]}, {G1B_PED2, ribf[i]}}, NONE, NONE, wf + 64 * i, NONE, false);
  g1job({{G1B_PED0, sc(SOP_MULK, rt, ni)}, {G1B_PED1, rs}, {G1B_PED2, sum(ribf)}}, NONE, NONE, wf + 64 * ni, NONE,
        false);
  for (uint32_t k = 0; k < no; k++)
    g1job({{G1B_PED0, rt}, {G1B_PED1, rov[k]}, {G1B_PED2, robf[k]}}, NONE, NONE, wf + 64 * (ni + 1 + k), NONE,
          false);
  g1job({{G1B_PED0, sc(SOP_MULK, rt, no)}, {G1B_PED1, rs}, {G1B_PED2, sum(robf)}}, NONE, NONE,
        wf + 64 * (nwf - 1), NONE, false);
  uint32_t c = challenge({{wf, 64 * nwf}, {tok, 64 * (ni + no)}});
  std::vector<uint32_t> r_ibf(ni), r_obf(no), r_iv(ni), r_ov(no);
  for (uint32_t i = 0; i < ni; i++) {
    r_ibf[i] = resp(ribf[i], c, ibf[i]);
    r_iv[i] = resp(riv[i], c, iv[i]);
  }
  for (uint32_t k = 0; k < no; k++) {
    r_obf[k] = resp(robf[k], c, obf[k]);
    r_ov[k] = resp(rov[k], c, ovs[k]);
  }
  uint32_t r_t = resp(rt, c, h_type), r_s = resp(rs, c, sum(iv));
  lit("{\"InputBlindingFactors\":");
  zr_list(r_ibf);
  lit(",\"OutputBlindingFactors\":");
  zr_list(r_obf);
  lit(",\"InputValues\":");
  zr_list(r_iv);
  lit(",\"OutputValues\":");
  zr_list(r_ov);
  lit(",\"Type\":");
  zr(r_t);
  lit(",\"Sum\":");
  zr(r_s);
  lit(",\"Challenge\":");
  zr(c);
  lit("}");
  std::pair<uint32_t, uint32_t> wfd = flush_doc();
  outer(wfd, need_range, rc);
  checks(first_pt);
}

void PB::issue(const IssueWit& w, size_t idx) {
  const uint32_t n = w.n_out;
  std::vector<uint32_t> vv((size_t)n * (pp.exponent > 0 ? (size_t)pp.exponent : 0), 0);
  {
    std::string e = range_digits(pp, w.values, n, idx, vv.data());
    if (err.empty()) err = e;
  }
  begin(w.seed);
  uint32_t first_pt = pl.n_pts;
  uint32_t tok = arena_alloc(64 * n);
  for (uint32_t k = 0; k < n; k++) point(w.outputs + 64 * k, 64, tok + 64 * k, SRC_OUT_PT, k);
  std::vector<uint32_t> v(n), bf(n);
  for (uint32_t k = 0; k < n; k++) {
    v[k] = zr32(w.values + 32 * k, SRC_OUT_VAL, k);
    bf[k] = zr32(w.bfs + 32 * k, SRC_OUT_BF, k);
  }
  uint32_t h_type = hash_pre(arena_data(w.type, w.type_len, SRC_TYPE), (uint32_t)w.type_len);
  // issue WellFormednessProver (issue/wellformedness.go:74-184)
  const std::string t = "issue/wf";
  uint32_t rt = w.anonymous ? rnd(t + "/r_type") : NONE;
  std::vector<uint32_t> rv(n), rbf(n);
  uint32_t coms = arena_alloc(64 * n);
  for (uint32_t k = 0; k < n; k++) {
    rv[k] = rnd(t + "/r_value/" + std::to_string(k));
    rbf[k] = rnd(t + "/r_bf/" + std::to_string(k));
    if (w.anonymous)
      g1job({{G1B_PED1, rv[k]}, {G1B_PED2, rbf[k]}, {G1B_PED0, rt}}, NONE, NONE, coms + 64 * k, NONE, false);
    else
      g1job({{G1B_PED1, rv[k]}, {G1B_PED2, rbf[k]}}, NONE, NONE, coms + 64 * k, NONE, false);
  }
  uint32_t c = challenge({{coms, 64 * n}, {tok, 64 * n}});
  std::vector<uint32_t> r_v(n), r_b(n);
  for (uint32_t k = 0; k < n; k++) {
    r_v[k] = resp(rv[k], c, v[k]);
    r_b[k] = resp(rbf[k], c, bf[k]);
  }
  lit("{\"Type\":");
  if (w.anonymous)
    zr(resp(rt, c, h_type));
  else
    lit("null");
  lit(",\"Values\":");
  zr_list(r_v);
  lit(",\"BlindingFactors\":");
  zr_list(r_b);
  lit(",\"TypeInTheClear\":");
  doc += w.anonymous ? std::string("\"\"") : go_json_str(w.type, w.type_len);
  lit(",\"Challenge\":");
  zr(c);
  lit("}");
  std::pair<uint32_t, uint32_t> wfd = flush_doc();
  std::pair<uint32_t, uint32_t> rc = range(tok, n, v, bf, vv, h_type, "issue/range");
  outer(wfd, true, rc);
  checks(first_pt);
}

// ---- shape templates.  A proof's plan depends on its witness only through
// the bytes PB records as patches (points, scalars, seed, type, the digits'
// signature points and values): every proof of one shape is the shape's
// template plan appended with relocated indices (plan_append) plus those
// bytes.  Planning a 4096-proof pass this way copies jobs instead of rebuilding
// tag strings, JSON documents and job lists per proof.
struct ProofTpl {
  Plan p;
  std::vector<Patch> patches;
  std::vector<BasePatch> bpatches;
  uint32_t img_arena = 0, img_out = 0;  // the piece's wire copies of p.arena / p.out
};

struct WitView {
  const uint8_t* seed;
  const uint8_t *in_pt, *out_pt, *in_val, *in_bf, *out_val, *out_bf;
  const char* type;
  const uint32_t* digs;  // output k's digit i at k * exponent + i (range_digits)
};

static void apply_patches(const PPInfo& pp, const ProofTpl& t, const PieceBase& o, const WitView& w, Plan& pl) {
  for (const BasePatch& q : t.bpatches) {
    uint32_t d = w.digs[q.k];
    G1Job& j = q.g1p ? pl.g1p[o.sec[PS_G1P] + q.job] : pl.g1[o.sec[PS_G1] + q.job];
    j.fbase[q.slot] = (uint8_t)(G1B_SIG0 + 2 * d + q.s);
  }
  for (const Patch& q : t.patches) {
    const uint8_t* src = nullptr;
    uint8_t tmp[32];
    uint32_t d = 0;
    if (q.kind >= SRC_SIG_R) d = w.digs[q.k];
    switch (q.kind) {
      case SRC_SEED: src = w.seed; break;
      case SRC_IN_PT: src = w.in_pt + 64 * q.k; break;
      case SRC_OUT_PT: src = w.out_pt + 64 * q.k; break;
      case SRC_IN_VAL: src = w.in_val + 32 * q.k; break;
      case SRC_IN_BF: src = w.in_bf + 32 * q.k; break;
      case SRC_OUT_VAL: src = w.out_val + 32 * q.k; break;
      case SRC_OUT_BF: src = w.out_bf + 32 * q.k; break;
      case SRC_TYPE: src = reinterpret_cast<const uint8_t*>(w.type); break;
      case SRC_SIG_R: src = pp.sig_r[d].data(); break;
      case SRC_SIG_S: src = pp.sig_s[d].data(); break;
      case SRC_DIGIT:  // zr_u64(d) and d.Bytes() of HashToZr: the same 32 big-endian bytes
        memset(tmp, 0, 32);
        for (int b = 0; b < 4; b++) tmp[31 - b] = (uint8_t)(d >> (8 * b));
        src = tmp;
        break;
    }
    if (!q.len) continue;
    if (!q.arena) {
      memcpy(pl.wire.data() + o.sec[PS_WIRE] + q.off, src, q.len);
    } else {  // device-initialised arena: the bytes travel in the wire pool
      uint32_t at = (uint32_t)pl.wire.size();
      pl.wire.insert(pl.wire.end(), src, src + q.len);
      pl.cp2.push_back({at, q.len, (uint32_t)(o.sec[PS_ARENA] + q.off), 0});
    }
  }
}

// templates need every signed value's encodings to have one length
static bool tpl_ok(const PPInfo& pp) {
  for (uint32_t d = 0; d < pp.base; d++)
    if (pp.sig_r[d].size() != pp.sig_r[0].size() || pp.sig_s[d].size() != pp.sig_s[0].size()) return false;
  return pp.base > 0 && pp.exponent > 0 && pp.pow.size() == (size_t)pp.exponent;
}

struct TplCache {
  std::vector<std::pair<std::string, ProofTpl>> v;
  ProofTpl* find(const std::string& key) {
    for (auto& e : v)
      if (e.first == key) return &e.second;
    return nullptr;
  }
};

static std::string key_of(const TransferWit& w) {
  char b[64];
  snprintf(b, sizeof b, "t%u/%u/%zu", w.n_in, w.n_out, w.type_len);
  return b;
}
static std::string key_of(const IssueWit& w) {
  char b[64];
  snprintf(b, sizeof b, "i%u/%u/%zu/", w.n_out, (unsigned)w.anonymous, w.type_len);
  // TypeInTheClear is JSON text of the template when the issue is not anonymous
  return w.anonymous ? std::string(b) : std::string(b) + std::string(w.type, w.type_len);
}

static void plan_one(PB& b, const TransferWit& x, size_t i) { b.transfer(x, i); }
static void plan_one(PB& b, const IssueWit& x, size_t i) { b.issue(x, i); }

static std::string tpl_digits(const PPInfo& pp, const TransferWit& w, size_t i, uint32_t* d) {
  if (w.n_in == 1 && w.n_out == 1) return "";  // no range proof (transfer.go:100-107)
  return range_digits(pp, w.out_values, w.n_out, i, d);
}
static std::string tpl_digits(const PPInfo& pp, const IssueWit& w, size_t i, uint32_t* d) {
  return range_digits(pp, w.values, w.n_out, i, d);
}
static WitView view_of(const TransferWit& w, const uint32_t* v) {
  return {w.seed, w.inputs, w.outputs, w.in_values, w.in_bfs, w.out_values, w.out_bfs, w.type, v};
}
static WitView view_of(const IssueWit& w, const uint32_t* v) {
  return {w.seed, nullptr, w.outputs, nullptr, nullptr, w.values, w.bfs, w.type, v};
}

template <class W>
std::string plan_prove_pieces(const PPInfo& pp, size_t n, const W* w, PlanWork& work, WorkPool& pool) {
  size_t np = plan_piece_count(n, pool.size());
  if (work.pieces.size() < np) work.pieces.resize(np);
  work.errs.assign(np, std::string());
  work.used = np;
  const bool tpl = tpl_ok(pp);
  pool.run(np, [&](size_t c) {
    Plan& p = work.pieces[c];
    p.clear();
    p.p2_g1out = true;
    p.dev_pools = tpl;
    size_t lo = n * c / np, hi = n * (c + 1) / np;
    if (!tpl) {  // direct planning (ragged signed-value encodings)
      PB b(p, pp);
      for (size_t i = lo; i < hi; i++) plan_one(b, w[i], i);
      work.errs[c] = b.err;
      return;
    }
    TplCache cache;
    std::vector<uint32_t> vals;
    for (size_t i = lo; i < hi; i++) {
      std::string key = key_of(w[i]);
      ProofTpl* t = cache.find(key);
      if (!t) {
        cache.v.emplace_back(key, ProofTpl());
        t = &cache.v.back().second;
        t->p.p2_g1out = true;
        PB b(t->p, pp);
        b.rec = &t->patches;
        b.brec = &t->bpatches;
        plan_one(b, w[i], i);
        // the shape's arena and output images, once per piece (the device copies
        // them into every proof's block, then the witness bytes over them)
        p.wire.resize((p.wire.size() + 15) & ~(size_t)15, 0);
        t->img_arena = (uint32_t)p.wire.size();
        p.wire.insert(p.wire.end(), t->p.arena.begin(), t->p.arena.end());
        t->img_out = (uint32_t)p.wire.size();
        p.wire.insert(p.wire.end(), t->p.out.begin(), t->p.out.end());
      }
      vals.assign((size_t)w[i].n_out * (size_t)pp.exponent, 0);
      std::string de = tpl_digits(pp, w[i], i, vals.data());
      if (!de.empty() && work.errs[c].empty()) work.errs[c] = de;
      PieceBase o = plan_append(p, t->p);
      p.cp.push_back({t->img_arena, (uint32_t)t->p.arena.size(), (uint32_t)o.sec[PS_ARENA], 0});
      p.cp.push_back({t->img_out, (uint32_t)t->p.out.size(), (uint32_t)o.sec[PS_OUT], 1});
      apply_patches(pp, *t, o, view_of(w[i], vals.data()), p);
    }
  });
  for (auto& e : work.errs)
    if (!e.empty()) return e;
  return "";
}

template <class W, class Fn>
std::string plan_prove(const PPInfo& pp, size_t n, const W* w, Plan& out, int threads, Fn fn) {
  WorkPool pool(threads);
  PlanWork work;
  (void)fn;
  std::string e = plan_prove_pieces(pp, n, w, work, pool);
  if (!e.empty()) return e;
  FlatPlan fp;
  e = flat_layout(work, true, fp);
  if (!e.empty()) return e;
  std::vector<uint8_t> blob(fp.bytes);
  flat_write(work, fp, blob.data(), std::vector<uint8_t>(C_SIZE, 0).data(), pool);
  plan_unflatten(fp, blob.data(), out);
  return "";
}

}  // namespace

std::string plan_prove_transfers(const PPInfo& pp, size_t n, const TransferWit* w, Plan& out, int threads) {
  return plan_prove(pp, n, w, out, threads, [](PB& b, const TransferWit& x, size_t i) { b.transfer(x, i); });
}

std::string plan_prove_issues(const PPInfo& pp, size_t n, const IssueWit* w, Plan& out, int threads) {
  return plan_prove(pp, n, w, out, threads, [](PB& b, const IssueWit& x, size_t i) { b.issue(x, i); });
}

std::string plan_prove_items_transfers(const PPInfo& pp, size_t n, const TransferWit* wit, PlanWork& w,
                                       WorkPool& pool) {
  return plan_prove_pieces(pp, n, wit, w, pool);
}

std::string plan_prove_items_issues(const PPInfo& pp, size_t n, const IssueWit* wit, PlanWork& w, WorkPool& pool) {
  return plan_prove_pieces(pp, n, wit, w, pool);
}

}  // namespace ftsh

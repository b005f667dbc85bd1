// Batch job model shared by the host planner (host/planner.cpp) and the HIP
// kernels (kernels.hip).  A batch of zkatdlog proofs is compiled on the host
// into flat, typed job arrays; each kernel runs one job per lane:
//
//   decode   wire G1 bytes -> Montgomery affine, on-curve check, canonical
//            RawBytes (+ base64 for the hashed signature JSON)
//   zr       wire Zr bytes (any length) -> canonical scalar mod r
//   scalar   derived scalars: a*b mod r, a*k mod r, sum mod r
//   g1       sum_i fixedbase_i * s_i  (-)  s * (sum_j w_j P_j)      -> G1 + bytes
//   g2       sum_i fixedbase_i * s_i  (PK0, PK1, PK2)                -> G2
//   miller   ML(P1, Q_pp) * ML(P2, Q2)  (Q_pp lines precomputed)    -> Fp12
//   fexp     final exponentiation -> GT bytes (gnark E12.Bytes order)
//   hash     SHA-256 over arena segments, mod r, compare with challenge
//   verdict  per proof: first failing check in reference order -> code
//
// Reference seams: transfer.Verifier.Verify (transfer/transfer.go:124),
// issue.Verifier.Verify (issue/issue.go:202), TransferZKProofValidate
// (validator/validator_transfer.go:84-98).
#pragma once
#include "fp29.h"
#include "fp_wide.h"
#include "glv.h"
#include "pairing.h"
#include "sha256.h"

namespace fts {

static constexpr uint32_t NONE = 0xFFFFFFFFu;

struct G1Dev {
  uint32_t x[8], y[8];  // Montgomery affine; all-zero = infinity
};
struct G2Dev {
  uint32_t x0[8], x1[8], y0[8], y1[8];
};
struct F12Dev {
  uint32_t w[96];
};

enum G1Base : uint8_t { G1B_PED0 = 0, G1B_PED1, G1B_PED2, G1B_PEDGEN, G1B_GEN, G1B_COUNT };
// The prover's table set appends the public parameters' PS signatures of the
// range digits (setup.go SignedValues): base G1B_SIG0 + 2 d is R_d, + 2 d + 1
// is S_d, so that R' = rr R_d and rr S_d are fixed-base products (16 table
// additions instead of a GLV variable-base chain).  fbase is 8 bits: digits
// base <= G1B_SIG_MAX_DIGITS.
static constexpr uint32_t G1B_SIG0 = G1B_COUNT;
static constexpr uint32_t G1B_SIG_MAX_DIGITS = (255 - G1B_SIG0) / 2;
enum G2Base : uint8_t { G2B_PK0 = 0, G2B_PK1, G2B_PK2, G2B_Q, G2B_COUNT };
// G2 fixed-base tables: signed FTS_G2TAB_C-bit windows, same layout as G1
// below (product library: C = 13, 20 windows, 4 x 20 x 4096 x 128 B = 42 MB;
// test-only host build: C = 8)
#ifndef FTS_G2TAB_C
#define FTS_G2TAB_C 8
#endif
static constexpr int G2TAB_C = FTS_G2TAB_C;
static constexpr int G2TAB_WINDOWS = (256 + G2TAB_C - 1) / G2TAB_C;
static constexpr int G2TAB_DIGITS = 1 << (G2TAB_C - 1);
// G1 fixed-base tables: signed FTS_G1TAB_C-bit windows, digits d in
// [-2^(C-1), 2^(C-1)], entries for |d| = 1 .. 2^(C-1) (d < 0: negate y).  The
// product library is built with C = 16 (16 mixed additions per fixed term;
// 5 bases x 16 x 32768 x 64 B = 168 MB, read by 64-byte gathers); the test-only
// host build keeps C = 8 (tables it can build per entry on the CPU).
#ifndef FTS_G1TAB_C
#define FTS_G1TAB_C 8
#endif
static constexpr int G1TAB_C = FTS_G1TAB_C;
static constexpr int G1TAB_WINDOWS = (256 + G1TAB_C - 1) / G1TAB_C;
static constexpr int G1TAB_DIGITS = 1 << (G1TAB_C - 1);

struct DecodeJob {
  uint32_t raw;       // offset of the element bytes in the wire pool
  uint32_t len;       // element length as received
  uint32_t out;       // pts index
  uint32_t bytes;     // arena offset for canonical RawBytes (NONE: skip)
  uint32_t b64;       // arena offset for 88 base64 chars (NONE: skip)
};

struct ZrJob {
  uint32_t raw, len;  // big-endian bytes in the wire pool (len <= ZR_MAX_LEN)
  uint32_t out;       // scalar index
};
static constexpr uint32_t ZR_MAX_LEN = 256;

enum ScalOp : uint32_t { SOP_MUL = 0, SOP_MULK = 1, SOP_SUM = 2, SOP_MADD = 3, SOP_MULK64 = 4 };
struct ScalJob {
  // MUL: a*b; MULK: a*(uint32)b; SUM: sum of list[a .. a+b); MADD: a + b*c
  // (Schnorr response r + c*w); MULK64: a*(b | c << 32)
  uint32_t op, a, b, out, c;
};

struct VTerm {
  uint32_t pt;        // pts index
  uint32_t w_lo, w_hi;
  uint32_t flags;     // VT_HORNER on a job's first term
};
// The job's variable part is sum_i b^i P_i given in Horner order: terms
// P_{e-1}, ..., P_0, each weight = b, computed as V = b V + P_t (PP-B range
// equality: 15 x (4 doublings + 1 addition) instead of 16 64-bit multiples)
static constexpr uint32_t VT_HORNER = 1;
// The term is subtracted (weight -w): the digit weight int64(math.Pow(b, i)) =
// -2^63 once b^i reaches 2^63 (range/proof.go:428), given as w = 2^63 | VT_NEG
static constexpr uint32_t VT_NEG = 2;

struct G1Job {
  uint32_t fscal[3];
  uint8_t fbase[3];
  uint8_t nfix;
  uint32_t vstart, vcount;  // VTerm range (variable points with small weights)
  uint32_t vscal;           // scalar of the variable part (NONE: no variable part)
  uint32_t vneg;            // 1: subtract the variable part
  uint32_t out;             // g1out index
  uint32_t bytes;           // arena offset for RawBytes (NONE: skip)
  uint32_t b64;             // arena offset for the 88 base64 chars of RawBytes (NONE: skip)
};

struct G2Job {
  uint32_t fscal[3];
  uint8_t fbase[3];
  uint8_t nfix;
  uint32_t out;
};

struct PairJob {
  uint32_t p1;     // g1out index, paired with the PP generator Q (precomputed lines)
  uint32_t p2;     // pts index (signature R); fixed pairs: g1out index paired with PK1
  uint32_t q2;     // g2out index (NONE with fixed pairs)
  uint32_t bytes;  // arena offset for the 384 GT bytes
  uint32_t p3;     // fixed pairs (prover): g1out index paired with PK2; else NONE
};

struct Seg {
  uint32_t off, len;  // arena byte range
};

struct HashJob {
  uint32_t seg_start, seg_count;
  uint32_t expect;    // scalar index of the claimed challenge (NONE: no compare)
  uint32_t out_scal;  // write HashToZr(data) to this scalar (NONE: skip)
};

// prover: rand(tag) = SHA-256(seed||tag||0) || SHA-256(seed||tag||1) mod r
// (the oracle's deterministic stand-in for crypto/rand, ftsoracle/zkat.py Rand)
struct RandJob {
  uint32_t seed;      // arena offset of the 32-byte per-proof seed
  uint32_t tag, len;  // arena range of the tag string
  uint32_t out;       // scalar index
};
// prover output: one fixed-length hole of a JSON template (base64 of an element)
enum EmitKind : uint32_t { EM_ZR = 0, EM_G1 = 1 };
struct EmitJob {
  uint32_t dst;   // arena offset of the 44 (Zr) / 88 (G1) base64 chars
  uint32_t kind;
  uint32_t src;   // EM_ZR: scalar index; EM_G1: arena offset of 64 RawBytes
};
// prover output: base64 of an inner JSON document into the outer proof
struct B64Job {
  uint32_t src, len;  // arena range
  uint32_t dst;       // offset in the proof output buffer
};
// prover: bytes the host does not write into the arena / proof output (a shape
// template's image, then the witness bytes patched over it), copied on the
// device from the wire pool
struct CopyJob {
  uint32_t src, len;  // wire range
  uint32_t dst;       // arena offset, or proof-output offset when to_out
  uint32_t to_out;
};

enum CheckKind : uint8_t { CK_STATIC = 0, CK_PTS = 1, CK_HASH = 2 };
struct Check {
  uint8_t kind;
  uint8_t code;  // error class reported if this check fails
  uint16_t pad;
  uint32_t a, b;  // CK_PTS: pts range [a, a+b); CK_HASH: hash job a
};
struct TxChecks {
  uint32_t wf_start, wf_count;  // first part ("well-formedness" / issue WF)
  uint32_t rg_start, rg_count;  // second part (range proof), may be empty
  uint32_t mode;                // 0: transfer precedence, 1: issue (sequential)
};

// error classes (mirror include/ftsamd.h)
enum : int32_t { E_OK = 0, E_PARSE = 1, E_MALFORMED = 2, E_WF = 3, E_RANGE = 4, E_MEMBERSHIP = 5, E_PANIC = 6 };

// ------------------------------------------------------------------ helpers
FTS_HD g1a g1_load(const G1Dev& d) {
  g1a a;
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a.x.v[i] = d.x[i];
    a.y.v[i] = d.y[i];
    o |= d.x[i] | d.y[i];
  }
  a.inf = (o == 0);
  return a;
}
FTS_HD void g1_store(G1Dev& d, const g1a& a) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    d.x[i] = a.inf ? 0u : a.x.v[i];
    d.y[i] = a.inf ? 0u : a.y.v[i];
  }
}
FTS_HD g2a g2_load(const G2Dev& d) {
  g2a a;
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a.x.c0.v[i] = d.x0[i];
    a.x.c1.v[i] = d.x1[i];
    a.y.c0.v[i] = d.y0[i];
    a.y.c1.v[i] = d.y1[i];
    o |= d.x0[i] | d.x1[i] | d.y0[i] | d.y1[i];
  }
  a.inf = (o == 0);
  return a;
}
FTS_HD void g2_store(G2Dev& d, const g2a& a) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    d.x0[i] = a.inf ? 0u : a.x.c0.v[i];
    d.x1[i] = a.inf ? 0u : a.x.c1.v[i];
    d.y0[i] = a.inf ? 0u : a.y.c0.v[i];
    d.y1[i] = a.inf ? 0u : a.y.c1.v[i];
  }
}
FTS_HD void f12_store(F12Dev& d, const fp12& f) {
  const fp* p = &f.c0.c0.c0;
  for (int k = 0; k < 12; k++)
    for (int i = 0; i < 8; i++) d.w[8 * k + i] = p[k].v[i];
}
FTS_HD fp12 f12_load(const F12Dev& d) {
  fp12 f;
  fp* p = &f.c0.c0.c0;
  for (int k = 0; k < 12; k++)
    for (int i = 0; i < 8; i++) p[k].v[i] = d.w[8 * k + i];
  return f;
}

// the standard base64 alphabet (A-Z a-z 0-9 + /) by arithmetic: a per-lane
// table lookup is a divergent memory load per character
FTS_HD uint8_t b64_char(uint32_t v) {
  const uint32_t c = v < 26 ? 'A' + v : (v < 52 ? 'a' + (v - 26) : (v < 62 ? '0' + (v - 52) : (v == 62 ? '+' : '/')));
  return (uint8_t)c;
}
FTS_HD void b64_encode_64(uint8_t* out, const uint8_t* in) {
  int o = 0;
  for (int k = 0; k < 63; k += 3) {
    uint32_t v = ((uint32_t)in[k] << 16) | ((uint32_t)in[k + 1] << 8) | in[k + 2];
    out[o++] = b64_char(v >> 18);
    out[o++] = b64_char((v >> 12) & 63);
    out[o++] = b64_char((v >> 6) & 63);
    out[o++] = b64_char(v & 63);
  }
  uint32_t v = (uint32_t)in[63] << 16;
  out[o++] = b64_char(v >> 18);
  out[o++] = b64_char((v >> 12) & 63);
  out[o++] = '=';
  out[o++] = '=';
}

// standard base64 (with '=' padding) of the 3-byte group g of in[0..len)
FTS_HD void b64_group(uint8_t* out, const uint8_t* in, uint32_t len, uint32_t g) {
  uint32_t k = 3 * g, rem = len - k;
  uint32_t v = (uint32_t)in[k] << 16;
  if (rem > 1) v |= (uint32_t)in[k + 1] << 8;
  if (rem > 2) v |= in[k + 2];
  out[0] = b64_char(v >> 18);
  out[1] = b64_char((v >> 12) & 63);
  out[2] = rem > 1 ? b64_char((v >> 6) & 63) : '=';
  out[3] = rem > 2 ? b64_char(v & 63) : '=';
}
FTS_HD void b64_encode(uint8_t* out, const uint8_t* in, uint32_t len) {
  for (uint32_t g = 0; 3 * g < len; g++) b64_group(out + 4 * g, in, len, g);
}

// ------------------------------------------------------------------ jobs
FTS_HD uint8_t job_decode(const DecodeJob& j, const uint8_t* wire, G1Dev* pts, uint8_t* arena) {
  g1a a;
  bool ok = g1_setbytes(wire + j.raw, j.len, a);
  G1Dev d;
  g1_store(d, a);
  pts[j.out] = d;
  if (j.bytes != NONE) g1_to_bytes_g(arena + j.bytes, a);
  if (j.b64 != NONE) {
    uint8_t tmp[64];
    g1_to_bytes(tmp, a);
    b64_encode_64(arena + j.b64, tmp);
  }
  return ok ? 1 : 0;
}

// G2 RawBytes (X.A1|X.A0|Y.A1|Y.A0), uncompressed only (public parameters)
FTS_HD uint8_t decode_g2(const uint8_t* b, uint32_t len, G2Dev& out, uint8_t* bytes_out) {
  g2a a;
  a.inf = true;
  bool ok = len >= 128 && (b[0] & 0xC0) == 0;
  if (ok) {
    uint32_t t[8];
    be32_to_limbs(t, b);
    a.x.c1 = fe_from_int<ModP>(t);
    be32_to_limbs(t, b + 32);
    a.x.c0 = fe_from_int<ModP>(t);
    be32_to_limbs(t, b + 64);
    a.y.c1 = fe_from_int<ModP>(t);
    be32_to_limbs(t, b + 96);
    a.y.c0 = fe_from_int<ModP>(t);
    a.inf = f2_is_zero(a.x) && f2_is_zero(a.y);
    ok = g2_on_curve(a);
  }
  g2_store(out, a);
  if (bytes_out) g2_to_bytes(bytes_out, a);
  return ok ? 1 : 0;
}

// G1 table entry idx = (base, window, |d| - 1): |d| * 2^(C window) * B (one
// scalar multiplication per entry: the host build and small C)
FTS_HD void job_tab_g1(uint32_t idx, const G1Dev* bases, G1Dev* tab) {
  uint32_t d = idx % G1TAB_DIGITS + 1, w = (idx / G1TAB_DIGITS) % G1TAB_WINDOWS,
           b = idx / (G1TAB_DIGITS * G1TAB_WINDOWS);
  uint32_t k[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // d << (C w) as 8 limbs (d < 2^C <= 2^16, C w < 256)
  uint32_t bit = (uint32_t)G1TAB_C * w, limb = bit >> 5, sh = bit & 31;
  uint64_t v = (uint64_t)d << sh;
  for (int q = 0; q < 8; q++) {
    if ((uint32_t)q == limb) k[q] = (uint32_t)v;
    if ((uint32_t)q == limb + 1) k[q] = (uint32_t)(v >> 32);
  }
  g1a r = jac_to_aff(aff_mul(g1_load(bases[b]), k));
  G1Dev o;
  g1_store(o, r);
  tab[idx] = o;
}
// G2 table entry idx = (base, window, |d| - 1): |d| * 2^(C window) * B
FTS_HD void job_tab_g2(uint32_t idx, const G2Dev* bases, G2Dev* tab) {
  uint32_t d = idx % G2TAB_DIGITS + 1, w = (idx / G2TAB_DIGITS) % G2TAB_WINDOWS,
           b = idx / (G2TAB_DIGITS * G2TAB_WINDOWS);
  uint32_t k[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t bit = (uint32_t)G2TAB_C * w, limb = bit >> 5, sh = bit & 31;
  uint64_t v = (uint64_t)d << sh;
  for (int q = 0; q < 8; q++) {
    if ((uint32_t)q == limb) k[q] = (uint32_t)v;
    if ((uint32_t)q == limb + 1) k[q] = (uint32_t)(v >> 32);
  }
  g2a r = jac_to_aff(aff_mul(g2_load(bases[b]), k));
  G2Dev o;
  g2_store(o, r);
  tab[idx] = o;
}

// big.Int SetBytes then mod r (scalar use) + "raw value < r" flag (Zr.Equals
// compares raw big integers, so a claimed challenge >= r never matches).
FTS_HD void job_zr(const ZrJob& j, const uint8_t* wire, uint32_t (*scal)[8], uint8_t* canon) {
  const uint8_t* b = wire + j.raw;
  uint32_t len = j.len;
  // strip leading zeros
  uint32_t s = 0;
  while (s < len && b[s] == 0) s++;
  uint32_t sig = len - s;
  // Horner over 32-byte chunks from the most significant end:
  // v_m = v_m * 2^256 + chunk   (Montgomery domain: mont(v*2^256) = v_m * R2 / R * R ...)
  fr acc = fe_zero<ModR>();
  fr r2 = fe_const<ModR>(R_R2);
  uint32_t first = sig % 32 == 0 ? 32 : sig % 32;
  uint32_t pos = s;
  bool firstc = true;
  while (pos < len) {
    uint32_t take = firstc ? first : 32;
    uint8_t chunk[32];
    for (int k = 0; k < 32; k++) chunk[k] = 0;
    for (uint32_t k = 0; k < take; k++) chunk[32 - take + k] = b[pos + k];
    pos += take;
    firstc = false;
    uint32_t t[8];
    be32_to_limbs(t, chunk);
    fr c = fe_from_int<ModR>(t);
    // acc * 2^256 in Montgomery form = acc_m * R2 (mont_mul divides by R once)
    acc = acc * r2 + c;
  }
  uint32_t out[8];
  fe_to_int(out, acc);
  for (int k = 0; k < 8; k++) scal[j.out][k] = out[k];
  // canonical: at most 32 significant bytes and value < r
  bool c = sig <= 32;
  if (c && sig > 0) {
    uint8_t full[32];
    for (int k = 0; k < 32; k++) full[k] = 0;
    for (uint32_t k = 0; k < sig; k++) full[32 - sig + k] = b[s + k];
    uint32_t t[8], d[8], mm[8];
    be32_to_limbs(t, full);
    for (int k = 0; k < 8; k++) mm[k] = R_MOD[k];
    c = sub8(d, t, mm) != 0;  // t < r
  }
  canon[j.out] = c ? 1 : 0;
}

FTS_HD void job_scalar(const ScalJob& j, uint32_t (*scal)[8], const uint32_t* list) {
  fr r;
  if (j.op == SOP_SUM) {
    r = fe_zero<ModR>();
    for (uint32_t k = 0; k < j.b; k++) r = r + fe_from_int<ModR>(scal[list[j.a + k]]);
  } else if (j.op == SOP_MADD) {
    r = fe_from_int<ModR>(scal[j.a]) + fe_from_int<ModR>(scal[j.b]) * fe_from_int<ModR>(scal[j.c]);
  } else if (j.op == SOP_MULK64) {
    uint32_t k[8] = {j.b, j.c, 0, 0, 0, 0, 0, 0};
    r = fe_from_int<ModR>(scal[j.a]) * fe_from_int<ModR>(k);
  } else {
    fr x = fe_from_int<ModR>(scal[j.a]);
    fr y;
    if (j.op == SOP_MUL) {
      y = fe_from_int<ModR>(scal[j.b]);
    } else {
      uint32_t k[8] = {j.b, 0, 0, 0, 0, 0, 0, 0};
      y = fe_from_int<ModR>(k);
    }
    r = x * y;
  }
  uint32_t out[8];
  fe_to_int(out, r);
  for (int k = 0; k < 8; k++) scal[j.out][k] = out[k];
}

// signed C-bit digit of window w of s (s < 2^254): the raw chunk plus the
// carry of the windows below, recomputed from window 0 (for code that visits
// windows out of order)
FTS_HD int32_t sdigit_at(const uint32_t s[8], int C, int w) {
  uint32_t carry = 0;
  int32_t d = 0;
  for (int v = 0; v <= w; v++) {
    uint32_t bit = (uint32_t)C * v, limb = bit >> 5, sh = bit & 31;
    uint64_t lo = limb < 8 ? s[limb] : 0, hi = limb + 1 < 8 ? s[limb + 1] : 0;
    uint32_t raw = (uint32_t)(((lo | (hi << 32)) >> sh) & ((1ull << C) - 1)) + carry;
    d = (int32_t)raw;
    carry = 0;
    if (raw > (1u << (C - 1))) {
      d = (int32_t)raw - (int32_t)(1u << C);
      carry = 1;
    }
  }
  return d;
}

FTS_HD g2j g2_fixed_acc(g2j acc, const G2Dev* tab, int base, const uint32_t s[8]) {
  uint32_t carry = 0;
  const G2Dev* tb = tab + (size_t)base * G2TAB_WINDOWS * G2TAB_DIGITS;
#pragma nounroll
  for (int w = 0; w < G2TAB_WINDOWS; w++) {
    uint32_t bit = (uint32_t)G2TAB_C * w, limb = bit >> 5, sh = bit & 31;
    uint64_t lo = limb < 8 ? s[limb] : 0, hi = limb + 1 < 8 ? s[limb + 1] : 0;
    uint32_t raw = (uint32_t)(((lo | (hi << 32)) >> sh) & ((1ull << G2TAB_C) - 1)) + carry;
    int32_t d = (int32_t)raw;
    carry = 0;
    if (raw > (1u << (G2TAB_C - 1))) {
      d = (int32_t)raw - (int32_t)(1u << G2TAB_C);
      carry = 1;
    }
    if (d) {
      g2a T = g2_load(tb[(size_t)w * G2TAB_DIGITS + (uint32_t)(d < 0 ? -d : d) - 1]);
      if (d < 0) T.y = f2_neg(T.y);
      acc = jac_add_aff(acc, T);
    }
  }
  return acc;
}

#ifndef FTS_G1_F29
#define FTS_G1_F29 1  // G1 loops in the carry-free 29-bit form (dev/fp29.h); 0: fp.h throughout
#endif

// sum_w d_w 2^(C w) B over the signed C-bit digits of s (s < r < 2^254, so the
// top window absorbs the last carry)
FTS_HD g1j g1_fixed_acc_fp(g1j acc, const G1Dev* tab, int base, const uint32_t s[8]);
FTS_HD g1j g1_fixed_acc(g1j acc, const G1Dev* tab, int base, const uint32_t s[8]) {
#if FTS_G1_F29
  // runs of mixed additions: the XYZZ accumulator (fp29.h x29_madd)
  x29 a{};
  a.inf = is_zero(acc.z);
  if (!a.inf) {
    j29 aj = j29_from(acc);
    f29 zz = f29_sqr(aj.z);
    a = {aj.x, aj.y, zz, f29_mul(zz, aj.z), false};
  }
  uint32_t carry = 0;
  const G1Dev* tb = tab + (size_t)base * G1TAB_WINDOWS * G1TAB_DIGITS;
#pragma nounroll
  for (int w = 0; w < G1TAB_WINDOWS; w++) {
    uint32_t bit = (uint32_t)G1TAB_C * w, limb = bit >> 5, sh = bit & 31;
    uint64_t lo = limb < 8 ? s[limb] : 0, hi = limb + 1 < 8 ? s[limb + 1] : 0;
    uint32_t raw = (uint32_t)(((lo | (hi << 32)) >> sh) & ((1ull << G1TAB_C) - 1)) + carry;
    int32_t d = (int32_t)raw;
    carry = 0;
    if (raw > (1u << (G1TAB_C - 1))) {
      d = (int32_t)raw - (int32_t)(1u << G1TAB_C);
      carry = 1;
    }
    if (d) {
      g1a T = g1_load(tb[(size_t)w * G1TAB_DIGITS + (uint32_t)(d < 0 ? -d : d) - 1]);
      f29 y = f29_from_fp(T.y);
      a = x29_madd(a, f29_from_fp(T.x), d < 0 ? f29_neg(y) : y);
    }
  }
  return j29_to(x29_to_j29(a));
#else
  return g1_fixed_acc_fp(acc, tab, base, s);
#endif
}
FTS_HD g1j g1_fixed_acc_fp(g1j acc, const G1Dev* tab, int base, const uint32_t s[8]) {
  uint32_t carry = 0;
  const G1Dev* tb = tab + (size_t)base * G1TAB_WINDOWS * G1TAB_DIGITS;
#pragma nounroll
  for (int w = 0; w < G1TAB_WINDOWS; w++) {
    uint32_t bit = (uint32_t)G1TAB_C * w, limb = bit >> 5, sh = bit & 31;
    uint64_t lo = limb < 8 ? s[limb] : 0, hi = limb + 1 < 8 ? s[limb + 1] : 0;
    uint32_t raw = (uint32_t)(((lo | (hi << 32)) >> sh) & ((1ull << G1TAB_C) - 1)) + carry;
    int32_t d = (int32_t)raw;
    carry = 0;
    if (raw > (1u << (G1TAB_C - 1))) {
      d = (int32_t)raw - (int32_t)(1u << G1TAB_C);
      carry = 1;
    }
    if (d) {
      g1a T = g1_load(tb[(size_t)w * G1TAB_DIGITS + (uint32_t)(d < 0 ? -d : d) - 1]);
      if (d < 0) T.y = fe_neg(T.y);
      acc = jac_add_aff(acc, T);
    }
  }
  return acc;
}

// k P for affine P and a scalar k < r.  Joint double-and-add over the two
// 128-bit GLV halves (Shamir): one mixed addition per bit with the operand
// chosen among P', phi(P)', P' + phi(P)' -- uniform across the wave.
FTS_HD g1j g1_mul_glv(const g1a& p, const uint32_t k[8]) {
  g1j acc = jac_inf<fp>();
  if (p.inf) return acc;
  uint32_t k1[4], k2[4];
  bool n1, n2;
  glv_split(k, k1, n1, k2, n2);
  g1a P1 = n1 ? aff_neg(p) : p;
  g1a P2;
  P2.x = p.x * fe_const<ModP>(GLV_BETA);
  P2.y = n2 ? fe_neg(p.y) : p.y;
  P2.inf = false;
  // S = P1 + P2 stays Jacobian (X:Y:Z); P1 != +-P2 for points of order r, so
  // Z != 0.  Instead of an inversion, run the loop on the isomorphic curve
  // y^2 = x^3 + b Z^6 through (x, y) -> (Z^2 x, Z^3 y): there S is the affine
  // point (X, Y), and the a = 0 doubling / mixed-addition formulas do not
  // involve b.  A result (X':Y':Z') there is (X':Y':Z' Z) on E.
  g1j Sj = jac_add_aff(jac_from_aff(P1), P2);
  fp z2 = sqr(Sj.z), z3 = z2 * Sj.z;
  P1.x = P1.x * z2;
  P1.y = P1.y * z3;
  P2.x = P2.x * z2;
  P2.y = P2.y * z3;
  g1a S;
  S.x = Sj.x;
  S.y = Sj.y;
  S.inf = false;
  // the scalars are consumed from the top bit by shifting them left (a
  // dynamically indexed limb array would live in scratch memory)
  uint32_t u0 = k1[0], u1 = k1[1], u2 = k1[2], u3 = k1[3];
  uint32_t v0 = k2[0], v1 = k2[1], v2 = k2[2], v3 = k2[3];
#pragma nounroll
  for (int i = 127; i >= 0; i--) {
    acc = jac_dbl(acc);
    uint32_t b1 = u3 >> 31, b2 = v3 >> 31;
    u3 = (u3 << 1) | (u2 >> 31);
    u2 = (u2 << 1) | (u1 >> 31);
    u1 = (u1 << 1) | (u0 >> 31);
    u0 <<= 1;
    v3 = (v3 << 1) | (v2 >> 31);
    v2 = (v2 << 1) | (v1 >> 31);
    v1 = (v1 << 1) | (v0 >> 31);
    v0 <<= 1;
    g1a T;
    T.x = b1 ? (b2 ? S.x : P1.x) : P2.x;
    T.y = b1 ? (b2 ? S.y : P1.y) : P2.y;
    T.inf = false;
    g1j nacc = jac_add_aff(acc, T);
    if (b1 | b2) acc = nacc;
  }
  acc.z = acc.z * Sj.z;  // back to E (the point at infinity keeps z = 0)
  return acc;
}

// Radix-16 Booth digit i of a 128-bit scalar: bits 4i-1 .. 4i+3 (bit -1 and
// bits >= 128 read as 0) give d = b(4i-1) + b(4i) + 2 b(4i+1) + 4 b(4i+2) - 8 b(4i+3)
// in [-8, 8]; k = sum_{i=0..32} d_i 16^i.  Limb selects instead of a
// dynamically indexed array (which would live in scratch memory).
FTS_HD int booth16(const uint32_t k[4], int i) {
  int pos = 4 * i - 1;
  uint32_t v;
  if (pos < 0) {
    v = (k[0] << 1) & 31u;
  } else {
    int l = pos >> 5, o = pos & 31;
    uint32_t lo = l == 0 ? k[0] : (l == 1 ? k[1] : (l == 2 ? k[2] : (l == 3 ? k[3] : 0u)));
    uint32_t hi = l == 0 ? k[1] : (l == 1 ? k[2] : (l == 2 ? k[3] : 0u));
    v = (uint32_t)(((((uint64_t)hi) << 32) | lo) >> o) & 31u;
  }
  return (int)(v & 1u) + (int)((v >> 1) & 7u) - 8 * (int)(v >> 4);
}

// k P with 4-bit signed windows over the two GLV halves: 33 windows of four
// doublings and two mixed additions with (|d| P1) and phi(|d| P1) from an
// 8-entry table -- 128 doublings + 66 additions instead of 128 + 128
// (g1_mul_glv).  The table 1..8 P1 is built in Jacobian coordinates and brought
// to ONE common Z = Zc without an inversion: entry e becomes the affine point
// (X_e s_e^2, Y_e s_e^3), s_e = Zc / Z_e, of the isomorphic curve
// y^2 = x^3 + b Zc^6 (the a = 0 doubling and mixed-addition formulas do not
// involve b), and the result (X:Y:Z) there is (X:Y:Z Zc) on E.
FTS_HD void g1dev_put(G1Dev& d, const fp& a, const fp& b) {
#pragma unroll
  for (int q = 0; q < 8; q++) {
    d.x[q] = a.v[q];
    d.y[q] = b.v[q];
  }
}
FTS_HD void g1dev_get(const G1Dev& d, fp& a, fp& b) {
#pragma unroll
  for (int q = 0; q < 8; q++) {
    a.v[q] = d.x[q];
    b.v[q] = d.y[q];
  }
}
// tb: 16 G1Dev entries at stride st (device: a per-batch buffer laid out
// [entry][job] so that a wave's accesses coalesce; host: a local array).
// Entries 0..7 hold the table, 8..15 the (Z, prefix) pairs while it is built.
// g1_mul_glv16_iso: k V for V = (X:Y:Z) Jacobian on E, Z != 0, without
// bringing V to affine first: (X, Y) is an affine point of the isomorphic curve
// y^2 = x^3 + b Z^6 (psi(x, y) = (x Z^2, y Z^3) maps E onto it and commutes with
// negation and phi(x, y) = (beta x, y)), so the same code runs on (X, Y) and
// the result (X':Y':Z') there is (X':Y':Z' Z) on E -- one product for an
// inversion.
FTS_HD g1j g1_mul_glv16_iso(const g1a& p, const fp& zin, const uint32_t k[8], G1Dev* tb, size_t st);
FTS_HD g1j g1_mul_glv16(const g1a& p, const uint32_t k[8], G1Dev* tb, size_t st) {
  if (p.inf) return jac_inf<fp>();
  return g1_mul_glv16_iso(p, fe_one<ModP>(), k, tb, st);
}
FTS_HD g1j g1_mul_glv16_iso(const g1a& p, const fp& zin, const uint32_t k[8], G1Dev* tb, size_t st) {
  g1j acc = jac_inf<fp>();
  uint32_t k1[4], k2[4];
  bool n1, n2;
  glv_split(k, k1, n1, k2, n2);
  g1a P1 = n1 ? aff_neg(p) : p;
  g1j T = jac_from_aff(P1);
  fp pre = fe_one<ModP>();
#pragma nounroll
  for (int e = 0; e < 8; e++) {
    if (e == 1) T = jac_dbl(T);
    if (e >= 2) T = jac_add_aff(T, P1);
    g1dev_put(tb[e * st], T.x, T.y);
    g1dev_put(tb[(8 + e) * st], T.z, pre);
    pre = pre * T.z;
  }
  const fp Zc = pre;
  fp suf = fe_one<ModP>();
#pragma nounroll
  for (int e = 7; e >= 0; e--) {
    fp X, Y, Z, pe;
    g1dev_get(tb[e * st], X, Y);
    g1dev_get(tb[(8 + e) * st], Z, pe);
    fp se = pe * suf;
    fp s2 = sqr(se);
    suf = suf * Z;
    g1dev_put(tb[e * st], X * s2, Y * (s2 * se));
  }
  const bool flip = n1 != n2;  // phi(e P1) = +-phi(e p): sign of the second half
#if FTS_G1_F29
  const f29 beta29 = f29_reduce(f29_from_fp(fe_const<ModP>(GLV_BETA)));
  j29 a = {f29{}, f29{}, f29{}, true};
#pragma nounroll
  for (int i = 32; i >= 0; i--) {
    int d1 = booth16(k1, i), d2 = booth16(k2, i);
    int m1 = d1 < 0 ? -d1 : d1, m2 = d2 < 0 ? -d2 : d2;
    fp x1, y1, x2, y2;
    g1dev_get(tb[(size_t)(m1 ? m1 - 1 : 0) * st], x1, y1);
    g1dev_get(tb[(size_t)(m2 ? m2 - 1 : 0) * st], x2, y2);
    if (i != 32) {
      a = j29_dbl(a);
      a = j29_dbl(a);
      a = j29_dbl(a);
      a = j29_dbl(a);
    }
    f29 Y = f29_from_fp(y1);
    j29 na = j29_madd(a, f29_from_fp(x1), (d1 < 0) ? f29_neg(Y) : Y);
    if (m1) a = na;
    Y = f29_from_fp(y2);
    na = j29_madd(a, f29_mul(f29_from_fp(x2), beta29), ((d2 < 0) != flip) ? f29_neg(Y) : Y);
    if (m2) a = na;
  }
  acc = j29_to(a);
#else
  const fp beta = fe_const<ModP>(GLV_BETA);
#pragma nounroll
  for (int i = 32; i >= 0; i--) {
    int d1 = booth16(k1, i), d2 = booth16(k2, i);
    int m1 = d1 < 0 ? -d1 : d1, m2 = d2 < 0 ? -d2 : d2;
    fp x1, y1, x2, y2;
    g1dev_get(tb[(size_t)(m1 ? m1 - 1 : 0) * st], x1, y1);
    g1dev_get(tb[(size_t)(m2 ? m2 - 1 : 0) * st], x2, y2);
    if (i != 32) {
      acc = jac_dbl(acc);
      acc = jac_dbl(acc);
      acc = jac_dbl(acc);
      acc = jac_dbl(acc);
    }
    g1a A;
    A.x = x1;
    A.y = (d1 < 0) ? fe_neg(y1) : y1;
    A.inf = false;
    g1j nacc = jac_add_aff(acc, A);
    if (m1) acc = nacc;
    A.x = x2 * beta;
    A.y = ((d2 < 0) != flip) ? fe_neg(y2) : y2;
    nacc = jac_add_aff(acc, A);
    if (m2) acc = nacc;
  }
#endif
  acc.z = acc.z * (Zc * zin);  // back to E (the point at infinity keeps z = 0)
  return acc;
}

#ifndef FTS_G1_VAR_W
#define FTS_G1_VAR_W 16  // 16: g1_mul_glv16 (signed 4-bit windows), 2: g1_mul_glv (joint binary)
#endif
#if FTS_G1_VAR_W == 16
#define G1_MUL_VAR(P, K, TB, ST) g1_mul_glv16(P, K, TB, ST)
#else
#define G1_MUL_VAR(P, K, TB, ST) g1_mul_glv(P, K)
#endif

FTS_HD void g1_emit_bytes(const G1Job& j, const g1a& r, uint8_t* arena) {
  if (j.bytes != NONE) g1_to_bytes_g(arena + j.bytes, r);
  if (j.b64 != NONE) {
    uint8_t tmp[64];
    g1_to_bytes(tmp, r);
    b64_encode_64(arena + j.b64, tmp);
  }
}

// ---- G1 jobs split into uniform parts (device path): item i of [0, 4n) is
// fixed-base slot f = i / n (0..2) or the variable part (f = 3) of job i % n;
// job_g1_combine adds the parts and converts to affine.  Same point as job_g1.
struct G1JDev {
  uint32_t x[8], y[8], z[8];  // Jacobian (Montgomery); z = 0: infinity
};
FTS_HD void g1j_store(G1JDev& d, const g1j& p) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    d.x[i] = p.x.v[i];
    d.y[i] = p.y.v[i];
    d.z[i] = p.z.v[i];
  }
}
FTS_HD g1j g1j_load(const G1JDev& d) {
  g1j p;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    p.x.v[i] = d.x[i];
    p.y.v[i] = d.y[i];
    p.z.v[i] = d.z[i];
  }
  return p;
}

// The variable point V of a G1 job's variable term, in Jacobian form, formed
// inline by doublings and mixed additions of the proof points (no call frames:
// out-of-line point routines here cost k_g1_part 400 B of scratch per lane on
// every launch) and handed to the GLV multiplication without an inversion
// (g1_mul_glv16_iso).
//   - a single unit-weight point;
//   - sum_t b^(count-1-t) P_t (VT_HORNER, the range-equality commitment sum)
//     with b a power of two (PP-B, b = 16): Horner, log2 b doublings a term;
//   - otherwise sum_t c_t P_t (c_t = b^(count-1-t), which fits 64 bits when the
//     planner marks the powers exact, or the explicit weights w_t) by one joint
//     left-to-right double-and-add over the c_t's bits (PP-A, b = 100, e = 2:
//     6 doublings and 4 additions).
FTS_HD uint64_t vterm_w(const VTerm& v) { return ((uint64_t)v.w_hi << 32) | v.w_lo; }
FTS_HD g1j g1_var_point(const G1Job& j, const VTerm* vterms, const G1Dev* pts) {
  const VTerm& v0 = vterms[j.vstart];
  const uint64_t b = vterm_w(v0);
  const bool horner = (v0.flags & VT_HORNER) != 0;
  if (j.vcount == 1 && (horner || b == 1) && !(v0.flags & VT_NEG)) return jac_from_aff(g1_load(pts[v0.pt]));
  if (horner && (b & (b - 1)) == 0) {
    const int top = b ? 63 - __builtin_clzll(b) : 0;
    g1j V = jac_from_aff(g1_load(pts[v0.pt]));
    for (uint32_t t = 1; t < j.vcount; t++) {
#pragma nounroll
      for (int q = 0; q < top; q++) V = jac_dbl(V);
      V = jac_add_aff(V, g1_load(pts[vterms[j.vstart + t].pt]));
    }
    return b ? V : jac_from_aff(g1_load(pts[vterms[j.vstart + j.vcount - 1].pt]));
  }
  // joint double-and-add; term t's weight: horner b^(count-1-t), else w_t
  uint64_t cmax = 0;
  if (horner) {
    cmax = 1;
    for (uint32_t t = 1; t < j.vcount; t++) cmax *= b;
  } else {
    for (uint32_t t = 0; t < j.vcount; t++) cmax |= vterm_w(vterms[j.vstart + t]);
  }
  g1j V = jac_inf<fp>();
  if (cmax == 0) return V;
  const int top = 63 - __builtin_clzll(cmax);
#pragma nounroll
  for (int q = top; q >= 0; q--) {
    if (q != top) V = jac_dbl(V);
    uint64_t c = 1;
#pragma nounroll
    for (uint32_t t = j.vcount; t-- > 0;) {
      const VTerm& vt = vterms[j.vstart + t];
      const uint64_t w = horner ? c : vterm_w(vt);
      if ((w >> q) & 1) {
        const g1a P = g1_load(pts[vt.pt]);
        V = jac_add_aff(V, (vt.flags & VT_NEG) ? aff_neg(P) : P);
      }
      c *= b;
    }
  }
  return V;
}

// One lane per job (host emulation): the variable part then the fixed-base
// slots, to affine.
FTS_HD void job_g1(const G1Job& j, const VTerm* vterms, const G1Dev* pts, const uint32_t (*scal)[8],
                   const G1Dev* tab, G1Dev* g1out, uint8_t* arena) {
  g1j acc = jac_inf<fp>();
  if (j.vscal != NONE) {
    g1j V = g1_var_point(j, vterms, pts);
    if (j.vneg) V = jac_neg(V);
    G1Dev loc[16];
    if (!is_zero(V.z)) acc = g1_mul_glv16_iso(g1a{V.x, V.y, false}, V.z, scal[j.vscal], loc, 1);
  }
  for (int f = 0; f < j.nfix; f++) acc = g1_fixed_acc(acc, tab, j.fbase[f], scal[j.fscal[f]]);
  g1a r = jac_to_aff(acc);
  G1Dev d;
  g1_store(d, r);
  g1out[j.out] = d;
  g1_emit_bytes(j, r, arena);
}

// Part f of job jb (i = f n + jb): f < 3 the fixed-base term f, f = 3 the
// variable term by GLV.  vtab: per-batch scratch of 16 n G1Dev entries for the
// variable parts' window tables (device); the host emulation may pass nullptr
// (a local table).
FTS_HD void job_g1_part(const G1Job* jobs, uint32_t n, uint32_t i, const VTerm* vterms, const G1Dev* pts,
                        const uint32_t (*scal)[8], const G1Dev* tab, G1JDev* part, G1Dev* vtab) {
  uint32_t f = i / n, jb = i - f * n;
  const G1Job& j = jobs[jb];
  g1j acc = jac_inf<fp>();
  if (f < 3) {
    if (f < j.nfix) acc = g1_fixed_acc(acc, tab, j.fbase[f], scal[j.fscal[f]]);
  } else if (j.vscal != NONE) {
    g1j V = g1_var_point(j, vterms, pts);
    if (j.vneg) V = jac_neg(V);
#if FTS_G1_VAR_W == 16
#if defined(__HIP_DEVICE_COMPILE__)
    G1Dev* tb = vtab + jb;
    const size_t st = n;
#else
    G1Dev loc[16];
    G1Dev* tb = vtab ? vtab + jb : loc;
    const size_t st = vtab ? n : 1;
#endif
    if (!is_zero(V.z)) acc = g1_mul_glv16_iso(g1a{V.x, V.y, false}, V.z, scal[j.vscal], tb, st);
#else
    acc = g1_mul_glv(jac_to_aff(V), scal[j.vscal]);
#endif
  }
  g1j_store(part[i], acc);
}

FTS_HD g1j job_g1_sum_parts(const G1Job& j, uint32_t jb, uint32_t n, const G1JDev* part) {
  g1j acc = g1j_load(part[3 * (size_t)n + jb]);
  for (uint32_t f = 0; f < 3; f++)
    if (f < j.nfix) acc = jac_add(acc, g1j_load(part[(size_t)f * n + jb]));
  return acc;
}

// affine result from the Jacobian sum and 1/z (any value when z = 0)
FTS_HD void job_g1_finish(const G1Job& j, const g1j& acc, const fp& zi, G1Dev* g1out, uint8_t* arena) {
  g1a r;
  r.inf = is_zero(acc.z);
  fp zi2 = sqr(zi);
  r.x = r.inf ? fe_zero<ModP>() : acc.x * zi2;
  r.y = r.inf ? fe_zero<ModP>() : acc.y * zi2 * zi;
  G1Dev d;
  g1_store(d, r);
  g1out[j.out] = d;
  g1_emit_bytes(j, r, arena);
}

// (x/y, 1/y) of the affine point of acc = (X:Y:Z) from inv = 1/(Z Y): x/y = X Z^2 inv,
// 1/y = Z^4 inv -- the normalised evaluation point of the fixed-Q Miller lines
// (sx29.h sq_fixed_line_n).  Unused for the point at infinity.
FTS_HD void g1_pnorm(const g1j& acc, const fp& inv, G1Dev& out) {
  fp z2 = sqr(acc.z);
  G1Dev d;
  g1_store(d, g1a{acc.x * z2 * inv, sqr(z2) * inv, false});
  out = d;
}

FTS_HD void job_g1_combine(const G1Job& j, uint32_t jb, uint32_t n, const G1JDev* part, G1Dev* g1out,
                           uint8_t* arena) {
  g1j acc = job_g1_sum_parts(j, jb, n, part);
  job_g1_finish(j, acc, is_zero(acc.z) ? fe_one<ModP>() : fp_inv(acc.z), g1out, arena);
}

FTS_HD void job_g2(const G2Job& j, const uint32_t (*scal)[8], const G2Dev* tab, G2Dev* g2out) {
  g2j acc = jac_inf<fp2>();
  for (int f = 0; f < j.nfix; f++) acc = g2_fixed_acc(acc, tab, j.fbase[f], scal[j.fscal[f]]);
  G2Dev d;
  g2_store(d, jac_to_aff(acc));
  g2out[j.out] = d;
}

FTS_HD void job_miller(const PairJob& j, const LineCoef* qlines, const G1Dev* g1out, const G1Dev* pts,
                       const G2Dev* g2out, F12Dev* fout, uint32_t idx) {
  fp12 f = miller_2(qlines, g1_load(g1out[j.p1]), g1_load(pts[j.p2]), g2_load(g2out[j.q2]));
  f12_store(fout[idx], f);
}

// the prover's fixed-pair product f(C, Q) f(A, PK1) f(B, PK2) (host emulation;
// the device runs k_miller_f3 on precomputed normalised lines of all three)
FTS_HD void job_miller3(const PairJob& j, const LineCoef* qlines, const LineCoef* pk1lines, const LineCoef* pk2lines,
                        const G1Dev* g1out, F12Dev* fout, uint32_t idx) {
  fp12 f = miller_fixed3(qlines, g1_load(g1out[j.p1]), pk1lines, g1_load(g1out[j.p2]), pk2lines,
                         g1_load(g1out[j.p3]));
  f12_store(fout[idx], f);
}

FTS_HD void job_fexp(const PairJob& j, const F12Dev* fin, uint32_t idx, uint8_t* arena, int variant = 0) {
  fp12 g = final_exp(f12_load(fin[idx]), variant);
  f12_to_bytes(arena + j.bytes, g);
}

FTS_HD uint8_t job_hash(const HashJob& j, const Seg* segs, const uint8_t* arena, uint32_t (*scal)[8],
                        const uint8_t* canon) {
  Sha256 s;
  s.init();
  for (uint32_t k = 0; k < j.seg_count; k++) {
    const Seg& g = segs[j.seg_start + k];
    s.update(arena + g.off, g.len);
  }
  uint8_t dg[32];
  s.final(dg);
  uint32_t h[8];
  digest_mod_r(h, dg);
  if (j.out_scal != NONE)
    for (int k = 0; k < 8; k++) scal[j.out_scal][k] = h[k];
  if (j.expect == NONE) return 1;
  uint32_t o = 0;
  for (int k = 0; k < 8; k++) o |= h[k] ^ scal[j.expect][k];
  return (o == 0 && canon[j.expect]) ? 1 : 0;
}

// prover randomness (RandJob)
FTS_HD void job_rand(const RandJob& j, const uint8_t* arena, uint32_t (*scal)[8]) {
  uint8_t h[2][32];
  for (int q = 0; q < 2; q++) {
    Sha256 s;
    s.init();
    s.update(arena + j.seed, 32);
    s.update(arena + j.tag, j.len);
    uint8_t b = (uint8_t)q;
    s.update(&b, 1);
    s.final(h[q]);
  }
  uint32_t t0[8], t1[8];
  be32_to_limbs(t0, h[0]);
  be32_to_limbs(t1, h[1]);
  // (h0 * 2^256 + h1) mod r; mont(h0) * R2 is the Montgomery form of h0 * 2^256
  fr v = fe_from_int<ModR>(t0) * fe_const<ModR>(R_R2) + fe_from_int<ModR>(t1);
  uint32_t out[8];
  fe_to_int(out, v);
  for (int k = 0; k < 8; k++) scal[j.out][k] = out[k];
}

// prover: byte b of a CopyJob (k_copy: one workgroup per job, lanes stride the bytes)
FTS_HD void job_copy_byte(const CopyJob& j, uint32_t b, const uint8_t* wire, uint8_t* arena, uint8_t* out) {
  (j.to_out ? out : arena)[j.dst + b] = wire[j.src + b];
}

// prover output holes (EmitJob): base64 of a 32-byte big-endian scalar or of
// 64 RawBytes already written into the arena
FTS_HD void job_emit(const EmitJob& j, const uint32_t (*scal)[8], uint8_t* arena) {
  if (j.kind == EM_ZR) {
    uint8_t b[32];
    limbs_to_be32(b, scal[j.src]);
    b64_encode(arena + j.dst, b, 32);
  } else {
    b64_encode_64(arena + j.dst, arena + j.src);
  }
}

FTS_HD int32_t eval_part(const Check* ck, uint32_t start, uint32_t count, const uint8_t* pt_ok,
                         const uint8_t* hash_ok) {
  for (uint32_t k = 0; k < count; k++) {
    const Check& c = ck[start + k];
    bool fail = false;
    if (c.kind == CK_STATIC) {
      fail = true;
    } else if (c.kind == CK_PTS) {
      for (uint32_t q = 0; q < c.b; q++) fail = fail || !pt_ok[c.a + q];
    } else {
      fail = !hash_ok[c.a];
    }
    if (fail) return c.code;
  }
  return E_OK;
}

// transfer.Verifier.Verify precedence (transfer/transfer.go:124-154): a panic
// in either part wins (the WF part runs first, synchronously); otherwise the
// WF error, then the range error.
// issue.Verifier.Verify (issue/issue.go:202-223) runs the parts sequentially:
// a WF error returns before the range proof is looked at.
FTS_HD int32_t job_verdict(const TxChecks& t, const Check* ck, const uint8_t* pt_ok, const uint8_t* hash_ok) {
  int32_t wf = eval_part(ck, t.wf_start, t.wf_count, pt_ok, hash_ok);
  if (wf == E_PANIC || (t.mode == 1 && wf != E_OK)) return wf;
  int32_t rg = eval_part(ck, t.rg_start, t.rg_count, pt_ok, hash_ok);
  if (rg == E_PANIC) return E_PANIC;
  return wf != E_OK ? wf : rg;
}

}  // namespace fts

// ------------------------------------------------------------------ sextet jobs
// Pairing jobs in the sextet layout (dev/sextet.h): lane k of the sextet of
// job idx holds coefficient k of the Miller-loop value.  F12Dev keeps gnark's
// E12 word order (C0.B0, C0.B1, C0.B2, C1.B0, C1.B1, C1.B2), so coefficient k
// lives at Fp2 index (k odd ? 3 + k/2 : k/2).
#include "sextet.h"

namespace fts {

FTS_HD int sx_f12_index(int k) { return (k & 1) ? 3 + (k >> 1) : (k >> 1); }

// Miller-loop lines of Q in consumption order (precompute_lines), each
// evaluated at P, stored at lines[n * njobs + idx].  A pair with an infinity
// point contributes 1 (gnark MillerLoop skips it): its lines are written as 1.
FTS_HD void g2lines_emit(const g2a& Q, const g1a& P, EvLineDev* lines, uint32_t idx, uint32_t njobs) {
  bool use = !(P.inf || Q.inf);
  g2p T = {Q.x, Q.y, f2_one()};
  uint32_t n = 0;
  auto emit = [&](const LineCoef& l) {
    fp2 c0 = use ? f2_mul_fp(l.r0, P.y) : f2_one();
    fp2 c3 = use ? f2_mul_fp(l.r1, P.x) : f2_zero();
    fp2 c4 = use ? l.r2 : f2_zero();
    evline_store(lines, n, idx, njobs, c0, c3, c4);
    n++;
  };
  // one inlined doubling and one inlined addition, the step schedule from a
  // table (uniform per step), so the loop keeps T in registers instead of the
  // call frames of out-of-line steps
#pragma nounroll
  for (int s = 0; s < MILLER_LINES; s++) {
    const int t = MILLER_STEPS.t[s];
    if (t == STEP_DBL) {
      emit(dbl_step_inl(T));
    } else {
      g2a A = t == STEP_FROB1 ? tw_frob(Q) : (t == STEP_FROB2 ? tw_frob2_neg(Q) : Q);
      if (t == STEP_SUB) A.y = f2_neg(A.y);
      emit(add_step_inl(T, A));
    }
  }
}

// Pair 2 of membership job idx (one lane): t' = c PK0 + v PK1 + h PK2 (the G2
// job with the same index; pok.go:175-183 folded), then its lines evaluated at
// P2 = R.  Layout [line][job]: a wave writes, and the sextet Miller kernel
// reads, consecutive jobs.
FTS_HD void job_g2lines(const G2Job& g, const PairJob& j, const uint32_t (*scal)[8], const G2Dev* tab,
                        G2Dev* g2out, const G1Dev* pts, EvLineDev* lines, uint32_t idx, uint32_t njobs) {
  job_g2(g, scal, tab, g2out);
  g2lines_emit(g2_load(g2out[g.out]), g1_load(pts[j.p2]), lines, idx, njobs);
}

// Split form of job_g2lines for the one-lane kernels: k_g2_part runs four
// lanes per job, lane q summing the table points of the (base, window)
// positions q, q + 4, ... into a Jacobian partial; k_g2lines1 adds the four
// partials, normalises t' and emits its lines.  Same t' (the affine sum does
// not depend on the order) and the same line bytes as job_g2lines.
struct G2PartDev {
  uint32_t w[48];  // Jacobian X, Y, Z (Fp2, Montgomery, c0 then c1)
};
FTS_HD void g2part_store(G2PartDev& d, const g2j& a) {
  const fp2* c[3] = {&a.x, &a.y, &a.z};
#pragma unroll
  for (int m = 0; m < 3; m++)
#pragma unroll
    for (int i = 0; i < 8; i++) {
      d.w[16 * m + i] = c[m]->c0.v[i];
      d.w[16 * m + 8 + i] = c[m]->c1.v[i];
    }
}
FTS_HD g2j g2part_load(const G2PartDev& d) {
  g2j a;
  fp2* c[3] = {&a.x, &a.y, &a.z};
#pragma unroll
  for (int m = 0; m < 3; m++)
#pragma unroll
    for (int i = 0; i < 8; i++) {
      c[m]->c0.v[i] = d.w[16 * m + i];
      c[m]->c1.v[i] = d.w[16 * m + 8 + i];
    }
  return a;
}
FTS_HD void job_g2_part(const G2Job& g, int q, const uint32_t (*scal)[8], const G2Dev* tab, G2PartDev& out) {
  g2j acc = jac_inf<fp2>();
#pragma nounroll
  for (int p = q; p < 3 * G2TAB_WINDOWS; p += 4) {
    int f = p / G2TAB_WINDOWS, w = p % G2TAB_WINDOWS;
    if (f < g.nfix) {
      int32_t d = sdigit_at(scal[g.fscal[f]], G2TAB_C, w);
      if (d) {
        g2a T = g2_load(tab[((size_t)g.fbase[f] * G2TAB_WINDOWS + w) * G2TAB_DIGITS + (uint32_t)(d < 0 ? -d : d) - 1]);
        if (d < 0) T.y = f2_neg(T.y);
        acc = jac_add_aff(acc, T);
      }
    }
  }
  g2part_store(out, acc);
}
// parts of job idx at part[q * njobs + idx]
FTS_HD void job_g2lines_parts(const G2Job& g, const PairJob& j, const G2PartDev* part, G2Dev* g2out,
                              const G1Dev* pts, EvLineDev* lines, uint32_t idx, uint32_t njobs) {
  g2j acc = g2part_load(part[idx]);
#pragma nounroll
  for (int q = 1; q < 4; q++) acc = jac_add_inl(acc, g2part_load(part[(size_t)q * njobs + idx]));
  G2Dev d;
  g2_store(d, jac_to_aff_inl(acc));  // inline: no call frame in scratch
  g2out[g.out] = d;
  g2lines_emit(g2_load(d), g1_load(pts[j.p2]), lines, idx, njobs);
}

// Sextet form of job_g2lines (same values): six lanes per membership digit.
//  phase A  t' = sum over (base, window) of table points: lane k takes the
//           pairs k, k+6, ... (16 mixed additions), then a 3-level tree of
//           Jacobian additions through LDS and one affine conversion;
//  phase B  the 88 Miller lines of t': each doubling / addition step runs as
//           layers of one reduced Fp2 product per lane (dbl_step / add_step
//           formulas), the running point T held identically by every lane;
//           the six lanes write the six Fp components of each evaluated line
//           (balanced 29-bit form, EvLineDev).
template <class X>
FTS_HD void sx_job_g2lines(const X& x, const G2Job& g, const PairJob& j, const uint32_t (*scal)[8],
                           const G2Dev* tab, G2Dev* g2out, const G1Dev* pts, EvLineDev* lines, uint32_t idx,
                           uint32_t njobs, bool valid) {
  const int k = x.k;
  // ---- phase A
  g2j acc = jac_inf<fp2>();
#pragma nounroll
  for (int p = k; p < 3 * G2TAB_WINDOWS; p += 6) {
    int f = p / G2TAB_WINDOWS, w = p % G2TAB_WINDOWS;
    if (f < g.nfix) {
      int32_t d = sdigit_at(scal[g.fscal[f]], G2TAB_C, w);
      if (d) {
        g2a T = g2_load(tab[((size_t)g.fbase[f] * G2TAB_WINDOWS + w) * G2TAB_DIGITS + (uint32_t)(d < 0 ? -d : d) - 1]);
        if (d < 0) T.y = f2_neg(T.y);
        acc = jac_add_aff(acc, T);
      }
    }
  }
  x.put(3 * k + 0, acc.x);
  x.put(3 * k + 1, acc.y);
  x.put(3 * k + 2, acc.z);
  x.sync();
  if (k < 3) acc = jac_add(acc, g2j{x.get(3 * k + 9), x.get(3 * k + 10), x.get(3 * k + 11)});
  x.sync();
  if (k < 3) {
    x.put(3 * k + 0, acc.x);
    x.put(3 * k + 1, acc.y);
    x.put(3 * k + 2, acc.z);
  }
  x.sync();
  acc = jac_add(g2j{x.get(0), x.get(1), x.get(2)}, g2j{x.get(3), x.get(4), x.get(5)});
  acc = jac_add(acc, g2j{x.get(6), x.get(7), x.get(8)});
  x.sync();
  g2a Q = jac_to_aff(acc);
  if (valid && k == 0) {
    G2Dev d;
    g2_store(d, Q);
    g2out[g.out] = d;
  }
  // ---- phase B
  g1a P = g1_load(pts[j.p2]);
  bool use = !(P.inf || Q.inf);
  const fp2 yP = f2_of_fp(P.y), xP = f2_of_fp(P.x), b3 = f2_const(TWIST_B);
  fp2 TX = Q.x, TY = Q.y, TZ = f2_one();
  int i = 64, sign = 0;
  bool pend = false;
#pragma nounroll
  for (int s = 0; s < MILLER_LINES; s++) {
    // line type: doubling, addition of +-Q (NAF digit), or a Frobenius line
    bool dbl = false;
    g2a Qa = Q;
    if (s >= MILLER_LINES - 2) {
      Qa = (s == MILLER_LINES - 2) ? tw_frob(Q) : tw_frob2_neg(Q);
    } else if (!pend) {
      dbl = true;
      sign = naf_digit(i);
      pend = sign != 0;
      if (!pend) i--;
    } else {
      if (sign < 0) Qa = aff_neg(Q);
      pend = false;
      i--;
    }
    fp2 l0, l1, l3;
    if (dbl) {
      // dbl_step: A = XY/2, B = Y^2, C = Z^2, E = 3C b', F = 3E, G = (B+F)/2,
      // H = (Y+Z)^2 - (B+C), I = E - B, J = X^2; line (-H, 3J, I)
      fp2 YZ = TY + TZ;
      x.put(SX_P + k, f2_pick(k, TX, TY, TZ, YZ, TX, TX) * f2_pick(k, TY, TY, TZ, YZ, TX, TX));
      x.sync();
      fp2 A = f2_half(x.get(SX_P + 0)), B = x.get(SX_P + 1), C = x.get(SX_P + 2);
      fp2 H = x.get(SX_P + 3) - (B + C), J = x.get(SX_P + 4);
      x.sync();
      x.put(SX_P + k, f2_pick(k, C + C + C, f2_neg(H), J + J + J, C, C, C) * f2_pick(k, b3, yP, xP, b3, b3, b3));
      x.sync();
      fp2 E = x.get(SX_P + 0);
      l0 = x.get(SX_P + 1);
      l1 = x.get(SX_P + 2);
      x.sync();
      l3 = E - B;
      fp2 F = E + E + E, G = f2_half(B + F);
      x.put(SX_P + k, f2_pick(k, A, G, E, B, A, A) * f2_pick(k, B - F, G, E, H, B, B));
      x.sync();
      TX = x.get(SX_P + 0);
      fp2 EE = x.get(SX_P + 2);
      TY = x.get(SX_P + 1) - (EE + EE + EE);
      TZ = x.get(SX_P + 3);
      x.sync();
    } else {
      // add_step: O = Y - Qy Z, L = X - Qx Z, C = O^2, D = L^2, E = L D, F = Z C,
      // G = X D, H = E + F - 2G; X3 = L H, Y3 = (G - H) O - Y E, Z3 = E Z;
      // line (L, -O, Qx O - L Qy)
      x.put(SX_P + k, f2_pick(k, Qa.y, Qa.x, Qa.y, Qa.y, Qa.y, Qa.y) * TZ);
      x.sync();
      fp2 O = TY - x.get(SX_P + 0), Lc = TX - x.get(SX_P + 1);
      x.sync();
      x.put(SX_P + k, f2_pick(k, O, Lc, Qa.x, Lc, Lc, f2_neg(O)) * f2_pick(k, O, Lc, O, Qa.y, yP, xP));
      x.sync();
      fp2 C = x.get(SX_P + 0), D = x.get(SX_P + 1);
      l3 = x.get(SX_P + 2) - x.get(SX_P + 3);
      l0 = x.get(SX_P + 4);
      l1 = x.get(SX_P + 5);
      x.sync();
      x.put(SX_P + k, f2_pick(k, Lc, TZ, TX, Lc, Lc, Lc) * f2_pick(k, D, C, D, D, D, D));
      x.sync();
      fp2 E = x.get(SX_P + 0), F = x.get(SX_P + 1), G = x.get(SX_P + 2);
      x.sync();
      fp2 H = E + F - (G + G);
      x.put(SX_P + k, f2_pick(k, TY, Lc, G - H, E, E, E) * f2_pick(k, E, H, O, TZ, TZ, TZ));
      x.sync();
      fp2 t1 = x.get(SX_P + 0);
      TX = x.get(SX_P + 1);
      TY = x.get(SX_P + 2) - t1;
      TZ = x.get(SX_P + 3);
      x.sync();
    }
    // lane k converts and writes component k (part k & 1 of coefficient k >> 1)
    const int m = k >> 1;
    fp2 v = m == 0 ? (use ? l0 : f2_one()) : (m == 1 ? (use ? l1 : f2_zero()) : (use ? l3 : f2_zero()));
    if (valid) evline_put(lines, s, k, idx, njobs, (k & 1) ? v.c1 : v.c0);
  }
}

template <class X>
FTS_HD void sx_job_miller(const X& x, const PairJob& j, const LineCoef* qlines, const EvLineDev* lines2,
                          const G1Dev* g1out, F12Dev* fout, uint32_t idx, uint32_t njobs, bool valid) {
  fp2 f = sx_miller_f(x, qlines, g1_load(g1out[j.p1]), lines2, idx, njobs);
  if (valid) {
    uint32_t* o = &fout[idx].w[16 * sx_f12_index(x.k)];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      o[i] = f.c0.v[i];
      o[8 + i] = f.c1.v[i];
    }
  }
}

}  // namespace fts

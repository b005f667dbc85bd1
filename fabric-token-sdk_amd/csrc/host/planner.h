// Host planner: zkatdlog proof bytes -> flat GPU job arrays (see dev/jobs.h).
#pragma once
#include <stdint.h>

#include <functional>
#include <string>
#include <vector>

#include "../dev/jobs.h"

namespace ftsh {

using namespace fts;

// Const region at the start of every batch arena: canonical RawBytes of the
// public-parameter points in the orders the transcripts hash them.
enum : uint32_t {
  C_PEDGEN = 0,    // P
  C_PED0 = 64,     // Ped0 | Ped1 | Ped2 contiguous
  C_PED1 = 128,
  C_PED2 = 192,
  C_Q_PK = 256,    // Q | PK0 | PK1 | PK2   (range transcript order)
  C_PK_Q = 384,    // PK0 | PK1 | PK2 | Q   (membership transcript order)
  C_SIZE = 896,
};
static constexpr uint32_t CONST_FLAG = 0x80000000u;  // Seg.off relative to the const region

// Parsed public parameters (setup.go:25-54); element bytes are decoded on GPU.
struct PPInfo {
  std::vector<uint8_t> pedgen, ped[3], pk[3], q;  // raw element bytes
  std::vector<std::vector<uint8_t>> sig_r, sig_s; // SignedValues
  uint32_t base = 0;                              // len(SignedValues)
  int64_t exponent = 0;
  int64_t curve = 0;
  std::string label;
  // digit weights w_i = int64(math.Pow(float64(base), float64(i))), i < exponent,
  // as the int64's bit pattern (range/proof.go:428; digit_weight below): base^i
  // while that is a float64, the rounded float64 above 2^53, and INT64_MIN once
  // it reaches 2^63
  std::vector<uint64_t> pow;
  int64_t pow_top = 0;                            // w_exponent: the prover's bound (range/proof.go:303)
  bool pow_exact = false;                         // every pow[i] is base^i exactly (float64 math.Pow was exact)
  // the prover's membership commitments as three fixed-G2 pairings (Q, PK1,
  // PK2; parse_pp: every line of the three normalisable and pp_sig_tables)
  bool fixed_pairs = false;
  // parity debugging (ftz_ctx_set_debug FTZ_DEBUG_CHALLENGES): every
  // verification transcript hash also writes its HashToZr into a scalar slot of
  // its own, which ftz_batch_challenges reads back (set before planning)
  bool debug_challenges = false;
  // the runtime's copy for planning WITHOUT the prover's table set (not built:
  // ftz_options.prover_tables = 0, or its allocation failed): pp_sig_tables false
  bool no_sigtab = false;
};
// The prover multiplies by the PS signature points of the digits through fixed-
// base tables (G1B_SIG0 ..) when every digit fits the 8-bit base index and no
// signature point is the identity (64 zero bytes); else through the variable-
// base path.  The runtime / host emulation build those tables on first use.
bool pp_sig_tables(const PPInfo& pp);
// Largest RangeProofParams.Exponent a context accepts (the reference bounds it
// only by != 0; a range proof then holds 2 x Exponent membership proofs per token).
static constexpr int64_t MAX_EXPONENT = 1024;
// Go math.Pow(x, float64(n)) for an integer n >= 0 and finite x >= 2 (Go
// src/math/pow.go, go1.18: Frexp, repeated mantissa squaring, Ldexp) and
// int64(f) as amd64 converts it (out of range -> INT64_MIN, [EXT]).
double go_pow_int(double x, int64_t n);
int64_t go_int64(double f);
// int64(math.Pow(float64(base), float64(i))): the weight of digit i
int64_t digit_weight(uint32_t base, int64_t i);
// The digits range.Prover.preProcess commits to (range/proof.go:297-311) for a
// value given as 32 big-endian bytes; 0 on success, 1 when the value is
// refused ("value of token outside authorized range"), 2 when the reference
// would panic (a digit >= base indexes past Signatures, :326).  Where the
// reference's bound int64(math.Pow(base, exponent)) overflows (PP-B) the
// build's [EXT] extension proves v < base^exponent by exact digits.
int prover_digits(const PPInfo& pp, const uint8_t* be32, uint32_t* digits);
// The recomputed challenges of one proof of a debug_challenges plan: its
// CK_HASH checks in check order (well-formedness, then the range part: every
// membership proof in (output, digit) order, then the range proof) as (class
// code E_WF / E_MEMBERSHIP / E_RANGE, scalar slot holding the HashToZr).
// Returns the number of such checks (entries beyond cap are not written).
size_t proof_challenge_slots(const TxChecks& t, const Check* ck, const HashJob* hmain, int32_t* kinds,
                             uint32_t* slots, size_t cap);
// Returns empty string on success, else an error message.
std::string parse_pp(const uint8_t* p, size_t n, const char* label, PPInfo& out);
// PublicParams.Validate (setup.go:238-273) on serialized PP: "" or the error text
std::string validate_pp(const uint8_t* p, size_t n, const char* label);

struct Plan {
  std::vector<uint8_t> wire;   // raw element bytes (decode / zr job inputs)
  std::vector<uint8_t> arena;  // per-proof arena regions (host-written parts)
  std::vector<DecodeJob> dec;
  std::vector<ZrJob> zr;
  std::vector<ScalJob> sc;
  std::vector<uint32_t> sclist;
  std::vector<VTerm> vt;
  std::vector<G1Job> g1;   // G1 jobs independent of the pairings
  std::vector<G1Job> g1p;  // G1 jobs whose outputs feed the Miller loops
  std::vector<G2Job> g2;
  std::vector<PairJob> pr;
  std::vector<Seg> seg;
  std::vector<HashJob> hpre, hmain;
  std::vector<Check> ck;
  std::vector<TxChecks> tx;
  // prover plans (planner_prove.cpp)
  std::vector<RandJob> rnd;
  std::vector<ScalJob> sc1;      // scalar jobs that read outputs of `sc` (run after it)
  std::vector<ScalJob> sc_post;  // responses, after the transcript hashes
  std::vector<EmitJob> emit;
  std::vector<B64Job> b64;
  std::vector<CopyJob> cp;        // device-side arena / output initialisation (before every other job)
  std::vector<CopyJob> cp2;       // then the witness bytes over it
  std::vector<uint8_t> out;       // outer proof JSON templates, concatenated
  std::vector<uint32_t> out_off;  // per proof: start in `out` (plus a final end)
  std::vector<uint32_t> item_off; // openings: arena offset of the 128-byte result (recomputed | decoded)
  bool p2_g1out = false;          // PairJob.p2 indexes g1out (prover) instead of pts
  // device-initialised pools (prover shape templates): the arena / out bytes are
  // not held here -- cp / cp2 write them on the device -- only their lengths
  bool dev_pools = false;
  size_t arena_len = 0, out_len = 0;
  uint32_t n_pts = 0, n_scal = 0, n_g1out = 0, n_g2out = 0;
  void clear();
};

struct TransferIn {
  const uint8_t* inputs;   // n_in x 64-byte gnark G1 RawBytes (ledger commitments)
  uint32_t n_in;
  const uint8_t* outputs;  // n_out x 64-byte RawBytes (TransferAction output commitments)
  uint32_t n_out;
  const uint8_t* proof;    // json(transfer.Proof)
  size_t proof_len;
};
struct IssueIn {
  const uint8_t* outputs;
  uint32_t n_out;
  const uint8_t* proof;    // json(issue.Proof)
  size_t proof_len;
  uint8_t anonymous;
};

// A token opening (token.TokenDataWitness / audit.AuditableToken data):
// the commitment H(type)*P0 + value*P1 + bf*P2 is recomputed
// (token/token.go:64-76 computeTokens; audit/auditor.go:208-234 InspectOutput
// compares it with `commitment` when that is given).
struct OpeningIn {
  const char* type;
  size_t type_len;
  const uint8_t* value;       // 32-byte big-endian Zr
  const uint8_t* bf;          // 32-byte big-endian Zr
  const uint8_t* commitment;  // 64-byte RawBytes to check, or null (commit only)
};

// One item of a (possibly mixed) batch: a block of a ledger carries transfer
// and issue actions side by side.
struct PlanItem {
  uint8_t kind;  // 0: transfer, 1: issue, 2: token opening
  TransferIn t;
  IssueIn i;
  OpeningIn o;
};

// A small persistent pool of host threads; run(n, f) calls f(0..n-1) across
// the pool and the caller and returns when all calls are done.  Concurrent
// run() calls are serialised.
class WorkPool {
 public:
  explicit WorkPool(int threads);
  ~WorkPool();
  WorkPool(const WorkPool&) = delete;
  WorkPool& operator=(const WorkPool&) = delete;
  void run(size_t n, const std::function<void(size_t)>& f);
  int size() const { return nthreads_ + 1; }

 private:
  struct State;
  State* st_;
  int nthreads_;
};

// Sections of a flattened plan: every job array and byte pool of a batch at a
// 256-byte aligned offset of ONE blob, so that a batch is one host->device copy
// (from pinned memory) and the device pointers are blob + offset.
enum PlanSec : int {
  PS_WIRE, PS_ARENA, PS_DEC, PS_ZR, PS_SC, PS_SCLIST, PS_VT, PS_G1, PS_G1P, PS_G2, PS_PR, PS_SEG, PS_HPRE,
  PS_HMAIN, PS_CK, PS_TX, PS_RND, PS_SC1, PS_SCPOST, PS_EMIT, PS_B64, PS_CP, PS_CP2, PS_OUT, PS_COUNT
};
static constexpr size_t WIRE_TAIL = 64;  // zero bytes after the wire pool (decode jobs may read past a short element)

// Where each per-thread piece lands in the flat plan.
struct PieceBase {
  size_t sec[PS_COUNT];               // element index (bytes for WIRE/ARENA/OUT) within each section
  uint32_t pts, scal, g1out, g2out;   // value-index bases
};

struct FlatPlan {
  size_t off[PS_COUNT] = {};  // byte offset of each section in the blob
  size_t cnt[PS_COUNT] = {};  // elements (bytes for WIRE / ARENA / OUT)
  size_t bytes = 0;           // blob size
  size_t upload = 0;          // host -> device bytes from the blob start: everything, or with
                              // dev_pools every section before ARENA (ARENA and OUT then come
                              // last and are written on the device; C_SIZE const bytes aside)
  bool dev_pools = false;
  size_t n_items = 0;
  uint32_t n_pts = 0, n_scal = 0, n_g1out = 0, n_g2out = 0;
  bool p2_g1out = false;      // prover plans: PairJob.p2 indexes g1out
  std::vector<PieceBase> base;
  std::vector<uint32_t> out_off;  // prover: per item start in OUT, plus the end
  std::vector<uint32_t> item_off; // openings: arena offset of each item's 128-byte result
  template <class T>
  T* ptr(uint8_t* blob, PlanSec s) const { return reinterpret_cast<T*>(blob + off[s]); }
};

// Reusable planning state of one batch slot: per-thread pieces keep their
// buffers between batches, so steady-state planning does not allocate.
struct PlanWork {
  std::vector<Plan> pieces;
  std::vector<std::string> errs;
  size_t used = 0;  // pieces of the current batch
};

// pieces a batch of n items is planned in (one per pool thread, >= 32 items each)
size_t plan_piece_count(size_t n, int threads);
// Plan n items into w's pieces (items split into contiguous ranges, one per
// piece, run on the pool).
void plan_items(const PPInfo& pp, size_t n, const PlanItem* items, PlanWork& w, WorkPool& pool);
// Offsets of every section and piece.  Returns "" or an error when a pool of
// the batch would overflow the 32-bit indices the device jobs use.
std::string flat_layout(const PlanWork& w, bool p2_g1out, FlatPlan& fp);
// Write the relocated pieces into blob (fp.bytes), the const region first:
// the caller's C_SIZE const bytes, the zero wire tail.  Parallel over pieces.
void flat_write(const PlanWork& w, const FlatPlan& fp, uint8_t* blob, const uint8_t* const_bytes, WorkPool& pool);

// Merged single-Plan form (test-only host emulation): plan, flatten and copy
// the sections back into `out`'s vectors (same relocation code as the device
// path).  Arena offsets are absolute: the const region occupies [0, C_SIZE).
void plan_transfers(const PPInfo& pp, size_t n, const TransferIn* tx, Plan& out, int threads);
void plan_issues(const PPInfo& pp, size_t n, const IssueIn* is, Plan& out, int threads);
void plan_unflatten(const FlatPlan& fp, const uint8_t* blob, Plan& out);
// Append b (indices local to b) to d with every index relocated (wire / arena
// first padded to 16 bytes); returns where b's sections landed in d.
PieceBase plan_append(Plan& d, const Plan& b);
void plan_items_merged(const PPInfo& pp, size_t n, const PlanItem* items, Plan& out, int threads);

// ------------------------------------------------------------------ prover
// Witness of one transfer / issue (token.TokenDataWitness: Type, Value,
// BlindingFactor; values and blinding factors as 32-byte big-endian Zr).
struct TransferWit {
  const uint8_t* inputs;   // n_in x 64-byte RawBytes
  uint32_t n_in;
  const uint8_t* outputs;  // n_out x 64-byte RawBytes
  uint32_t n_out;
  const uint8_t* in_values;
  const uint8_t* in_bfs;
  const uint8_t* out_values;
  const uint8_t* out_bfs;
  const char* type;
  size_t type_len;
  const uint8_t* seed;     // 32 bytes
};
struct IssueWit {
  const uint8_t* outputs;
  uint32_t n_out;
  const uint8_t* values;
  const uint8_t* bfs;
  const char* type;
  size_t type_len;
  uint8_t anonymous;
  const uint8_t* seed;
};
// Build prover plans (planner_prove.cpp).  Returns "" or the first witness
// error ("proof i: ...", e.g. a value outside [0, base^exponent)).
std::string plan_prove_transfers(const PPInfo& pp, size_t n, const TransferWit* w, Plan& out, int threads);
std::string plan_prove_issues(const PPInfo& pp, size_t n, const IssueWit* w, Plan& out, int threads);
// Piece form (the runtime's slots): returns "" or the first witness error.
std::string plan_prove_items_transfers(const PPInfo& pp, size_t n, const TransferWit* wit, PlanWork& w,
                                       WorkPool& pool);
std::string plan_prove_items_issues(const PPInfo& pp, size_t n, const IssueWit* wit, PlanWork& w, WorkPool& pool);

}  // namespace ftsh

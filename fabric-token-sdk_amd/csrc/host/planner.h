// Host planner: zkatdlog proof bytes -> flat GPU job arrays (see dev/jobs.h).
#pragma once
#include <stdint.h>

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
  std::vector<uint64_t> pow;                      // base^i, i < exponent
};
// Returns empty string on success, else an error message.
std::string parse_pp(const uint8_t* p, size_t n, const char* label, PPInfo& out);

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
  std::vector<uint8_t> out;       // outer proof JSON templates, concatenated
  std::vector<uint32_t> out_off;  // per proof: start in `out` (plus a final end)
  bool p2_g1out = false;          // PairJob.p2 indexes g1out (prover) instead of pts
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

// Build a plan for a batch (multi-threaded over proofs).  Arena offsets in the
// plan are absolute: the const region occupies [0, C_SIZE).
void plan_transfers(const PPInfo& pp, size_t n, const TransferIn* tx, Plan& out, int threads);
void plan_issues(const PPInfo& pp, size_t n, const IssueIn* is, Plan& out, int threads);

// Append piece b (indices local to b) to a, relocating every index.
void plan_merge(Plan& a, const Plan& b);

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

}  // namespace ftsh

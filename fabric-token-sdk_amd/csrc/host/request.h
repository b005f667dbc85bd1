// Host decoding of a raw zkatdlog token request:
//   * driver.TokenRequest (token/driver/request.go:24-38) as Go encoding/asn1
//     Unmarshal reads it (FromBytes, :35-38): a DER SEQUENCE of four SEQUENCE OF
//     OCTET STRING (Issues, Transfers, Signatures, AuditorSignatures);
//   * the actions inside it, Go encoding/json (gojson.h) into
//     transfer.TransferAction (crypto/transfer/sender.go:105-116, :179-181) and
//     issue.IssueAction (crypto/issue/issue.go:20-31, :89-91), with token.Token
//     (crypto/token/token.go:20-25) for outputs and for the ledger's inputs.
// The ZK verification of the decoded actions runs through the job engine
// (runtime: ftz_verify_token_requests).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace ftsh {

struct Slice {
  const uint8_t* p;
  size_t len;
};

// Go encoding/asn1 rules for this schema: definite, minimal lengths (long form
// only for >= 128, no leading zero bytes, < 2^31), identifier bytes exactly
// 0x30 (SEQUENCE) and 0x04 (primitive OCTET STRING), every element inside its
// parent; extra bytes after the four fields inside the outer SEQUENCE and after
// the outer SEQUENCE are ignored (Go allows both).  Returns "" or an error.
std::string der_token_request(const uint8_t* raw, size_t len, std::vector<Slice> out[4]);

// One decoded G1 element of an action (math.G1 UnmarshalJSON, deferred use).
struct ElemRef {
  uint8_t st;      // DecStatus: D_OK, D_NIL (JSON null -> nil pointer), D_PANIC (curve id != BN254)
  uint8_t bad;     // D_OK bytes that gnark SetBytes rejects for their length alone (short buffer)
  size_t off;      // 64-byte slot in the request's commitment pool (D_OK only)
};

struct ActionOut {
  bool nil_token = false;      // a JSON null entry in OutputTokens
  std::vector<ElemRef> data;   // OutputTokens[k].Data (nil token: st = D_NIL)
};

struct TransferAct {
  std::vector<std::string> inputs;  // Inputs (ledger keys)
  std::vector<ElemRef> in_coms;     // InputCommitments (decoded at unmarshal, unused by the verifier)
  ActionOut out;
  std::vector<uint8_t> proof;
  bool proof_nil = true;
};

struct IssueAct {
  ActionOut out;
  std::vector<uint8_t> proof;
  bool anonymous = false;
};

// Decoders: "" on success, else the reason the reference's json.Unmarshal
// fails.  Element bytes land in `pool` as 64-byte gnark slots (compressed
// encodings zero-padded; gnark SetBytes reads 32 bytes for them).
std::string dec_transfer_action(const uint8_t* p, size_t n, TransferAct& a, std::vector<uint8_t>& pool);
std::string dec_issue_action(const uint8_t* p, size_t n, IssueAct& a, std::vector<uint8_t>& pool);
// token.Token of a ledger input: "" and the Data element, or an error
std::string dec_token(const uint8_t* p, size_t n, ElemRef& data, std::vector<uint8_t>& pool);

}  // namespace ftsh

// ---- request-level ZK validation (Validator.VerifyTokenRequestFromRaw,
// crypto/validator/validator.go:45-108, without the signature / HTLC /
// metadata checks that stay in Go).  The device work goes through hooks so the
// test-only host emulation runs the same orchestration.
#include "../../../include/ftsamd.h"
#include <functional>

namespace ftsh {

// calling-thread time per pipeline stage, ms (optional, RequestHooks.stats)
struct RequestStats {
  double decode = 0, check = 0, lookup = 0, tokens = 0, build = 0, drain = 0;
};

struct RequestHooks {
  // gnark SetBytes check of n 64-byte element slots: ok[i] = 1 / 0; FTZ_SUCCESS or an API error
  std::function<int(size_t n, const uint8_t* slots, uint8_t* ok)> check;
  // thread-safe: called from helper threads, several requests in flight at once
  std::function<int(size_t n, const ftz_transfer* tx, int32_t* codes)> verify_transfers;
  std::function<int(size_t n, const ftz_issue* is, int32_t* codes)> verify_issues;
  // ledger: one key at a time (get_state) or a chunk's keys in one call
  // (get_states, preferred when set); both on the calling thread only
  ftz_get_state_fn get_state = nullptr;
  ftz_get_states_fn get_states = nullptr;
  void* user = nullptr;
  // parallel for over [0, k) (decoding); unset: serial on the calling thread
  std::function<void(size_t k, const std::function<void(size_t)>& f)> par;
#ifndef FTS_REQ_CHUNK
#define FTS_REQ_CHUNK 4096
#endif
#ifndef FTS_REQ_INFLIGHT
#define FTS_REQ_INFLIGHT 8
#endif
  size_t chunk = FTS_REQ_CHUNK;        // requests decoded per pipeline step
  size_t inflight = FTS_REQ_INFLIGHT;  // chunks whose ZK verification may be in flight at once
  RequestStats* stats = nullptr;
};

// codes[r]: FTZ_OK or the first failing check of request r in the reference's
// order; failed[r] (optional): the failing action's index (issues first, then
// transfers), -1 for a request-level failure or none.  Returns FTZ_SUCCESS or
// an API error (err set).
//
// Pipelined over chunks of h.chunk requests: chunk k+1 is decoded (h.par), its
// elements checked (h.check) and its ledger inputs loaded (get_state(s), the
// calling thread) while the ZK verification of chunks k, k-1, ... runs in the
// job engine (h.verify_*, one helper thread per chunk and action kind).
int verify_token_requests(size_t n, const ftz_bytes* reqs, const RequestHooks& h, int32_t* codes, int32_t* failed,
                          std::string& err);

}  // namespace ftsh

/* ftsamd -- MI355X batch verifier for the zkatdlog (nogh) driver of the
 * Fabric Token SDK.  C ABI: plain pointers and sizes, no torch / HIP types.
 *
 * Reference interfaces this boundary replaces (paths relative to
 * /root/reference/token/core/zkatdlog/):
 *   ftz_ctx_create        crypto/setup.go:134-151   PublicParams.Deserialize (+ Validate :238-273)
 *                         nogh/driver/driver.go:114-124 Driver.NewValidator (PP parsed once per process)
 *   ftz_verify_transfers  crypto/transfer/transfer.go:66-77,124-154
 *                         transfer.NewVerifier(inputs, outputs, pp).Verify(proof)
 *                         as called by crypto/validator/validator_transfer.go:84-98
 *                         TransferZKProofValidate (inputs = ledger commitments)
 *   ftz_verify_issues     crypto/issue/issue.go:194-223
 *                         issue.NewVerifier(tokens, anonymous, pp).Verify(proof)
 *                         as called by crypto/validator/validator.go:181-191 verifyIssue
 * The Go error classes map to the FTZ_ERR_* codes below; a proof on which the
 * reference would panic (nil dereference, foreign curve id) is reported as
 * FTZ_ERR_PANIC (reject) instead of crashing the process.
 *
 * Thread-safety and batching: a context may be used from any number of
 * threads.  ftz_verify_transfers / ftz_verify_issues are synchronous for the
 * caller but go through one job engine per context: a call of any size is cut
 * into device batches of at most `batch` proofs (planned on host threads while
 * earlier batches run on the GPU, `slots` batches in flight), and concurrent
 * small calls -- the Go shim verifies one TransferAction per call
 * (validator_transfer.go:84-98) -- are coalesced into shared batches
 * (micro-batching).  Results are delivered per call.
 */
#ifndef FTSAMD_H
#define FTSAMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* per-proof verdict codes (0 = accept) */
#define FTZ_OK 0
#define FTZ_ERR_PARSE 1      /* json / base64 / element decoding failed            */
#define FTZ_ERR_MALFORMED 2  /* "not well formed", nil fields, length mismatches    */
#define FTZ_ERR_WF 3         /* "invalid zero-knowledge transfer" / issue WF        */
#define FTZ_ERR_RANGE 4      /* "invalid range proof"                               */
#define FTZ_ERR_MEMBERSHIP 5 /* "invalid membership proof"                          */
#define FTZ_ERR_PANIC 6      /* the reference would panic on this proof             */
#define FTZ_ERR_OPENING 7    /* audit: "output ... does not match the provided opening" */
/* 8 = FTZ_ERR_INPUT (token requests, below) */

/* API return codes */
#define FTZ_SUCCESS 0
#define FTZ_E_INVALID (-1) /* bad argument                                         */
#define FTZ_E_PP (-2)      /* public parameters rejected                            */
#define FTZ_E_DEVICE (-3)  /* no usable MI355X / HIP error (see ftz_last_error)     */
#define FTZ_E_NOMEM (-4)

typedef struct ftz_ctx ftz_ctx;
typedef struct ftz_batch ftz_batch;

/* One transfer action: commitments are 64-byte gnark G1 RawBytes (X||Y). */
typedef struct {
  const uint8_t* inputs; /* n_in  x 64 bytes: input token commitments (ledger)   */
  uint32_t n_in;
  const uint8_t* outputs; /* n_out x 64 bytes: output token commitments          */
  uint32_t n_out;
  const uint8_t* proof; /* json(transfer.Proof) as carried in TransferAction.Proof */
  size_t proof_len;
} ftz_transfer;

typedef struct {
  const uint8_t* outputs; /* n_out x 64 bytes: issued token commitments          */
  uint32_t n_out;
  const uint8_t* proof; /* json(issue.Proof)                                      */
  size_t proof_len;
  uint8_t anonymous; /* IssueAction.Anonymous                                     */
} ftz_issue;

/* Per-kernel timing of the last ftz_batch_run (HIP events on the batch stream). */
#define FTZ_NKERNELS 12
typedef struct {
  /* decode, zr, hash_pre, scalar, g1_pairing, g2 + pair-2 lines (stream 3), miller, fexp, g1_side (stream 2), hash,
   * verdict, total */
  float ms[FTZ_NKERNELS];
  uint64_t jobs[FTZ_NKERNELS];
} ftz_stats;

/* Final exponentiation variant [EXT] (GT bytes feed every
 * membership transcript, sigproof/membership.go:247,260-277):
 *   FTZ_FEXP_EXACT    f^((p^12-1)/r) -- the Scott et al. (ePrint 2008/490) hard
 *                     part of gnark-crypto v0.6.0 (go.mod:53), the default;
 *   FTZ_FEXP_FUENTES  f^(2x(6x^2+3x+1)(p^12-1)/r) -- the Fuentes-Castaneda et al.
 *                     chain later gnark-crypto releases use. */
#define FTZ_FEXP_EXACT 0
#define FTZ_FEXP_FUENTES 1

typedef struct {
  uint32_t struct_size; /* sizeof(ftz_options)                                          */
  uint32_t batch;       /* max proofs per device batch (default 8192: 4096 leaves the
                           pairing kernels at 1.6 sextet waves per SIMD, profiles/r02g_*) */
  uint32_t slots;       /* batch slots of the job engine = batches in flight (default 4;
                           measured best of 4/5/6/8, profiles/r02_slots_sweep.txt)      */
  uint32_t window_us;   /* micro-batching: how long a partial batch may wait for more
                           callers while the GPU is busy (default 1000; seam sweep,
                           profiles/r03k/seamsweep.jsonl)                                */
  uint32_t threads;     /* host planning threads (0: min(16, hardware threads))         */
  uint32_t fexp;        /* FTZ_FEXP_EXACT (default) or FTZ_FEXP_FUENTES                 */
  uint32_t hold_inflight; /* a partial batch waits (up to window_us) for more callers
                           only while at least this many batches are in flight
                           (default 2; 0: always, also with the GPU idle -- closed-loop
                           callers resubmit together; FTZ_HOLD_NEVER: ship at once)       */
  uint32_t small_pass;  /* device passes of at most this many G2 jobs run the low-latency
                           layout of the t' / pair-2 line stage (six lanes per job
                           instead of one; same bytes); default 4096, 0 = never; an
                           explicit ftz_ctx_set_layout(FTZ_STAGE_G2LINES) overrides it  */
  uint32_t msm_window_bits; /* MSM planner overrides (ftz_msm_*), 0 = the planner's choice: */
  uint32_t msm_slot_cap;    /*   window bits c, bucket slot cap T, slots per segment S    */
  uint32_t msm_seg_slots;
  uint32_t msm_glv;     /* 1 (default): GLV-split scalars in the MSM; 0: plain 256-bit   */
  uint32_t msm_precompute; /* 1: resident-point MSM -- ftz_msm_load also stores 2^(c w) P
                           for every window w (W x the point memory) and runs use one shared
                           bucket set and no Horner chain; for fixed bases (ftz_msm_set_scalars)
                           0 (default): plain variable-base Pippenger                      */
  uint32_t prover_tables; /* 1 (default): the first ftz_prove_* call builds fixed-base tables
                           of the PP's digit signatures R_d, S_d (32 MB per point with
                           16-bit windows: 2 x base x 32 MB, 6.4 GB at base 100, once per
                           context) and proves through them and fixed-G2 pairings; if
                           that allocation fails the context proves on the
                           variable-base path instead (same bytes, slower) and does not
                           retry.  0: never build them (variable-base path).            */
  uint32_t msm_radix_bits; /* MSM sort digit bits per radix pass: 0 = the planner's choice
                           (9 where it saves a pass, else 8), or 8 / 9                   */
  uint32_t first_pass;  /* proofs in a pass dispatched while no pass is in flight (the
                           start of a job): default 4096, 0 = batch.  A smaller first
                           pass reaches the device after half the planning step: a
                           20-step bench job 707k -> 725k transfers/s (mean of 4 on one
                           box, profiles/r05/first_pass_ab.txt)                        */
  uint32_t tail_split;  /* the last pass of the queue (pending <= batch) is cut in two
                           halves of at least this many proofs, whose kernel chains then
                           overlap: 0 (default) = off (measured no gain on the 20-step
                           job, profiles/r05/tail_split_ab.txt)                         */
  uint32_t msm_graph;   /* 1: ftz_msm_run replays its launch chain (keys, sort, bucket,
                           segment, tree and Horner kernels) as one HIP graph captured on
                           the handle's first run; 0 (default): direct launches (the
                           graph measured the same: 2^16 0.92-0.93 ms either way,
                           profiles/r06/msm_graph.txt)                                   */
  uint32_t request_threads; /* threads decoding token requests (ftz_verify_token_requests*;
                           0 = threads): they share the host's cores with the planning
                           threads that feed the device                                  */
} ftz_options;
#define FTZ_HOLD_NEVER 0xFFFFFFFFu
void ftz_options_default(ftz_options* opt);

/* pp: json(driver.SerializedPublicParameters{Identifier:"zkatdlog", Raw}) as
 * produced by crypto.PublicParams.Serialize (setup.go:119-128) and read by
 * PublicParams.Deserialize (setup.go:134-151) + Validate (setup.go:238-273).
 * device: HIP device ordinal (the local rank in a multi-GPU job). */
int ftz_ctx_create(const uint8_t* pp, size_t pp_len, int device, ftz_ctx** out);
int ftz_ctx_create_ex(const uint8_t* pp, size_t pp_len, int device, const ftz_options* opt, ftz_ctx** out);
/* Call only when no other call on the context is running. */
void ftz_ctx_destroy(ftz_ctx* ctx);
/* last error message of the calling thread (empty string if none) */
const char* ftz_last_error(void);
/* number of host threads used to plan a batch; only before the first
 * ftz_verify_* call on the context (FTZ_E_INVALID afterwards) */
int ftz_ctx_set_threads(ftz_ctx* ctx, int threads);
/* profiling: 1 = run every kernel of a batch on one stream (per-kernel times
 * without overlap), 0 = the normal three-stream schedule */
int ftz_ctx_set_serial(ftz_ctx* ctx, int serial);
/* testing the job engine's failure isolation: planning a device pass that
 * holds an item whose proof pointer equals `proof` fails (FTZ_E_INVALID,
 * "poisoned item"), as a planner limit would; NULL clears it.  The engine must
 * then deliver that error to the one request holding the item and the right
 * codes to every other caller whose items shared the pass. */
int ftz_ctx_debug_poison(ftz_ctx* ctx, const uint8_t* proof);
/* parity debugging: with FTZ_DEBUG_CHALLENGES set, batches loaded afterwards
 * (ftz_batch_load_*) keep every recomputed Fiat-Shamir challenge -- the
 * HashToZr of each well-formedness, membership and range transcript
 * (transfer/wellformedness.go, sigproof/membership.go:260-277,
 * range/proof.go:371-389) -- whether or not it matches the proof's claim.  Set
 * it before any call plans on the context; 0 clears it. */
#define FTZ_DEBUG_CHALLENGES 1
int ftz_ctx_set_debug(ftz_ctx* ctx, int flags);
/* profiling: kernel layout of a pipeline stage (results are identical; only
 * speed differs).  stage FTZ_STAGE_G2LINES (the verifier's t' = c PK0 + v PK1
 * + h PK2 and its 88 pair-2 Miller lines; default one lane) or
 * FTZ_STAGE_PROVER_G2LINES (the prover's t = rv PK1 + rh PK2 and its lines at
 * R'; default sextet); layout FTZ_LAYOUT_ONE_LANE (one lane per job) or
 * FTZ_LAYOUT_SEXTET (six lanes per job, ten jobs per wave). */
#define FTZ_STAGE_G2LINES 0
#define FTZ_STAGE_PROVER_G2LINES 1
#define FTZ_LAYOUT_ONE_LANE 1
#define FTZ_LAYOUT_SEXTET 6
int ftz_ctx_set_layout(ftz_ctx* ctx, int stage, int layout);
/* crypto.PublicParams.Validate (setup.go:238-273) on serialized public
 * parameters, as the FSC node's loader runs it (nogh/loaders.go:133):
 * FTZ_SUCCESS, or FTZ_E_PP with the reference's error text in
 * ftz_last_error().  Point encodings are checked by ftz_ctx_create. */
int ftz_pp_validate(const uint8_t* pp, size_t pp_len);
/* crypto.Setup (setup.go:214-236: pssign KeyGen(1), GeneratePedersenParameters
 * :153-166, GenerateRangeProofParameters :168-184 with the R = generator quirk of
 * pssign/sign.go:97-98, QuantityPrecision 64) followed by Serialize
 * (setup.go:119-128): out receives json(driver.SerializedPublicParameters) for
 * SignedValues of 0..base-1 and the given Exponent / IdemixIssuerPK (NULL: JSON
 * null) / IdemixCurveID.  The reference draws its scalars from crypto/rand;
 * here rand(tag) = SHA-256(seed||tag||0) || SHA-256(seed||tag||1) mod r, so a
 * seed reproduces a parameter set.  Host-side (once per network): no context
 * or GPU needed.  *out_len = the size; FTZ_E_INVALID if cap is too small. */
int ftz_pp_setup(uint64_t base, uint32_t exponent, const uint8_t* idemix_pk, size_t idemix_pk_len, int idemix_curve,
                 const uint8_t* seed, size_t seed_len, uint8_t* out, size_t cap, size_t* out_len);
/* the context's resolved options (threads, batch, slots, window, fexp) */
int ftz_ctx_options(const ftz_ctx* ctx, ftz_options* out);
/* PP properties: base (len(SignedValues)) and exponent */
int ftz_ctx_info(const ftz_ctx* ctx, uint32_t* base, uint32_t* exponent);

/* Verify n proofs (any n: large calls are split into device batches and
 * pipelined, small concurrent calls share batches); codes[i] receives FTZ_OK
 * or an FTZ_ERR_* class. */
int ftz_verify_transfers(ftz_ctx* ctx, size_t n, const ftz_transfer* tx, int32_t* codes);
int ftz_verify_issues(ftz_ctx* ctx, size_t n, const ftz_issue* is, int32_t* codes);

/* Job-engine counters since context creation (or the last reset): device
 * batches, proofs, host planning time (parse + layout into the pinned staging
 * blob), enqueue time (H2D copy + kernel launches), device time per batch
 * (HIP events from the H2D copy to the verdict download), and the caller-side
 * wait of the completion thread. */
typedef struct {
  uint64_t batches;
  uint64_t proofs;
  double plan_ms;    /* sum over batches */
  double submit_ms;  /* sum over batches */
  double device_ms;  /* sum over batches, upload -> verdicts downloaded */
  double wall_ms;    /* first submission -> last completion */
  uint32_t max_in_flight;
} ftz_engine_stats;
int ftz_ctx_engine_stats(ftz_ctx* ctx, ftz_engine_stats* out, int reset);

/* Host-side time of ftz_prove_transfers / ftz_prove_issues since context
 * creation (or the last reset), summed over device passes: waiting for a pass
 * to finish, copying its proofs into the caller's buffer, planning + flattening
 * the next pass into pinned staging, and enqueueing it (H2D copy + launches). */
typedef struct {
  uint64_t passes;
  uint64_t proofs;
  double wait_ms;
  double copy_ms;
  double plan_ms;
  double submit_ms;
  double wall_ms;    /* sum over calls, entry -> return */
} ftz_prover_host_stats;
int ftz_ctx_prover_stats(ftz_ctx* ctx, ftz_prover_host_stats* out, int reset);

/* Staged form: plan + upload once, then run the GPU pipeline on resident
 * inputs any number of times (used by bench.py to time the device path).
 * One staged batch is one device pass: n must keep every job pool of the
 * batch below 2^31 entries / bytes (FTZ_E_INVALID otherwise; a 2-in/2-out
 * PP-A transfer uses ~4 KB of arena, so up to ~500k transfers). */
int ftz_batch_load_transfers(ftz_ctx* ctx, size_t n, const ftz_transfer* tx, ftz_batch** out);
int ftz_batch_load_issues(ftz_ctx* ctx, size_t n, const ftz_issue* is, ftz_batch** out);
int ftz_batch_run(ftz_batch* b); /* = ftz_batch_submit + ftz_batch_wait */
/* Asynchronous form: enqueue the pipeline on the batch's own HIP streams and
 * return; several batches may be in flight at once (a validator pipelining
 * blocks).  ftz_batch_wait blocks until the batch's last submission is done
 * and records its ftz_stats; codes/bitmap wait implicitly.  A batch must not
 * be resubmitted before its previous submission was waited for. */
int ftz_batch_submit(ftz_batch* b);
int ftz_batch_wait(ftz_batch* b);
int ftz_batch_codes(ftz_batch* b, int32_t* codes);
/* verdict bitmap: bit i set <=> proof i accepted; (n+7)/8 bytes */
int ftz_batch_bitmap(ftz_batch* b, uint8_t* bits);
int ftz_batch_stats(const ftz_batch* b, ftz_stats* out);
size_t ftz_batch_size(const ftz_batch* b);
void ftz_batch_destroy(ftz_batch* b);
/* the recomputed challenges of proof i of a batch loaded with
 * FTZ_DEBUG_CHALLENGES, after ftz_batch_run: one per transcript the planner
 * scheduled, in check order -- well-formedness (FTZ_ERR_WF), then every
 * membership proof in (output, digit) order (FTZ_ERR_MEMBERSHIP), then the
 * range proof (FTZ_ERR_RANGE) -- as kinds[k] and 32-byte big-endian values at
 * values + 32 k.  *count = the number available (entries beyond cap are not
 * written).  A proof rejected before its transcripts are planned has none. */
int ftz_batch_challenges(ftz_batch* b, size_t i, int32_t* kinds, uint8_t* values, size_t cap, size_t* count);

/* ---- token commitments and auditor opening checks.
 * A token opening is token.TokenDataWitness{Type, Value, BlindingFactor}
 * (crypto/token/token.go): value and bf as 32-byte big-endian Zr.  The
 * commitment is H(type)*Ped0 + value*Ped1 + bf*Ped2 with H = HashToZr
 * (computeTokens, token/token.go:64-76; common/schnorr.go:59-76).  Note
 * GetTokensWithWitness (token.go:78-98) takes uint64 values through
 * NewZrFromInt(int64(v)): a caller passes that Zr (v mod r for v < 2^63). */
typedef struct {
  const char* type;
  size_t type_len;
  const uint8_t* value; /* 32 bytes */
  const uint8_t* bf;    /* 32 bytes */
} ftz_token_opening;
/* out: n x 64-byte RawBytes commitments */
int ftz_commit_tokens(ftz_ctx* ctx, size_t n, const ftz_token_opening* t, uint8_t* out);
/* Auditor InspectOutput / InspectInputs commitment check (audit/auditor.go:208-234):
 * codes[i] = FTZ_OK if commitments[i] (64-byte RawBytes, gnark decoding rules)
 * equals the recomputed commitment of t[i], FTZ_ERR_OPENING if it does not,
 * FTZ_ERR_PARSE if the bytes are not a valid G1 encoding.  (The owner
 * identity check InspectTokenOwnerFunc is idemix, outside this library.) */
int ftz_audit_openings(ftz_ctx* ctx, size_t n, const uint8_t* commitments, const ftz_token_opening* t,
                       int32_t* codes);

/* ---- raw token requests (the wire format around the path).
 * A request is asn1.Marshal(driver.TokenRequest{Issues, Transfers, Signatures,
 * AuditorSignatures [][]byte}) (token/driver/request.go:24-38). */
typedef struct {
  const uint8_t* p;
  size_t len;
} ftz_bytes;
/* Go encoding/asn1 decoding as TokenRequest.FromBytes does it (request.go:35-38):
 * counts[0..3] = len(Issues), len(Transfers), len(Signatures), len(AuditorSignatures);
 * elems[0 .. sum(counts)) receive the byte slices in that order, pointing into
 * raw (when cap is large enough).  FTZ_SUCCESS, or FTZ_E_INVALID for bytes
 * the reference rejects (message in ftz_last_error) or a too small cap. */
int ftz_token_request_decode(const uint8_t* raw, size_t len, size_t counts[4], ftz_bytes* elems, size_t cap);
/* Ledger lookup (driver.GetStateFnc, validator.go:45; the Go shim passes a cgo
 * export over getState): 0 and *val / *val_len (valid until the next call on
 * the same thread), or non-zero when the state cannot be read.  Called on the
 * thread that called ftz_verify_token_requests only, never concurrently; the
 * library copies each value before the next call. */
typedef int (*ftz_get_state_fn)(void* user, const char* key, size_t key_len, const uint8_t** val, size_t* val_len);
/* Batched ledger lookup (one cgo crossing per pipeline chunk instead of one per
 * input): vals[i] = the value of keys[i], {NULL, 0} when it does not exist.
 * Returns 0, or non-zero when the states cannot be read (every transfer with
 * an input in this call then fails with FTZ_ERR_INPUT, as a GetState error
 * does).  Called on the thread that called ftz_verify_token_requests_batched
 * only, never concurrently; the values must stay valid until the next
 * get_states call or the return of ftz_verify_token_requests_batched (the
 * library copies them before either).  The Go side may look the keys up
 * concurrently itself. */
typedef int (*ftz_get_states_fn)(void* user, size_t n, const ftz_bytes* keys, ftz_bytes* vals);
#define FTZ_ERR_INPUT 8 /* an input to spend is missing on the ledger or is not a token.Token */
/* ZK validation of n raw token requests as Validator.VerifyTokenRequestFromRaw
 * performs it (crypto/validator/validator.go:45-108) minus the checks that stay
 * in Go (auditor / issuer / owner signatures, HTLC scripts, metadata counting):
 * ASN.1 and action JSON decoding (a failure rejects the whole request with
 * FTZ_ERR_PARSE, as unmarshalIssueActions / unmarshalTransferActions do), then
 * every issue action (issue.Verifier) and every transfer action (inputs loaded
 * through get_state and decoded as token.Token -- FTZ_ERR_INPUT --, then
 * transfer.Verifier) in order; all actions of all requests are verified in
 * shared device batches.  codes[i] = FTZ_OK or the first failing check of
 * request i; failed_action (may be NULL) = that action's index (issues first,
 * then transfers), -1 if none or request-level.
 * Pipelined: requests are decoded on the library's own host threads in chunks,
 * and while chunk k's actions are verified on the device, chunk k+1 is decoded
 * and its inputs looked up (on the calling thread).  Thread-safe: calls on one
 * context from several threads share the device batches. */
int ftz_verify_token_requests(ftz_ctx* ctx, size_t n, const ftz_bytes* reqs, ftz_get_state_fn get_state, void* user,
                              int32_t* codes, int32_t* failed_action);
/* The same with the batched ledger lookup (recommended for block-level
 * binding: one callback per pipeline chunk of up to 4096 requests). */
int ftz_verify_token_requests_batched(ftz_ctx* ctx, size_t n, const ftz_bytes* reqs, ftz_get_states_fn get_states,
                                      void* user, int32_t* codes, int32_t* failed_action);
/* profiling: the calling thread's time in each stage of the request pipeline,
 * summed over the context's ftz_verify_token_requests* calls, in ms: ms[0]
 * decode (ASN.1 + action JSON, parallel), [1] element checks (device), [2]
 * ledger callbacks, [3] token decoding (parallel), [4] job building, [5]
 * waiting for the verdicts of earlier chunks; reset != 0 zeroes them after. */
int ftz_ctx_request_stats(ftz_ctx* ctx, double ms[6], int reset);

/* ---- idemix owner signatures, on BN254 or FP256BN_AMCL.
 * Replaces, per input token of a transfer, what TransferSignatureValidate
 * (crypto/validator/validator_transfer.go:42-82) runs after loading the token:
 * ctx.Deserializer.GetOwnerVerifier(tok.Owner) (nogh/deserializer.go:64-66 ->
 * interop/htlc/deserializer.go:31-43 -> identity/owner.go:62-68 ->
 * identity/msp/idemix/deserializer.go:83-95, common.go:40-117) and
 * verifier.Verify(message, sigma) (common/backend.go:32-41 ->
 * identity/msp/idemix/deserializer.go:153-163 -> IBM/idemix NymSignature.Ver):
 * owner = the token's Owner bytes (ASN.1 RawOwner), msg = the signed request
 * bytes, sig = the NymSignature proto.  ftz_idemix_create takes
 * PublicParams.IdemixIssuerPK (setup.go:36) -- the IssuerPublicKey proto -- and
 * PublicParams.IdemixCurveID, which selects the translator as
 * identity/msp/idemix/deserializer.go:40-51 does: FTZ_CURVE_BN254 (1, the
 * curve cmd/pp/dlog/gen.go:117 and every NWO topology deploy: gurvy
 * translator, gnark point decoding, 64-byte G1 in the transcript) or
 * FTZ_CURVE_FP256BN_AMCL (0, amcl translator).  The IPK's own proof is checked
 * once by the Go deserializer (NewDeserializer) and is not re-checked here; an
 * IPK whose HSk / HRand do not decode on the curve, or are the point at
 * infinity, is refused with FTZ_E_PP. */
#define FTZ_ERR_OWNER 9        /* the owner identity does not deserialize (RawOwner, idemix identity, nym) */
#define FTZ_ERR_SIGNATURE 10   /* the signature does not unmarshal, or "pseudonym signature invalid"       */
#define FTZ_ERR_UNSUPPORTED 11 /* owner type verified in Go (an HTLC script owner)                          */
#define FTZ_ERR_AUDIT 12       /* the token owner does not match its audit info (AuditInfo.Match failed)    */
#define FTZ_CURVE_FP256BN_AMCL 0
#define FTZ_CURVE_BN254 1
typedef struct ftz_idemix ftz_idemix;
typedef struct {
  const uint8_t* owner; /* token.Token.Owner: asn1(RawOwner{Type, Identity})                  */
  size_t owner_len;
  const uint8_t* msg;   /* the signed message (request bytes || anchor)                        */
  size_t msg_len;
  const uint8_t* sig;   /* proto(NymSignature)                                                 */
  size_t sig_len;
} ftz_owner_sig;
int ftz_idemix_create(ftz_ctx* ctx, const uint8_t* ipk, size_t ipk_len, int curve_id, ftz_idemix** out);
/* codes[i] = FTZ_OK, FTZ_ERR_OWNER, FTZ_ERR_SIGNATURE or FTZ_ERR_UNSUPPORTED; thread-safe */
int ftz_verify_owner_signatures(ftz_idemix* ix, size_t n, const ftz_owner_sig* s, int32_t* codes);
/* Strict nym import (opt-in, default off; FP256BN only -- on BN254 gnark's
 * SetBytes already refuses an off-curve nym, FTZ_ERR_OWNER).  amcl NewECPbigs turns an off-curve
 * NymX/NymY into the point at infinity [EXT, unpinned: amcl is not in the
 * reference], and NymSignature.Ver then accepts a signature made against the
 * identity without any secret; parity with that reading is the default.  With
 * on != 0 an off-curve nym is FTZ_ERR_OWNER before any curve arithmetic (a
 * deliberate deviation from the reference, for deployments that prefer to
 * reject until the amcl behaviour is confirmed).  Applies to later calls. */
int ftz_idemix_set_strict_nym(ftz_idemix* ix, int on);
void ftz_idemix_destroy(ftz_idemix* ix);

/* Auditor owner inspection (the owner half of
 * crypto/audit/auditor.go:208-274 InspectOutput / InspectInputs ->
 * InspectTokenOwner): the idemix matcher of the token's OwnerInfo
 * (identity/msp/idemix/audit.go:32-46 DeserializeAuditInfo, Go encoding/json)
 * checks the owner identity (audit.go:51-83 AuditInfo.Match ->
 * CSP.Verify(EidNymAuditOpts) -> IBM/idemix AuditNymEid [EXT]:
 * HAttrs[2]^HashToZr(Attributes[2]) * HRand^RNymEid == the identity proof's
 * EidNym).  codes: FTZ_OK, FTZ_ERR_OWNER (redeem token, empty OwnerInfo,
 * undecodable RawOwner or audit info), FTZ_ERR_AUDIT (Match failed),
 * FTZ_ERR_UNSUPPORTED (a script owner: inspected in Go), FTZ_ERR_PANIC. */
typedef struct {
  const uint8_t* owner;      /* token.Token.Owner: asn1(RawOwner{Type, Identity}) */
  size_t owner_len;
  const uint8_t* audit_info; /* the owner's OwnerInfo: json(AuditInfo)           */
  size_t audit_info_len;
} ftz_owner_audit;
int ftz_audit_owners(ftz_idemix* ix, size_t n, const ftz_owner_audit* items, int32_t* codes);

/* ---- standalone BN254 G1 multi-scalar multiplication (BASELINE configs[2]):
 * out = sum_i k_i P_i as 64-byte gnark RawBytes.  Points: n x 64-byte
 * uncompressed RawBytes (must be canonical and on the curve); scalars: n x 32
 * bytes big-endian, reduced mod r.  The reference path has no MSM; this is the
 * operation mathlib exposes from gnark-crypto as G1Jac.MultiExp.  Pippenger
 * with signed windows over GLV half-scalars (k = k1 + k2 lambda, |k_i| < 2^128,
 * points P_i and phi(P_i)), c = floor(log2(2n) / 2) + 7 clamped to [8, 20].
 * Sizes: n in [1, 2^28], and windows x 2n < 2^30 sort entries (n up to
 * ~2^26; FTZ_E_INVALID beyond), or windows x 2n < 2^31 resident points with
 * msm_precompute. */
typedef struct ftz_msm ftz_msm;
int ftz_msm_g1(ftz_ctx* ctx, size_t n, const uint8_t* points, const uint8_t* scalars, uint8_t out[64]);
/* staged form: upload once, run on HBM-resident inputs (bench) */
int ftz_msm_load(ftz_ctx* ctx, size_t n, const uint8_t* points, const uint8_t* scalars, ftz_msm** out);
/* test/bench inputs with known discrete logs: P_i = (i + offset) G generated on the device */
int ftz_msm_load_gen(ftz_ctx* ctx, size_t n, uint32_t offset, const uint8_t* scalars, ftz_msm** out);
int ftz_msm_run(ftz_msm* m, uint8_t out[64]);
/* replace the scalars of a loaded MSM (n x 32 bytes big-endian); the points, and
 * with msm_precompute their window multiples, stay resident */
int ftz_msm_set_scalars(ftz_msm* m, const uint8_t* scalars);
/* set the scalars and run in one call, for scalars that start in host memory:
 * the 32n bytes are copied in chunks on a copy stream while the key kernel of
 * the chunks already on the device runs (big-endian -> reduced limbs -> GLV
 * halves -> window digits in one pass), then the rest of ftz_msm_run.  The
 * scalars stay loaded, as with ftz_msm_set_scalars.  Page-locked memory
 * (ftz_host_alloc) copies at the full link rate. */
int ftz_msm_run_scalars(ftz_msm* m, const uint8_t* scalars, uint8_t out[64]);
/* page-locked host memory for staging large inputs (scalars, proof bytes) */
int ftz_host_alloc(size_t bytes, void** out);
void ftz_host_free(void* p);
/* device time of the last ftz_msm_run in ms (HIP events) and the window size */
int ftz_msm_info(const ftz_msm* m, float* last_ms, uint32_t* window_bits);
void ftz_msm_destroy(ftz_msm* m);
/* Sum of n <= 4096 RawBytes G1 points (the identity = 64 zero bytes accepted):
 * the final add of a point-split multi-GPU MSM: each rank runs
 * ftz_msm_g1 on its contiguous slice of the points, the 64-byte partials are
 * all-gathered (RCCL), and every rank sums them here (zkatdlog/dist.py msm_shard). */
int ftz_g1_sum(ftz_ctx* ctx, size_t n, const uint8_t* points, uint8_t out[64]);

/* ---- batch prover (BASELINE configs[4]).
 * Replaces transfer.NewProver(inW, outW, in, out, pp).Prove()
 * (token/core/zkatdlog/crypto/transfer/transfer.go:42,89-121) and
 * issue.NewProver(...).Prove() (crypto/issue/issue.go:151,162-184): the proof
 * JSON bytes, byte-identical to the reference's encoding.  Witnesses follow
 * token.TokenDataWitness (crypto/token/token.go): Value and BlindingFactor as
 * 32-byte big-endian Zr.  Randomness: the reference draws from crypto/rand;
 * here every random scalar is SHA-256(seed||tag||0)||SHA-256(seed||tag||1) mod r
 * from a caller-supplied 32-byte seed per proof (the Go shim passes 32 bytes of
 * crypto/rand), so proofs are reproducible for testing.  A value outside
 * [0, base^exponent) fails the load with FTZ_E_INVALID ("can't compute range
 * proof: value of token outside authorized range", range/proof.go:300-302). */
typedef struct {
  const uint8_t* inputs;     /* n_in x 64-byte RawBytes (ledger input commitments) */
  uint32_t n_in;
  const uint8_t* outputs;    /* n_out x 64-byte RawBytes (output commitments)      */
  uint32_t n_out;
  const uint8_t* in_values;  /* n_in x 32-byte BE Zr                               */
  const uint8_t* in_bfs;     /* n_in x 32-byte BE Zr                               */
  const uint8_t* out_values; /* n_out x 32-byte BE Zr                              */
  const uint8_t* out_bfs;    /* n_out x 32-byte BE Zr                              */
  const char* type;          /* token type (TokenDataWitness.Type)                 */
  size_t type_len;
  const uint8_t* seed;       /* 32 bytes                                           */
} ftz_transfer_witness;
typedef struct {
  const uint8_t* outputs;    /* n_out x 64-byte RawBytes (issued commitments)      */
  uint32_t n_out;
  const uint8_t* values;     /* n_out x 32-byte BE Zr                              */
  const uint8_t* bfs;        /* n_out x 32-byte BE Zr                              */
  const char* type;
  size_t type_len;
  uint8_t anonymous;
  const uint8_t* seed;       /* 32 bytes                                           */
} ftz_issue_witness;
typedef struct ftz_prover ftz_prover;
/* one call: proofs concatenated into buf (cap bytes; ftz_prover_bytes tells the
 * size), offsets[n+1] delimit proof i; codes[i] = FTZ_ERR_PARSE if a commitment
 * of proof i does not decode, else FTZ_OK */
int ftz_prove_transfers(ftz_ctx* ctx, size_t n, const ftz_transfer_witness* w, uint8_t* buf, size_t cap,
                        size_t* offsets, int32_t* codes);
int ftz_prove_issues(ftz_ctx* ctx, size_t n, const ftz_issue_witness* w, uint8_t* buf, size_t cap,
                     size_t* offsets, int32_t* codes);
/* staged form: plan + upload once, run on HBM-resident witnesses (bench) */
int ftz_prover_load_transfers(ftz_ctx* ctx, size_t n, const ftz_transfer_witness* w, ftz_prover** out);
int ftz_prover_load_issues(ftz_ctx* ctx, size_t n, const ftz_issue_witness* w, ftz_prover** out);
int ftz_prover_run(ftz_prover* p); /* = ftz_prover_submit + ftz_prover_wait */
/* asynchronous form on the prover's own streams (as ftz_batch_submit / ftz_batch_wait) */
int ftz_prover_submit(ftz_prover* p);
int ftz_prover_wait(ftz_prover* p);
size_t ftz_prover_bytes(const ftz_prover* p);
int ftz_prover_proofs(ftz_prover* p, uint8_t* buf, size_t cap, size_t* offsets, int32_t* codes);
int ftz_prover_stats(const ftz_prover* p, ftz_stats* out);
void ftz_prover_destroy(ftz_prover* p);

#ifdef __cplusplus
}
#endif
#endif /* FTSAMD_H */

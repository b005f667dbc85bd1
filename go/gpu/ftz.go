/*
SPDX-License-Identifier: Apache-2.0
*/

// Package gpu binds the MI355X batch verifier / prover (libftsamd.so, C ABI in
// include/ftsamd.h of this repository) into the zkatdlog (nogh) driver of the
// Fabric Token SDK. It lives at token/core/zkatdlog/crypto/validator/gpu in the
// SDK tree; see go/README.md for the file layout and INTEGRATION.md for the
// reference functions each entry point replaces.
//
// Every function here is a thin marshaller: Go values are flattened to the
// byte layouts the ABI documents (64-byte gnark RawBytes G1 points, 32-byte
// big-endian Zr, the proofs' own JSON), the buffers are pinned for the
// duration of one C call, and verdict codes are turned back into the error
// texts of the Go code they replace. There is no CPU fallback: NewVerifier
// fails when the library cannot open an MI355X.
package gpu

/*
#cgo CFLAGS: -I${SRCDIR}/include
#cgo LDFLAGS: -L${SRCDIR}/lib -lftsamd -Wl,-rpath,${SRCDIR}/lib
#include <stdlib.h>
#include "ftsamd.h"
*/
import "C"

import (
	"crypto/sha256"
	"os"
	"runtime"
	"sort"
	"strconv"
	"sync"
	"unsafe"

	math "github.com/IBM/mathlib"
	"github.com/hyperledger-labs/fabric-token-sdk/token/core/zkatdlog/crypto"
	issue2 "github.com/hyperledger-labs/fabric-token-sdk/token/core/zkatdlog/crypto/issue"
	"github.com/hyperledger-labs/fabric-token-sdk/token/core/zkatdlog/crypto/validator"
	"github.com/pkg/errors"
)

// Verifier owns one device context: the public parameters parsed and checked
// once, their fixed-base tables resident in HBM, and the job engine that
// merges concurrent calls into shared device passes. Safe for concurrent use.
type Verifier struct {
	mu  sync.RWMutex
	ctx *C.ftz_ctx
}

// Options mirrors ftz_options (include/ftsamd.h); zero fields keep the
// library defaults.
type Options struct {
	Batch        uint32 // max proofs per device pass (default 8192)
	Slots        uint32 // passes in flight (default 4)
	WindowUs     uint32 // how long a partial pass waits for more callers (default 1000)
	Threads      uint32 // host planning threads (default min(16, hardware threads))
	ProverTables int    // -1: no prover fixed-base tables; 0: default (on)
}

// DeviceFromEnv reads the opt-in FTS_GPU_DEVICE: unset or empty = the Go
// validator; "local" = the LOCAL_RANK of a one-process-per-GPU launch (0 when
// unset); a number = that HIP device ordinal.
func DeviceFromEnv() (int, bool) {
	s := os.Getenv("FTS_GPU_DEVICE")
	if s == "" {
		return 0, false
	}
	if s == "local" {
		s = os.Getenv("LOCAL_RANK")
		if s == "" {
			return 0, true
		}
	}
	d, err := strconv.Atoi(s)
	if err != nil || d < 0 {
		return -1, true // malformed: NewVerifier then fails loudly
	}
	return d, true
}

// NewVerifier replaces the pp.Deserialize + pp.Validate done once in
// Driver.NewValidator (nogh/driver/driver.go:114-124, crypto/setup.go:134-151,
// 238-273): ftz_ctx_create refuses public parameters Validate would refuse.
// device is the HIP device ordinal (one process per GPU: the local rank).
func NewVerifier(pp *crypto.PublicParams, device int) (*Verifier, error) {
	return NewVerifierWithOptions(pp, device, nil)
}

// NewVerifierWithOptions is NewVerifier with the engine policy set
// (ftz_ctx_create_ex).
func NewVerifierWithOptions(pp *crypto.PublicParams, device int, o *Options) (*Verifier, error) {
	raw, err := pp.Serialize()
	if err != nil {
		return nil, err
	}
	return newVerifierRaw(raw, device, o)
}

func newVerifierRaw(raw []byte, device int, o *Options) (*Verifier, error) {
	var opt C.ftz_options
	C.ftz_options_default(&opt)
	if o != nil {
		if o.Batch != 0 {
			opt.batch = C.uint32_t(o.Batch)
		}
		if o.Slots != 0 {
			opt.slots = C.uint32_t(o.Slots)
		}
		if o.WindowUs != 0 {
			opt.window_us = C.uint32_t(o.WindowUs)
		}
		if o.Threads != 0 {
			opt.threads = C.uint32_t(o.Threads)
		}
		if o.ProverTables < 0 {
			opt.prover_tables = 0
		}
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	var ctx *C.ftz_ctx
	if rc := C.ftz_ctx_create_ex(ptr(&pin, raw), C.size_t(len(raw)), C.int(device), &opt, &ctx); rc != C.FTZ_SUCCESS {
		return nil, errors.Errorf("invalid public parameters or no device: %s", lastError())
	}
	v := &Verifier{ctx: ctx}
	runtime.SetFinalizer(v, (*Verifier).Close)
	return v, nil
}

// shared holds the process's (Verifier, OwnerVerifier) pairs, one per
// (device, SHA-256 of the serialized public parameters): one process can run
// several TMSs (one per network, channel and namespace; tms.go:294 ->
// core.NewValidator), each with its own public parameters, on one device.
var shared struct {
	mu   sync.Mutex
	m    map[sharedKey]*sharedEntry
	tick uint64
}

type sharedKey struct {
	device int
	pp     [32]byte
}

type sharedEntry struct {
	key      sharedKey
	v        *Verifier
	ov       *OwnerVerifier // nil when SupportsIdemixCurve(pp.IdemixCurveID) is false
	refs     int            // live Handles
	lastUsed uint64         // shared.tick when the last Handle was released
}

// MaxIdleContexts bounds the contexts per device that no validator holds: the
// least recently released beyond it are closed. A context a Handle holds is
// never closed by the cache.
var MaxIdleContexts = 2

// Handle is one validator's hold on a shared (device, PP) context pair. Its
// methods are the validator callbacks; a method value (h.VerifyIssue) keeps
// the Handle, and so the pair, alive for as long as the validator holds it.
// Release, or the finalizer once the Handle is unreachable, drops the hold.
type Handle struct {
	e    *sharedEntry
	once sync.Once
}

// Shared returns a Handle on the process-wide Verifier and OwnerVerifier of
// (device, pp). Driver.NewValidator runs per request on some paths (the Orion
// custodian: services/network/orion/approval.go:100 ->
// token.NewServicesFromPublicParams -> core.NewValidator), so a device context
// -- the PP's fixed-base tables in HBM, streams, planning threads -- is built
// once per (device, PP) and reused by every validator of that PP. Parameters
// of different TMSs get their own contexts side by side; idle contexts beyond
// MaxIdleContexts per device are closed outside the cache lock.
func Shared(pp *crypto.PublicParams, device int) (*Handle, error) {
	raw, err := pp.Serialize()
	if err != nil {
		return nil, err
	}
	key := sharedKey{device: device, pp: sha256.Sum256(raw)}
	shared.mu.Lock()
	if shared.m == nil {
		shared.m = map[sharedKey]*sharedEntry{}
	}
	if e := shared.m[key]; e != nil {
		e.refs++
		shared.mu.Unlock()
		return newHandle(e), nil
	}
	shared.mu.Unlock()
	// build outside the lock (table construction takes a while); a racing
	// Shared for the same key keeps the first entry and closes its own pair
	v, err := newVerifierRaw(raw, device, nil)
	if err != nil {
		return nil, err
	}
	var ov *OwnerVerifier
	if SupportsIdemixCurve(pp.IdemixCurveID) {
		if ov, err = v.NewOwnerVerifier(pp); err != nil {
			v.Close()
			return nil, err
		}
	}
	shared.mu.Lock()
	e := shared.m[key]
	if e == nil {
		e = &sharedEntry{key: key, v: v, ov: ov}
		shared.m[key] = e
		v, ov = nil, nil
	}
	e.refs++
	shared.mu.Unlock()
	closePair(v, ov)
	return newHandle(e), nil
}

func newHandle(e *sharedEntry) *Handle {
	h := &Handle{e: e}
	runtime.SetFinalizer(h, (*Handle).Release)
	return h
}

func closePair(v *Verifier, ov *OwnerVerifier) {
	if ov != nil {
		ov.Close()
	}
	if v != nil {
		v.Close()
	}
}

// Release drops this Handle's hold (idempotent). The pair stays cached; it is
// closed only when more than MaxIdleContexts idle pairs share its device.
func (h *Handle) Release() {
	h.once.Do(func() {
		runtime.SetFinalizer(h, nil)
		var evict []*sharedEntry
		shared.mu.Lock()
		h.e.refs--
		shared.tick++
		h.e.lastUsed = shared.tick
		var idle []*sharedEntry
		for _, e := range shared.m {
			if e.key.device == h.e.key.device && e.refs == 0 {
				idle = append(idle, e)
			}
		}
		sort.Slice(idle, func(i, j int) bool { return idle[i].lastUsed > idle[j].lastUsed })
		for len(idle) > MaxIdleContexts {
			e := idle[len(idle)-1]
			idle = idle[:len(idle)-1]
			delete(shared.m, e.key)
			evict = append(evict, e)
		}
		shared.mu.Unlock()
		for _, e := range evict { // Close waits for calls in flight: never under shared.mu
			closePair(e.v, e.ov)
		}
	})
}

// Verifier is the shared context pair's zero-knowledge verifier.
func (h *Handle) Verifier() *Verifier { return h.e.v }

// OwnerVerifier is the pair's idemix owner-signature verifier, nil when the
// library does not verify owner signatures on pp.IdemixCurveID.
func (h *Handle) OwnerVerifier() *OwnerVerifier { return h.e.ov }

// TransferZKProofValidate is Verifier.TransferZKProofValidate (validator_transfer.go:84-98).
func (h *Handle) TransferZKProofValidate(ctx *validator.Context) error {
	return h.e.v.TransferZKProofValidate(ctx)
}

// VerifyIssue is Verifier.VerifyIssue (validator.go:181-191).
func (h *Handle) VerifyIssue(action *issue2.IssueAction) error { return h.e.v.VerifyIssue(action) }

// TransferSignatureValidate is OwnerVerifier.TransferSignatureValidate
// (validator_transfer.go:42-82); only for a Handle whose OwnerVerifier is not nil.
func (h *Handle) TransferSignatureValidate(ctx *validator.Context) error {
	return h.e.ov.TransferSignatureValidate(ctx)
}

// SharedContexts is the number of device contexts Shared holds (tests).
func SharedContexts() int {
	shared.mu.Lock()
	defer shared.mu.Unlock()
	return len(shared.m)
}

// Close releases the device context. Calls after Close fail.
func (v *Verifier) Close() {
	v.mu.Lock()
	defer v.mu.Unlock()
	if v.ctx != nil {
		C.ftz_ctx_destroy(v.ctx)
		v.ctx = nil
	}
}

// Closed reports whether Close has run.
func (v *Verifier) Closed() bool {
	v.mu.RLock()
	defer v.mu.RUnlock()
	return v.ctx == nil
}

// use runs f with the context held against a concurrent Close.
func (v *Verifier) use(f func(ctx *C.ftz_ctx) error) error {
	v.mu.RLock()
	defer v.mu.RUnlock()
	if v.ctx == nil {
		return errors.New("gpu verifier closed")
	}
	return f(v.ctx)
}

func lastError() string { return C.GoString(C.ftz_last_error()) }

// ptr pins b for the duration of the C call it is passed to and returns its
// address as the ABI's const uint8_t*; nil for an empty slice.
func ptr(pin *runtime.Pinner, b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	pin.Pin(&b[0])
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

// cArray allocates n elements of T in C memory, where pinned Go pointers may
// be stored (the ABI's descriptor arrays); release with C.free(&s[0]).
func cArray[T any](n int) []T {
	var z T
	return unsafe.Slice((*T)(C.malloc(C.size_t(n)*C.size_t(unsafe.Sizeof(z)))), n)
}

// rawBytes flattens G1 points to the ABI's n x 64-byte gnark RawBytes.
func rawBytes(ps []*math.G1) []byte {
	b := make([]byte, 0, 64*len(ps))
	for _, p := range ps {
		b = append(b, p.Bytes()...)
	}
	return b
}

// errText maps a verdict code to the error text of the Go code it stands for
// (the class, not the wrapped detail: the library reports one code per proof).
var errText = map[C.int32_t]string{
	C.FTZ_ERR_PARSE:       "failed to unmarshal proof",
	C.FTZ_ERR_MALFORMED:   "proof not well formed",
	C.FTZ_ERR_WF:          "invalid zero-knowledge transfer",
	C.FTZ_ERR_RANGE:       "invalid range proof",
	C.FTZ_ERR_MEMBERSHIP:  "invalid membership proof",
	C.FTZ_ERR_PANIC:       "proof would crash the reference verifier",
	C.FTZ_ERR_OPENING:     "output does not match the provided opening",
	C.FTZ_ERR_INPUT:       "input to spend does not exist or is not a token",
	C.FTZ_ERR_OWNER:       "failed deserializing owner",
	C.FTZ_ERR_SIGNATURE:   "pseudonym signature invalid",
	C.FTZ_ERR_UNSUPPORTED: "owner type verified in Go",
	C.FTZ_ERR_AUDIT:       "owner does not match its audit info",
}

// Verdict codes (include/ftsamd.h FTZ_*), for callers and tests without cgo.
const (
	CodeOK          = int(C.FTZ_OK)
	CodeOwner       = int(C.FTZ_ERR_OWNER)
	CodeSignature   = int(C.FTZ_ERR_SIGNATURE)
	CodeUnsupported = int(C.FTZ_ERR_UNSUPPORTED)
)

// CodeError is a failed verdict: Code is the library's FTZ_ERR_* value.
type CodeError struct {
	Code int
	msg  string
}

func (e *CodeError) Error() string { return e.msg }

func codeErr(c C.int32_t) error {
	if c == C.FTZ_OK {
		return nil
	}
	t, ok := errText[c]
	if !ok {
		t = "verification failed"
	}
	return &CodeError{Code: int(c), msg: t}
}

// Transfer is one transfer proof to verify: ledger input commitments, output
// commitments and the proof bytes of TransferAction.Proof.
type Transfer struct {
	Inputs, Outputs []*math.G1
	Proof           []byte
}

// VerifyTransfers verifies n transfer proofs in one call (shared device
// passes): errs[i] is nil or what transfer.NewVerifier(in, out,
// pp).Verify(proof) (crypto/transfer/transfer.go:66-77,124-154) would fail with.
func (v *Verifier) VerifyTransfers(ts []Transfer) ([]error, error) {
	in, out, proofs := make([][]byte, len(ts)), make([][]byte, len(ts)), make([][]byte, len(ts))
	for i, t := range ts {
		in[i], out[i], proofs[i] = rawBytes(t.Inputs), rawBytes(t.Outputs), t.Proof
	}
	codes, err := v.verifyTransfersRaw(in, out, proofs)
	return codeErrs(codes), err
}

func codeErrs(codes []int) []error {
	if codes == nil {
		return nil
	}
	errs := make([]error, len(codes))
	for i, c := range codes {
		errs[i] = codeErr(C.int32_t(c))
	}
	return errs
}

// verifyTransfersRaw: in[i] / out[i] are n x 64-byte RawBytes, codes as the ABI.
func (v *Verifier) verifyTransfersRaw(in, out, proofs [][]byte) ([]int, error) {
	n := len(proofs)
	if n == 0 {
		return nil, nil
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	// C.malloc'd descriptor array: it holds pinned Go pointers, which cgo allows in C memory
	tx := cArray[C.ftz_transfer](n)
	defer C.free(unsafe.Pointer(&tx[0]))
	for i := range proofs {
		tx[i] = C.ftz_transfer{inputs: ptr(&pin, in[i]), n_in: C.uint32_t(len(in[i]) / 64), outputs: ptr(&pin, out[i]),
			n_out: C.uint32_t(len(out[i]) / 64), proof: ptr(&pin, proofs[i]), proof_len: C.size_t(len(proofs[i]))}
	}
	codes := make([]C.int32_t, n)
	err := v.use(func(ctx *C.ftz_ctx) error {
		if rc := C.ftz_verify_transfers(ctx, C.size_t(n), &tx[0], &codes[0]); rc != C.FTZ_SUCCESS {
			return errors.Errorf("gpu verifier: %s", lastError())
		}
		return nil
	})
	if err != nil {
		return nil, err
	}
	return ints(codes), nil
}

func ints(codes []C.int32_t) []int {
	out := make([]int, len(codes))
	for i, c := range codes {
		out[i] = int(c)
	}
	return out
}

// TransferZKProofValidate is a drop-in for validator.TransferZKProofValidate
// (crypto/validator/validator_transfer.go:84-98): the same inputs (the ledger
// commitments TransferSignatureValidate loaded into ctx.InputTokens), the same
// outputs and proof. Concurrent callers share device passes (the job engine).
func (v *Verifier) TransferZKProofValidate(ctx *validator.Context) error {
	in := make([]*math.G1, len(ctx.InputTokens))
	for i, tok := range ctx.InputTokens {
		in[i] = tok.GetCommitment()
	}
	errs, err := v.VerifyTransfers([]Transfer{{Inputs: in, Outputs: ctx.Action.GetOutputCommitments(),
		Proof: ctx.Action.GetProof()}})
	if err != nil {
		return err
	}
	return errs[0]
}

// VerifyIssue replaces the issue2.NewVerifier(coms, anonymous, pp).Verify(proof)
// call of Validator.verifyIssue (crypto/validator/validator.go:181-191).
func (v *Verifier) VerifyIssue(action *issue2.IssueAction) error {
	coms, err := action.GetCommitments()
	if err != nil {
		return errors.New("failed to verify issue")
	}
	errs, err := v.VerifyIssues([]Issue{{Outputs: coms, Anonymous: action.IsAnonymous(), Proof: action.GetProof()}})
	if err != nil {
		return err
	}
	return errs[0]
}

// Issue is one issue proof to verify.
type Issue struct {
	Outputs   []*math.G1
	Anonymous bool
	Proof     []byte
}

// VerifyIssues verifies n issue proofs in one call (crypto/issue/issue.go:194-223).
func (v *Verifier) VerifyIssues(is []Issue) ([]error, error) {
	out, proofs, anon := make([][]byte, len(is)), make([][]byte, len(is)), make([]bool, len(is))
	for i, x := range is {
		out[i], proofs[i], anon[i] = rawBytes(x.Outputs), x.Proof, x.Anonymous
	}
	codes, err := v.verifyIssuesRaw(out, anon, proofs)
	return codeErrs(codes), err
}

func (v *Verifier) verifyIssuesRaw(out [][]byte, anonymous []bool, proofs [][]byte) ([]int, error) {
	n := len(proofs)
	if n == 0 {
		return nil, nil
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	d := cArray[C.ftz_issue](n)
	defer C.free(unsafe.Pointer(&d[0]))
	for i := range proofs {
		var anon C.uint8_t
		if anonymous[i] {
			anon = 1
		}
		d[i] = C.ftz_issue{outputs: ptr(&pin, out[i]), n_out: C.uint32_t(len(out[i]) / 64), proof: ptr(&pin, proofs[i]),
			proof_len: C.size_t(len(proofs[i])), anonymous: anon}
	}
	codes := make([]C.int32_t, n)
	err := v.use(func(ctx *C.ftz_ctx) error {
		if rc := C.ftz_verify_issues(ctx, C.size_t(n), &d[0], &codes[0]); rc != C.FTZ_SUCCESS {
			return errors.Errorf("gpu verifier: %s", lastError())
		}
		return nil
	})
	if err != nil {
		return nil, err
	}
	return ints(codes), nil
}

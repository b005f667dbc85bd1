/*
SPDX-License-Identifier: Apache-2.0
*/

package gpu

/*
#include <stdlib.h>
#include "ftsamd.h"
// callbacks.c: C function pointers to the exported Go lookups below
ftz_get_state_fn ftz_go_get_state_fn(void);
ftz_get_states_fn ftz_go_get_states_fn(void);
*/
import "C"

import (
	"runtime"
	"runtime/cgo"
	"unsafe"

	"github.com/hyperledger-labs/fabric-token-sdk/token/driver"
	"github.com/pkg/errors"
)

// GetStatesFnc looks up many ledger keys at once: vals[i] is the value of
// keys[i], nil when it does not exist. A ledger that can serve a batch (a
// state database's multi-get, a block-local cache) implements it directly;
// BatchOf adapts a driver.GetStateFnc.
type GetStatesFnc = func(keys []string) ([][]byte, error)

// BatchOf turns a per-key lookup (driver.GetStateFnc, token/driver/validator.go:12)
// into a GetStatesFnc that looks the keys up in order.
func BatchOf(get driver.GetStateFnc) GetStatesFnc {
	return func(keys []string) ([][]byte, error) {
		vals := make([][]byte, len(keys))
		for i, k := range keys {
			v, err := get(k)
			if err != nil {
				return nil, err
			}
			vals[i] = v
		}
		return vals, nil
	}
}

// blockLedger is what the C callbacks see through a cgo.Handle: the Go lookup
// and the pins keeping the latest values alive until the library has copied
// them (the ABI's contract: until the next callback or the call's return).
type blockLedger struct {
	get  driver.GetStateFnc
	gets GetStatesFnc
	pin  runtime.Pinner
}

// ledgerOf reads the cgo.Handle verifyBlock passes by reference as the ABI's
// void* user (the runtime/cgo pattern: a pointer to the handle, never the
// handle's integer value converted to a pointer).
func ledgerOf(user unsafe.Pointer) *blockLedger {
	return (*(*cgo.Handle)(user)).Value().(*blockLedger)
}

//export goGetState
func goGetState(user unsafe.Pointer, key *C.char, keyLen C.size_t, val **C.uint8_t, valLen *C.size_t) C.int {
	l := ledgerOf(user)
	l.pin.Unpin() // the previous value has been copied
	v, err := l.get(C.GoStringN(key, C.int(keyLen)))
	if err != nil {
		return 1
	}
	*valLen = C.size_t(len(v))
	*val = ptr(&l.pin, v)
	return 0
}

//export goGetStates
func goGetStates(user unsafe.Pointer, n C.size_t, keys *C.ftz_bytes, vals *C.ftz_bytes) C.int {
	l := ledgerOf(user)
	l.pin.Unpin() // the previous chunk's values have been copied
	ks := unsafe.Slice(keys, int(n))
	vs := unsafe.Slice(vals, int(n))
	names := make([]string, len(ks))
	for i, k := range ks {
		names[i] = C.GoStringN((*C.char)(unsafe.Pointer(k.p)), C.int(k.len))
	}
	got, err := l.gets(names)
	if err != nil || len(got) != len(names) {
		return 1
	}
	for i, v := range got {
		vs[i] = C.ftz_bytes{p: ptr(&l.pin, v), len: C.size_t(len(v))}
	}
	return 0
}

// VerifyBlock runs the ZK part of Validator.VerifyTokenRequestFromRaw
// (crypto/validator/validator.go:45-108) for every raw token request of a
// block in ONE library call: ASN.1 + action JSON decoding, the inputs loaded
// through getStates (one callback per pipeline chunk of up to 4096 requests),
// every issue and transfer proof verified in shared device passes. errs[i] is
// nil or request i's first failing check, wrapped with its action index (issues
// first, then transfers). The checks that stay in Go -- auditor / issuer x509
// signatures, idemix owner signatures (OwnerVerifier, one call for the block),
// HTLC scripts, metadata counting -- run beside it.
func (v *Verifier) VerifyBlock(getStates GetStatesFnc, raws [][]byte) ([]error, error) {
	return v.verifyBlock(&blockLedger{gets: getStates}, raws)
}

// VerifyBlockPerKey is VerifyBlock with one callback per input (the
// reference's GetStateFnc shape; one cgo crossing per key).
func (v *Verifier) VerifyBlockPerKey(getState driver.GetStateFnc, raws [][]byte) ([]error, error) {
	return v.verifyBlock(&blockLedger{get: getState}, raws)
}

func (v *Verifier) verifyBlock(l *blockLedger, raws [][]byte) ([]error, error) {
	if len(raws) == 0 {
		return nil, nil
	}
	defer l.pin.Unpin()
	h := cgo.NewHandle(l)
	defer h.Delete()
	// &h is a Go pointer to pointer-free memory: cgo keeps it valid (and
	// pinned) for the duration of the call, which is as long as the library
	// may use it
	var pin runtime.Pinner
	defer pin.Unpin()
	reqs := cArray[C.ftz_bytes](len(raws))
	defer C.free(unsafe.Pointer(&reqs[0]))
	for i, r := range raws {
		reqs[i] = C.ftz_bytes{p: ptr(&pin, r), len: C.size_t(len(r))}
	}
	codes := make([]C.int32_t, len(raws))
	failed := make([]C.int32_t, len(raws))
	err := v.use(func(ctx *C.ftz_ctx) error {
		var rc C.int
		if l.gets != nil {
			rc = C.ftz_verify_token_requests_batched(ctx, C.size_t(len(raws)), &reqs[0], C.ftz_go_get_states_fn(),
				unsafe.Pointer(&h), &codes[0], &failed[0])
		} else {
			rc = C.ftz_verify_token_requests(ctx, C.size_t(len(raws)), &reqs[0], C.ftz_go_get_state_fn(),
				unsafe.Pointer(&h), &codes[0], &failed[0])
		}
		if rc != C.FTZ_SUCCESS {
			return errors.Errorf("gpu verifier: %s", lastError())
		}
		return nil
	})
	if err != nil {
		return nil, err
	}
	errs := make([]error, len(raws))
	for i, c := range codes {
		if e := codeErr(c); e != nil {
			if failed[i] >= 0 {
				e = errors.Wrapf(e, "action %d", failed[i])
			}
			errs[i] = e
		}
	}
	return errs, nil
}

// RequestStats returns the calling threads' time (ms) in each stage of the
// request pipeline since the last reset: decode, element checks, ledger
// callbacks, token decoding, job building, waiting on earlier chunks.
func (v *Verifier) RequestStats(reset bool) ([6]float64, error) {
	var ms [6]C.double
	var out [6]float64
	r := C.int(0)
	if reset {
		r = 1
	}
	err := v.use(func(ctx *C.ftz_ctx) error {
		if rc := C.ftz_ctx_request_stats(ctx, &ms[0], r); rc != C.FTZ_SUCCESS {
			return errors.Errorf("gpu verifier: %s", lastError())
		}
		return nil
	})
	for i := range ms {
		out[i] = float64(ms[i])
	}
	return out, err
}

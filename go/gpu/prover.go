/*
SPDX-License-Identifier: Apache-2.0
*/

package gpu

/*
#include <stdlib.h>
#include "ftsamd.h"
*/
import "C"

import (
	"crypto/rand"
	"runtime"
	"unsafe"

	math "github.com/IBM/mathlib"
	"github.com/hyperledger-labs/fabric-token-sdk/token/core/zkatdlog/crypto/token"
	"github.com/pkg/errors"
)

// The reference provers draw their blinding scalars from crypto/rand. The GPU
// prover takes 32 bytes of crypto/rand per proof as a seed and derives every
// random scalar from it (SHA-256(seed||tag||0) || SHA-256(seed||tag||1) mod r),
// so proofs have the reference's distribution and a recorded seed replays a
// proof byte for byte (what the parity tests do).

// TransferWitness is one transfer to prove: the arguments of
// transfer.NewProver(inW, outW, in, out, pp) (crypto/transfer/transfer.go:42).
type TransferWitness struct {
	InW, OutW []*token.TokenDataWitness
	In, Out   []*math.G1
	Seed      []byte // 32 bytes; nil: drawn from crypto/rand
}

// IssueWitness is one issue to prove: issue.NewProver(tw, tokens, anonymous, pp)
// (crypto/issue/issue.go:151).
type IssueWitness struct {
	TW        []*token.TokenDataWitness
	Tokens    []*math.G1
	Anonymous bool
	Seed      []byte
}

func zrs(ws []*token.TokenDataWitness, f func(*token.TokenDataWitness) *math.Zr) []byte {
	b := make([]byte, 0, 32*len(ws))
	for _, w := range ws {
		b = append(b, f(w).Bytes()...) // 32-byte big-endian
	}
	return b
}

func value(w *token.TokenDataWitness) *math.Zr { return w.Value }
func blind(w *token.TokenDataWitness) *math.Zr { return w.BlindingFactor }

func seedOf(s []byte) ([]byte, error) {
	if s != nil {
		if len(s) != 32 {
			return nil, errors.New("prover seed must be 32 bytes")
		}
		return s, nil
	}
	s = make([]byte, 32)
	_, err := rand.Read(s)
	return s, err
}

func cstr(pin *runtime.Pinner, s string) (*C.char, C.size_t) {
	b := []byte(s)
	return (*C.char)(unsafe.Pointer(ptr(pin, b))), C.size_t(len(b))
}

// ProveTransfers replaces n calls of transfer.NewProver(inW, outW, in, out,
// pp).Prove() (crypto/transfer/transfer.go:89-121): proofs[i] is the same JSON
// wire format. A value outside [0, base^exponent) fails the whole call, as the
// reference's range prover fails ("value of token outside authorized range").
func (v *Verifier) ProveTransfers(ws []TransferWitness) ([][]byte, error) {
	if len(ws) == 0 {
		return nil, nil
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	d := cArray[C.ftz_transfer_witness](len(ws))
	defer C.free(unsafe.Pointer(&d[0]))
	for i, w := range ws {
		if len(w.InW) != len(w.In) || len(w.OutW) != len(w.Out) || len(w.InW) == 0 {
			return nil, errors.Errorf("transfer %d: witness and commitment counts differ", i)
		}
		seed, err := seedOf(w.Seed)
		if err != nil {
			return nil, err
		}
		ty, tyLen := cstr(&pin, w.InW[0].Type)
		d[i] = C.ftz_transfer_witness{inputs: ptr(&pin, rawBytes(w.In)), n_in: C.uint32_t(len(w.In)),
			outputs: ptr(&pin, rawBytes(w.Out)), n_out: C.uint32_t(len(w.Out)),
			in_values: ptr(&pin, zrs(w.InW, value)), in_bfs: ptr(&pin, zrs(w.InW, blind)),
			out_values: ptr(&pin, zrs(w.OutW, value)), out_bfs: ptr(&pin, zrs(w.OutW, blind)),
			_type: ty, type_len: tyLen, seed: ptr(&pin, seed)}
	}
	return v.prove(len(ws), func(ctx *C.ftz_ctx, p **C.ftz_prover) C.int {
		return C.ftz_prover_load_transfers(ctx, C.size_t(len(ws)), &d[0], p)
	})
}

// ProveIssues replaces n calls of issue.NewProver(...).Prove()
// (crypto/issue/issue.go:162-184).
func (v *Verifier) ProveIssues(ws []IssueWitness) ([][]byte, error) {
	if len(ws) == 0 {
		return nil, nil
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	d := cArray[C.ftz_issue_witness](len(ws))
	defer C.free(unsafe.Pointer(&d[0]))
	for i, w := range ws {
		if len(w.TW) != len(w.Tokens) || len(w.TW) == 0 {
			return nil, errors.Errorf("issue %d: witness and commitment counts differ", i)
		}
		seed, err := seedOf(w.Seed)
		if err != nil {
			return nil, err
		}
		var anon C.uint8_t
		if w.Anonymous {
			anon = 1
		}
		ty, tyLen := cstr(&pin, w.TW[0].Type)
		d[i] = C.ftz_issue_witness{outputs: ptr(&pin, rawBytes(w.Tokens)), n_out: C.uint32_t(len(w.Tokens)),
			values: ptr(&pin, zrs(w.TW, value)), bfs: ptr(&pin, zrs(w.TW, blind)), _type: ty, type_len: tyLen,
			anonymous: anon, seed: ptr(&pin, seed)}
	}
	return v.prove(len(ws), func(ctx *C.ftz_ctx, p **C.ftz_prover) C.int {
		return C.ftz_prover_load_issues(ctx, C.size_t(len(ws)), &d[0], p)
	})
}

// prove runs the staged prover (load = plan + upload, run, copy the proofs out
// into one Go buffer sized by ftz_prover_bytes).
func (v *Verifier) prove(n int, load func(*C.ftz_ctx, **C.ftz_prover) C.int) ([][]byte, error) {
	var out [][]byte
	err := v.use(func(ctx *C.ftz_ctx) error {
		var p *C.ftz_prover
		if rc := load(ctx, &p); rc != C.FTZ_SUCCESS {
			return errors.Errorf("gpu prover: %s", lastError())
		}
		defer C.ftz_prover_destroy(p)
		if rc := C.ftz_prover_run(p); rc != C.FTZ_SUCCESS {
			return errors.Errorf("gpu prover: %s", lastError())
		}
		size := int(C.ftz_prover_bytes(p))
		buf := make([]byte, size+1)
		offs := make([]C.size_t, n+1)
		codes := make([]C.int32_t, n)
		if rc := C.ftz_prover_proofs(p, (*C.uint8_t)(unsafe.Pointer(&buf[0])), C.size_t(size), &offs[0], &codes[0]); rc != C.FTZ_SUCCESS {
			return errors.Errorf("gpu prover: %s", lastError())
		}
		out = make([][]byte, n)
		for i := 0; i < n; i++ {
			if codes[i] != C.FTZ_OK {
				return errors.Errorf("proof %d: invalid commitment", i)
			}
			out[i] = buf[offs[i]:offs[i+1]:offs[i+1]]
		}
		return nil
	})
	return out, err
}

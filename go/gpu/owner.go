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
	"runtime"
	"unsafe"

	math "github.com/IBM/mathlib"
	"github.com/hyperledger-labs/fabric-smart-client/platform/view/view"
	"github.com/hyperledger-labs/fabric-token-sdk/token/core/zkatdlog/crypto"
	"github.com/hyperledger-labs/fabric-token-sdk/token/core/zkatdlog/crypto/token"
	"github.com/hyperledger-labs/fabric-token-sdk/token/core/zkatdlog/crypto/validator"
	"github.com/hyperledger-labs/fabric-token-sdk/token/driver"
	"github.com/pkg/errors"
)

// OwnerVerifier verifies idemix owner signatures (NymSignature.Ver) on the
// device, on the curve PublicParams.IdemixCurveID selects: BN254 (the curve
// cmd/pp/dlog/gen.go and the NWO topologies deploy) or FP256BN_AMCL.
type OwnerVerifier struct {
	v  *Verifier
	ix *C.ftz_idemix
}

// NewOwnerVerifier takes PublicParams.IdemixIssuerPK and IdemixCurveID
// (crypto/setup.go:36-38), the inputs of idemix.NewDeserializer
// (nogh/deserializer.go:50). The issuer key's own proof is checked once by the
// Go deserializer, as in the reference; the library refuses a key whose HSk or
// HRand does not decode on the curve.
func (v *Verifier) NewOwnerVerifier(pp *crypto.PublicParams) (*OwnerVerifier, error) {
	return v.newOwnerVerifierRaw(pp.IdemixIssuerPK, int(pp.IdemixCurveID))
}

func (v *Verifier) newOwnerVerifierRaw(ipk []byte, curve int) (*OwnerVerifier, error) {
	var pin runtime.Pinner
	defer pin.Unpin()
	var ix *C.ftz_idemix
	err := v.use(func(ctx *C.ftz_ctx) error {
		if rc := C.ftz_idemix_create(ctx, ptr(&pin, ipk), C.size_t(len(ipk)), C.int(curve), &ix); rc != C.FTZ_SUCCESS {
			return errors.Errorf("ftz_idemix_create: %s", lastError())
		}
		return nil
	})
	if err != nil {
		return nil, err
	}
	o := &OwnerVerifier{v: v, ix: ix}
	runtime.SetFinalizer(o, (*OwnerVerifier).Close)
	return o, nil
}

// Close releases the verifier (before the Verifier it was made from).
func (o *OwnerVerifier) Close() {
	if o.ix != nil {
		C.ftz_idemix_destroy(o.ix)
		o.ix = nil
	}
}

// OwnerSig is one owner signature: the token's Owner bytes (asn1 RawOwner),
// the signed message and the NymSignature proto.
type OwnerSig struct {
	Owner, Msg, Sig []byte
}

// Verify returns one code per signature: FTZ_OK (0), FTZ_ERR_OWNER,
// FTZ_ERR_SIGNATURE or FTZ_ERR_UNSUPPORTED (an HTLC script owner, which the
// caller verifies in Go).
func (o *OwnerVerifier) Verify(items []OwnerSig) ([]int, error) {
	if len(items) == 0 {
		return nil, nil
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	d := cArray[C.ftz_owner_sig](len(items))
	defer C.free(unsafe.Pointer(&d[0]))
	for i, it := range items {
		d[i] = C.ftz_owner_sig{owner: ptr(&pin, it.Owner), owner_len: C.size_t(len(it.Owner)),
			msg: ptr(&pin, it.Msg), msg_len: C.size_t(len(it.Msg)), sig: ptr(&pin, it.Sig), sig_len: C.size_t(len(it.Sig))}
	}
	codes := make([]C.int32_t, len(items))
	err := o.v.use(func(*C.ftz_ctx) error {
		if rc := C.ftz_verify_owner_signatures(o.ix, C.size_t(len(items)), &d[0], &codes[0]); rc != C.FTZ_SUCCESS {
			return errors.Errorf("gpu owner verifier: %s", lastError())
		}
		return nil
	})
	if err != nil {
		return nil, err
	}
	out := make([]int, len(codes))
	for i, c := range codes {
		out[i] = int(c)
	}
	return out, nil
}

// capture is the driver.Verifier handed to SignatureProvider.HasBeenSignedBy:
// the provider advances its cursor and calls Verify(message, sigma) exactly as
// for the Go verifier (common/backend.go:32-41); capture records both and
// accepts, and the real verdict comes from the device afterwards.
type capture struct{ msg, sigma []byte }

func (c *capture) Verify(message, sigma []byte) error {
	c.msg, c.sigma = message, sigma
	return nil
}

// errPseudonym is the text of a failing idemix NymSignature.Ver (IBM/idemix
// nymsignature.go), which HasBeenSignedBy returns and the reference wraps.
var errPseudonym = errors.New("pseudonym signature invalid: zero-knowledge proof is invalid")

// sigInput is one input of a transfer action as the reference's loop sees it.
type sigInput struct {
	key      string
	tok      *token.Token
	verifier driver.Verifier // the Go owner verifier (GetOwnerVerifier)
	item     OwnerSig
}

// sigSteps are the reference loop's effects, injectable for the precedence
// test (gpu_test.go): load the ledger token of one input, deserialize its
// owner, let the signature provider hand out the next signature, and verify a
// batch of owner signatures (codes as ftz_verify_owner_signatures).
type sigSteps struct {
	load   func(key string) (*token.Token, error)
	owner  func(raw view.Identity) (driver.Verifier, error)
	signed func(owner view.Identity, v driver.Verifier) ([]byte, error)
	verify func(items []OwnerSig) ([]int, error)
}

// transferSignatures runs validator.TransferSignatureValidate's loop
// (crypto/validator/validator_transfer.go:50-76) with every owner signature of
// the action verified in one device batch, and returns exactly the reference's
// first error: per input, in order, the ledger load, the owner deserialization
// ("failed deserializing owner [i][in][UniqueID]"), the provider's cursor and
// then the signature itself ("failed signature verification [i][in][UniqueID]").
// When a step of input j fails, the signatures of inputs 0..j-1 -- which the
// reference verified before reaching input j -- are checked first, so a bad
// signature on an earlier input still wins.
func transferSignatures(keys []string, st sigSteps) ([]sigInput, error) {
	ins := make([]sigInput, 0, len(keys))
	// check verifies the signatures of ins on the device and returns the
	// reference's error for the first bad one
	check := func() error {
		if len(ins) == 0 {
			return nil
		}
		items := make([]OwnerSig, len(ins))
		for i := range ins {
			items[i] = ins[i].item
		}
		codes, err := st.verify(items)
		if err != nil {
			return err
		}
		for i, c := range codes {
			in := ins[i]
			var verr error
			switch c {
			case int(C.FTZ_OK):
			case int(C.FTZ_ERR_UNSUPPORTED), int(C.FTZ_ERR_OWNER):
				// an owner the library does not verify (HTLC script) or decodes
				// differently from the Go deserializer: the Go verifier decides
				verr = in.verifier.Verify(in.item.Msg, in.item.Sig)
			default:
				verr = errPseudonym
			}
			if verr != nil {
				return errors.Wrapf(verr, "failed signature verification [%d][%s][%s]", i, in.key,
					view.Identity(in.tok.Owner).UniqueID())
			}
		}
		return nil
	}
	fail := func(err error) ([]sigInput, error) {
		if e := check(); e != nil {
			return nil, e
		}
		return nil, err
	}
	for i, key := range keys {
		tok, err := st.load(key)
		if err != nil {
			return fail(err)
		}
		verifier, err := st.owner(tok.Owner)
		if err != nil {
			return fail(errors.Wrapf(err, "failed deserializing owner [%d][%s][%s]", i, key,
				view.Identity(tok.Owner).UniqueID()))
		}
		c := &capture{}
		if _, err := st.signed(tok.Owner, c); err != nil { // insufficient signatures
			return fail(errors.Wrapf(err, "failed signature verification [%d][%s][%s]", i, key,
				view.Identity(tok.Owner).UniqueID()))
		}
		ins = append(ins, sigInput{key: key, tok: tok, verifier: verifier,
			item: OwnerSig{Owner: tok.Owner, Msg: c.msg, Sig: c.sigma}})
	}
	if err := check(); err != nil {
		return nil, err
	}
	return ins, nil
}

// TransferSignatureValidate is a drop-in for validator.TransferSignatureValidate
// (crypto/validator/validator_transfer.go:42-82): the same ledger loads, owner
// deserialization, signature order and error texts, with the owners'
// signatures of the action verified in one device call (transferSignatures).
func (o *OwnerVerifier) TransferSignatureValidate(ctx *validator.Context) error {
	keys, err := ctx.Action.GetInputs()
	if err != nil {
		return errors.Wrapf(err, "failed to retrieve inputs to spend")
	}
	ins, err := transferSignatures(keys, sigSteps{
		load: func(in string) (*token.Token, error) {
			raw, err := ctx.Ledger.GetState(in)
			if err != nil {
				return nil, errors.Wrapf(err, "failed to retrieve input to spend [%s]", in)
			}
			if len(raw) == 0 {
				return nil, errors.Errorf("input to spend [%s] does not exists", in)
			}
			tok := &token.Token{}
			if err := tok.Deserialize(raw); err != nil {
				return nil, errors.Wrapf(err, "failed to deserialize input to spend [%s]", in)
			}
			return tok, nil
		},
		owner:  ctx.Deserializer.GetOwnerVerifier,
		signed: ctx.SignatureProvider.HasBeenSignedBy,
		verify: o.Verify,
	})
	if err != nil {
		return err
	}
	tokens, sigs := make([]*token.Token, len(ins)), make([][]byte, len(ins))
	for i, in := range ins {
		tokens[i], sigs[i] = in.tok, in.item.Sig
	}
	ctx.InputTokens, ctx.Signatures = tokens, sigs
	return nil
}

// SupportsIdemixCurve reports whether the library verifies owner signatures on
// the idemix curve PublicParams.IdemixCurveID names (ftz_idemix_create: BN254
// and FP256BN_AMCL). Other curves (e.g. FP256BN_AMCL_MIRACL, which
// identity/msp/idemix/deserializer.go:47 also accepts) keep the Go
// validator.TransferSignatureValidate; the ZK checks still run on the GPU.
func SupportsIdemixCurve(id math.CurveID) bool {
	return id == math.BN254 || id == math.FP256BN_AMCL
}

// OwnerAudit is one auditor owner inspection: the token's Owner bytes and the
// owner's OwnerInfo (json AuditInfo).
type OwnerAudit struct {
	Owner, AuditInfo []byte
}

// AuditOwners replaces AuditInfo.Match behind the auditor's
// InspectTokenOwnerFunc (crypto/audit/auditor.go:226-230,252-274;
// identity/msp/idemix/audit.go:51-83) for n owners: codes as ftz_audit_owners.
func (o *OwnerVerifier) AuditOwners(items []OwnerAudit) ([]int, error) {
	if len(items) == 0 {
		return nil, nil
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	d := cArray[C.ftz_owner_audit](len(items))
	defer C.free(unsafe.Pointer(&d[0]))
	for i, it := range items {
		d[i] = C.ftz_owner_audit{owner: ptr(&pin, it.Owner), owner_len: C.size_t(len(it.Owner)),
			audit_info: ptr(&pin, it.AuditInfo), audit_info_len: C.size_t(len(it.AuditInfo))}
	}
	codes := make([]C.int32_t, len(items))
	err := o.v.use(func(*C.ftz_ctx) error {
		if rc := C.ftz_audit_owners(o.ix, C.size_t(len(items)), &d[0], &codes[0]); rc != C.FTZ_SUCCESS {
			return errors.Errorf("gpu owner audit: %s", lastError())
		}
		return nil
	})
	if err != nil {
		return nil, err
	}
	out := make([]int, len(codes))
	for i, c := range codes {
		out[i] = int(c)
	}
	return out, nil
}

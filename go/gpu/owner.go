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

	"github.com/hyperledger-labs/fabric-token-sdk/token/core/zkatdlog/crypto"
	"github.com/hyperledger-labs/fabric-token-sdk/token/core/zkatdlog/crypto/token"
	"github.com/hyperledger-labs/fabric-token-sdk/token/core/zkatdlog/crypto/validator"
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

// TransferSignatureValidate is a drop-in for validator.TransferSignatureValidate
// (crypto/validator/validator_transfer.go:42-82): the same ledger loads, error
// texts and signature order, with the owners' signatures of the action verified
// in one device call. Owners the library does not verify (HTLC scripts,
// FTZ_ERR_UNSUPPORTED) go through ctx.Deserializer.GetOwnerVerifier as before.
func (o *OwnerVerifier) TransferSignatureValidate(ctx *validator.Context) error {
	inputs, err := ctx.Action.GetInputs()
	if err != nil {
		return errors.Wrapf(err, "failed to retrieve inputs to spend")
	}
	tokens := make([]*token.Token, 0, len(inputs))
	sigs := make([][]byte, 0, len(inputs))
	items := make([]OwnerSig, 0, len(inputs))
	for _, in := range inputs {
		raw, err := ctx.Ledger.GetState(in)
		if err != nil {
			return errors.Wrapf(err, "failed to retrieve input to spend [%s]", in)
		}
		if len(raw) == 0 {
			return errors.Errorf("input to spend [%s] does not exists", in)
		}
		tok := &token.Token{}
		if err := tok.Deserialize(raw); err != nil {
			return errors.Wrapf(err, "failed to deserialize input to spend [%s]", in)
		}
		c := &capture{}
		if _, err := ctx.SignatureProvider.HasBeenSignedBy(tok.Owner, c); err != nil {
			return errors.Wrapf(err, "failed signature verification [%s]", in) // insufficient signatures
		}
		tokens, sigs = append(tokens, tok), append(sigs, c.sigma)
		items = append(items, OwnerSig{Owner: tok.Owner, Msg: c.msg, Sig: c.sigma})
	}
	codes, err := o.Verify(items)
	if err != nil {
		return err
	}
	for i, c := range codes {
		switch c {
		case C.FTZ_OK:
		case C.FTZ_ERR_UNSUPPORTED:
			verifier, err := ctx.Deserializer.GetOwnerVerifier(tokens[i].Owner)
			if err != nil {
				return errors.Wrapf(err, "failed deserializing owner [%d][%s]", i, inputs[i])
			}
			if err := verifier.Verify(items[i].Msg, sigs[i]); err != nil {
				return errors.Wrapf(err, "failed signature verification [%d][%s]", i, inputs[i])
			}
		case C.FTZ_ERR_OWNER:
			return errors.Errorf("failed deserializing owner [%d][%s]", i, inputs[i])
		default:
			return errors.Errorf("failed signature verification [%d][%s]: pseudonym signature invalid", i, inputs[i])
		}
	}
	ctx.InputTokens, ctx.Signatures = tokens, sigs
	return nil
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

"""Owner-signature error precedence: the reference's
TransferSignatureValidate (crypto/validator/validator_transfer.go:50-76)
deserializes input i's owner, consumes its signature and verifies it before it
loads input i+1.  The shim batches the signatures (go/gpu/owner.go
transferSignatures; the Python mirror zkatdlog.transfer_signature_validate)
and must still return the reference's first error with its text, UniqueID
suffix included.  The same cases as go/gpu/gpu_test.go
TestTransferSignaturePrecedence; the batch verifier is a stub returning fixed
FTZ codes (host logic only, no GPU)."""
import pytest

import zkatdlog
from zkatdlog import _abi as A

KEYS = ["k0", "k1"]


def uid(k):
    return zkatdlog._unique_id(b"owner-" + k.encode())


def run(nsig, codes, bad_owner=None, go_verdict=None):
    state = {"cursor": 0}

    def load(key):
        return b"owner-" + key.encode()

    class GoVerifier:
        def verify(self, m, s):
            if go_verdict:
                raise ValueError(go_verdict)

    def owner_verifier(owner):
        if bad_owner is not None and owner == b"owner-k%d" % bad_owner:
            raise ValueError("bad nym")
        return GoVerifier()

    def signed(owner, verifier):
        if state["cursor"] >= nsig:
            raise ValueError("invalid state, insufficient number of signatures")
        state["cursor"] += 1
        verifier.verify(b"msg", b"sig")
        return b"sig"

    return zkatdlog.transfer_signature_validate(KEYS, load, owner_verifier, signed,
                                                lambda items: codes[:len(items)], unique_id=zkatdlog._unique_id)


PSEUDO = zkatdlog.PSEUDONYM_INVALID


@pytest.mark.parametrize("nsig,codes,bad_owner,want", [
    (1, [A.FTZ_ERR_SIGNATURE, 0], None, "failed signature verification [0][k0][%s]: " + PSEUDO),
    (1, [0, 0], None, "failed signature verification [1][k1][%s]: invalid state, insufficient number of signatures"),
    (2, [A.FTZ_ERR_SIGNATURE, 0], 1, "failed signature verification [0][k0][%s]: " + PSEUDO),
    (2, [0, 0], 1, "failed deserializing owner [1][k1][%s]: bad nym"),
    (2, [0, A.FTZ_ERR_SIGNATURE], None, "failed signature verification [1][k1][%s]: " + PSEUDO),
])
def test_first_error_in_reference_order(nsig, codes, bad_owner, want):
    key = want.split("[")[2].split("]")[0]
    with pytest.raises(zkatdlog.SignatureError) as e:
        run(nsig, codes, bad_owner)
    assert str(e.value) == want % uid(key)


def test_all_good_returns_tokens_and_signatures():
    out = run(2, [0, 0])
    assert out == [(b"owner-k0", b"sig"), (b"owner-k1", b"sig")]


def test_unsupported_owner_goes_to_the_go_verifier():
    """FTZ_ERR_UNSUPPORTED (HTLC script owners) and FTZ_ERR_OWNER (the library
    decodes an owner the Go deserializer accepted differently): the Go
    verifier's own verdict and text"""
    assert run(2, [A.FTZ_ERR_UNSUPPORTED, A.FTZ_ERR_OWNER])
    with pytest.raises(zkatdlog.SignatureError) as e:
        run(2, [A.FTZ_ERR_UNSUPPORTED, 0], go_verdict="htlc: bad preimage")
    assert str(e.value) == "failed signature verification [0][k0][%s]: htlc: bad preimage" % uid("k0")

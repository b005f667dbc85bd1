"""TEST INFRASTRUCTURE ONLY -- oracle restatement of the raw token-request
path; nothing in the product imports it.

* driver.TokenRequest{Issues, Transfers, Signatures, AuditorSignatures [][]byte}
  (token/driver/request.go:24-38) as Go 1.18 encoding/asn1 Unmarshal reads it
  in FromBytes (:35-38): parseTagAndLength (definite, minimal lengths; long form
  only for >= 128; no leading zero length bytes; < 2^31), parseField on the
  struct (SEQUENCE, extra trailing elements inside it ignored), parseSequenceOf
  for [][]byte (every element a primitive universal OCTET STRING), trailing
  bytes after the outer SEQUENCE ignored (FromBytes drops `rest`).
* transfer.TransferAction (crypto/transfer/sender.go:105-116, Deserialize
  :179-181), issue.IssueAction (crypto/issue/issue.go:20-31, OutputTokens
  tagged json:"outputs"; Deserialize :89-91), token.Token
  (crypto/token/token.go:20-25, Deserialize :38-40) through the Go
  encoding/json restatement in gojson.py; math.G1 UnmarshalJSON decodes its
  bytes (gnark SetBytes) at unmarshal time.
* Validator.VerifyTokenRequestFromRaw / VerifyTokenRequest
  (crypto/validator/validator.go:45-108): unmarshal all issue actions, then all
  transfer actions (any failure rejects the request); then every issue
  (verifyIssue :181-191: GetCommitments fails on a nil output, issue.go:94-103)
  and every transfer (TransferSignatureValidate's ledger loads,
  validator_transfer.go:42-81, then TransferZKProofValidate :84-98) in order.
  The signature, HTLC and metadata checks stay in Go and are not restated.
"""
from . import bn254 as C
from . import gojson as J
from . import zkat as Z

ERR_INPUT = 8  # an input to spend is missing on the ledger or is not a token.Token


class Asn1Error(Exception):
    pass


def _header(b, off, want):
    if off >= len(b):
        raise Asn1Error("sequence truncated")
    ident = b[off]
    off += 1
    if ident & 0x1F == 0x1F or ident != want:
        raise Asn1Error("tags don't match")
    if off >= len(b):
        raise Asn1Error("truncated tag or length")
    first = b[off]
    off += 1
    if first & 0x80:
        nb = first & 0x7F
        if nb == 0:
            raise Asn1Error("indefinite length found (not DER)")
        length = 0
        for _ in range(nb):
            if off >= len(b):
                raise Asn1Error("truncated tag or length")
            v = b[off]
            off += 1
            if length >= 1 << 23:
                raise Asn1Error("length too large")
            length = (length << 8) | v
            if length == 0:
                raise Asn1Error("superfluous leading zeros in length")
        if length < 0x80:
            raise Asn1Error("non-minimal length")
    else:
        length = first
    if length > len(b) - off:
        raise Asn1Error("data truncated")
    return off, length


def der_token_request(raw):
    """-> [issues, transfers, signatures, auditor_signatures] (lists of bytes)."""
    raw = bytes(raw)
    if not raw:
        raise Asn1Error("empty token request")
    off, body = _header(raw, 0, 0x30)
    inner = raw[off:off + body]
    k = 0
    out = []
    for _ in range(4):
        k, L = _header(inner, k, 0x30)
        seq = inner[k:k + L]
        items, j = [], 0
        while j < len(seq):
            j, el = _header(seq, j, 0x04)
            items.append(seq[j:j + el])
            j += el
        out.append(items)
        k += L
    return out


def _der_len(n):
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def der_encode_token_request(fields):
    """asn1.Marshal(TokenRequest) for four lists of byte strings (fixture maker)."""
    def seq(body):
        return b"\x30" + _der_len(len(body)) + body
    return seq(b"".join(seq(b"".join(b"\x04" + _der_len(len(x)) + x for x in f)) for f in fields))


# ---------------------------------------------------------------- JSON actions
class _Elem:
    """A decoded math.G1 field: nil, a point, or a foreign-curve element (the
    reference panics when the verifier uses it)."""

    def __init__(self, kind, point=None):
        self.kind, self.point = kind, point  # "nil" | "ok" | "foreign"


def _g1(v):
    e = J.dec_elem(v)
    if e is None:
        return _Elem("nil")
    curve, raw = e
    if curve != J.BN254:
        return _Elem("foreign")
    try:
        return _Elem("ok", C.g1_from_bytes(raw))
    except C.DecodeError as ex:
        raise J.GoJSONError("math.G1: %s" % ex)


def _top(raw):
    v = J.parse(raw)
    if v[0] == "null":
        return None
    if v[0] != "obj":
        raise J.GoJSONError("cannot unmarshal %s into struct" % v[0])
    return v


def _outputs(v):
    """[]*token.Token -> list of _Elem (a nil token -> None)."""
    if v is None or v[0] == "null":
        return []
    if v[0] != "arr":
        raise J.GoJSONError("cannot unmarshal into []*token.Token")
    out = []
    for t in v[1]:
        if t[0] == "null":
            out.append(None)
            continue
        if t[0] != "obj":
            raise J.GoJSONError("cannot unmarshal into token.Token")
        J.dec_bytes(J.field(t, "Owner"))
        out.append(_g1(J.field(t, "Data")))
    return out


def _metadata(v):
    if v is None or v[0] == "null":
        return
    if v[0] != "obj":
        raise J.GoJSONError("cannot unmarshal into map[string][]byte")
    for _, x in v[1]:
        J.dec_bytes(x)


# []*token.Token fields: duplicate keys merge into the existing tokens (gojson.resolve)
TRANSFER_SCHEMA = {"OutputTokens": (J.SLICE, {})}
ISSUE_SCHEMA = {"outputs": (J.SLICE, {})}


def decode_transfer_action(raw):
    v = _top(raw)
    a = {"inputs": [], "outputs": [], "proof": None}
    if v is None:
        return a
    v = J.resolve(v, TRANSFER_SCHEMA)
    ins = J.field(v, "Inputs")
    if ins is not None and ins[0] != "null":
        if ins[0] != "arr":
            raise J.GoJSONError("cannot unmarshal into []string")
        a["inputs"] = [J.dec_string(x) for x in ins[1]]
    ic = J.field(v, "InputCommitments")
    if ic is not None and ic[0] != "null":
        if ic[0] != "arr":
            raise J.GoJSONError("cannot unmarshal into []*math.G1")
        for x in ic[1]:
            _g1(x)
    a["outputs"] = _outputs(J.field(v, "OutputTokens"))
    a["proof"] = J.dec_bytes(J.field(v, "Proof"))
    _metadata(J.field(v, "Metadata"))
    return a


def decode_issue_action(raw):
    v = _top(raw)
    a = {"outputs": [], "proof": None, "anonymous": False}
    if v is None:
        return a
    v = J.resolve(v, ISSUE_SCHEMA)
    J.dec_bytes(J.field(v, "Issuer"))
    a["outputs"] = _outputs(J.field(v, "outputs"))
    a["proof"] = J.dec_bytes(J.field(v, "Proof"))
    an = J.field(v, "Anonymous")
    if an is not None and an[0] != "null":
        if an[0] != "bool":
            raise J.GoJSONError("cannot unmarshal into bool")
        a["anonymous"] = an[1]
    _metadata(J.field(v, "Metadata"))
    return a


def decode_token(raw):
    """token.Token.Deserialize -> _Elem of Data."""
    v = _top(raw)
    if v is None:
        return _Elem("nil")
    J.dec_bytes(J.field(v, "Owner"))
    return _g1(J.field(v, "Data"))


# ---------------------------------------------------------------- validation
def _zk(pp, kind, ins, outs, proof, anonymous):
    if kind == "issue":
        return Z.issue_verify(pp, outs, proof, anonymous)[1]
    return Z.transfer_verify(pp, ins, outs, proof)[1]


def verify_token_request(pp, raw, get_state, zk=_zk):
    """-> (code, failed_action_index or -1).  get_state(key: str) -> bytes or
    None (missing / error).  zk(pp, kind, ins, outs, proof, anonymous) -> code
    is the action verifier (default: the oracle's issue_verify /
    transfer_verify; the fixture maker passes a memo of the golden corpus)."""
    try:
        fields = der_token_request(raw)
        issues = [decode_issue_action(x) for x in fields[0]]
        transfers = [decode_transfer_action(x) for x in fields[1]]
    except (Asn1Error, J.GoJSONError):
        return Z.ERR_PARSE, -1
    for k, a in enumerate(issues):
        if any(o is None for o in a["outputs"]):
            return Z.ERR_MALFORMED, k  # "invalid issue: there is a nil output" -> "failed to verify issue"
        if any(o.kind != "ok" for o in a["outputs"]):
            return Z.ERR_PANIC, k
        code = zk(pp, "issue", [], [o.point for o in a["outputs"]], a["proof"] or b"", a["anonymous"])
        if code != Z.OK:
            return code, k
    for t, a in enumerate(transfers):
        at = len(issues) + t
        ins = []
        for key in a["inputs"]:
            val = get_state(key)
            if not val:
                return ERR_INPUT, at
            try:
                ins.append(decode_token(val))
            except J.GoJSONError:
                return ERR_INPUT, at
        if any(o is None or o.kind != "ok" for o in a["outputs"]) or any(e.kind != "ok" for e in ins):
            return Z.ERR_PANIC, at
        code = zk(pp, "transfer", [e.point for e in ins], [o.point for o in a["outputs"]], a["proof"] or b"", False)
        if code != Z.OK:
            return code, at
    return Z.OK, -1

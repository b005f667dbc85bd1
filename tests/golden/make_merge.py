#!/usr/bin/env python3
"""Make tests/golden/json_merge_cases.json: proofs and public parameters whose
JSON repeats a struct-typed key (Go 1.18 encoding/json merges such a value
into the one already decoded instead of replacing it; ftsoracle.gojson.resolve),
each with the oracle's verdict.  Test data only.

Proof cases rewrite the RangeCorrectness document of golden PP-A proofs
(range/proof.go:25-57 RangeProof -> EqualityProofs, []*MembershipProof ->
[]*sigproof.MembershipProof -> *pssign.Signature); PP cases rewrite the
RangeProofParams of the golden PP-A (setup.go:25-54) and carry
PublicParams.Validate's answer.

    python tests/golden/make_merge.py
"""
import base64
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle", "py"))
from ftsoracle import bn254 as C  # noqa: E402
from ftsoracle import gojson as J  # noqa: E402
from ftsoracle import zkat as Z  # noqa: E402

NULL = ("null", None)


def dump(v):
    """compact JSON text of a parsed value (members kept in order, duplicates kept)"""
    t = v[0]
    if t == "obj":
        return "{" + ",".join(J.enc_str(k) + ":" + dump(x) for k, x in v[1]) + "}"
    if t == "arr":
        return "[" + ",".join(dump(x) for x in v[1]) + "]"
    if t == "str":
        return J.enc_str(v[1])
    if t == "null":
        return "null"
    if t == "bool":
        return "true" if v[1] else "false"
    return v[1]  # number token


def get(o, k):
    return next(x for kk, x in o[1] if kk == k)


def only(o, keys):
    return ("obj", [(k, x) for k, x in o[1] if k in keys])


def without(o, keys):
    return ("obj", [(k, x) for k, x in o[1] if k not in keys])


def replace(o, k, members):
    """o with member k replaced by the list of (key, value) members"""
    out = []
    for kk, x in o[1]:
        out.extend(members if kk == k else [(kk, x)])
    return ("obj", out)


def flip_zr(z):
    """a mathlib Zr element with its last byte flipped"""
    raw = bytearray(base64.b64decode(get(z, "element")[1]))
    raw[-1] ^= 1
    return replace(z, "element", [("element", ("str", base64.b64encode(bytes(raw)).decode()))])


def rebuild(proof, rc):
    outer = J.parse(proof)
    return J.enc_struct([("WellFormedness", J.enc_bytes(J.dec_bytes(J.field(outer, "WellFormedness")))),
                         ("RangeCorrectness", J.enc_bytes(dump(rc).encode()))]).encode()


def rc_of(proof):
    return J.parse(J.dec_bytes(J.field(J.parse(proof), "RangeCorrectness")))


def main():
    g = json.load(open(os.path.join(HERE, "zkatdlog_golden.json")))["pp_a"]
    pp = Z.PublicParams.from_json(g["pp"].encode())
    cases = {c["name"]: c for c in g["cases"]}
    rows = []

    def add(name, base, rc):
        c = cases[base]
        proof = rebuild(base64.b64decode(c["proof"]), rc)
        outs = [C.g1_from_bytes(bytes.fromhex(c["outputs"])[64 * i:64 * i + 64])
                for i in range(len(c["outputs"]) // 128)]
        if c["kind"] == "issue":
            code = Z.issue_verify(pp, outs, proof, c["anonymous"])[1]
        else:
            ins = [C.g1_from_bytes(bytes.fromhex(c["inputs"])[64 * i:64 * i + 64])
                   for i in range(len(c["inputs"]) // 128)]
            code = Z.transfer_verify(pp, ins, outs, proof)[1]
        rows.append({"name": name, "base": base, "kind": c["kind"], "inputs": c.get("inputs", ""),
                     "outputs": c["outputs"], "anonymous": c.get("anonymous", False),
                     "proof": base64.b64encode(proof).decode(), "expect": code})

    for base in ("valid_2in_2out", "issue_valid_1"):
        rc = rc_of(base64.b64decode(cases[base]["proof"]))
        eq = get(rc, "EqualityProofs")
        mps = get(rc, "MembershipProofs")
        n = len(mps[1])
        tag = "t" if base.startswith("valid") else "i"
        # *EqualityProofs: two partial objects merge
        add(tag + "_eq_split_merges", base, replace(rc, "EqualityProofs", [
            ("EqualityProofs", only(eq, ("Type", "Value"))),
            ("equalityProofs", without(eq, ("Type", "Value")))]))
        add(tag + "_eq_null_resets", base, replace(rc, "EqualityProofs", [
            ("EqualityProofs", eq), ("EqualityProofs", NULL)]))
        add(tag + "_eq_null_between", base, replace(rc, "EqualityProofs", [
            ("EqualityProofs", only(eq, ("Type", "Value"))), ("EqualityProofs", NULL),
            ("EqualityProofs", without(eq, ("Type", "Value")))]))
        add(tag + "_eq_later_leaf_wins", base, replace(rc, "EqualityProofs", [
            ("EqualityProofs", replace(eq, "Type", [("Type", flip_zr(get(eq, "Type")))])),
            ("EqualityProofs", only(eq, ("Type",)))]))
        add(tag + "_eq_bad_type_first", base, replace(rc, "EqualityProofs", [
            ("EqualityProofs", ("str", "x")), ("EqualityProofs", eq)]))
        # []*MembershipProof: element-wise merge, truncation keeps the backing array
        add(tag + "_mps_fieldwise_merge", base, replace(rc, "MembershipProofs", [
            ("MembershipProofs", ("arr", [only(m, ("Commitments",)) for m in mps[1]])),
            ("MembershipProofs", ("arr", [only(m, ("SignatureProofs",)) for m in mps[1]]))]))
        add(tag + "_mps_truncated_then_reexposed", base, replace(rc, "MembershipProofs", [
            ("MembershipProofs", ("arr", mps[1] + [mps[1][0]])),
            ("MembershipProofs", ("arr", [("obj", [])])),
            ("MembershipProofs", ("arr", [("obj", [])] * n))]))
        add(tag + "_mps_empty_array_resets", base, replace(rc, "MembershipProofs", [
            ("MembershipProofs", mps), ("MembershipProofs", ("arr", [])),
            ("MembershipProofs", ("arr", [("obj", [])] * n))]))
        add(tag + "_mps_null_resets", base, replace(rc, "MembershipProofs", [
            ("MembershipProofs", mps), ("MembershipProofs", NULL),
            ("MembershipProofs", ("arr", [only(m, ("Commitments",)) for m in mps[1]]))]))
        add(tag + "_mps_null_element_resets", base, replace(rc, "MembershipProofs", [
            ("MembershipProofs", mps), ("MembershipProofs", ("arr", [NULL] + [("obj", [])] * (n - 1)))]))
        # []*sigproof.MembershipProof inside element 0, and its *pssign.Signature
        m0 = mps[1][0]
        sps = get(m0, "SignatureProofs")
        sp0 = sps[1][0]
        sig = get(sp0, "Signature")
        bad_sp0 = replace(sp0, "Value", [("Value", flip_zr(get(sp0, "Value")))])
        fixed = replace(m0, "SignatureProofs", [
            ("SignatureProofs", ("arr", [bad_sp0] + sps[1][1:])),
            ("SignatureProofs", ("arr", [only(sp0, ("Value",))] + [("obj", [])] * (len(sps[1]) - 1)))])
        add(tag + "_sigproofs_later_value_repairs", base,
            replace(rc, "MembershipProofs", [("MembershipProofs", ("arr", [fixed] + mps[1][1:]))]))
        split_sig = replace(sp0, "Signature", [("Signature", only(sig, ("R",))), ("Signature", only(sig, ("S",)))])
        add(tag + "_signature_split_merges", base, replace(rc, "MembershipProofs", [("MembershipProofs", ("arr", [
            replace(m0, "SignatureProofs", [("SignatureProofs", ("arr", [split_sig] + sps[1][1:]))])] + mps[1][1:]))]))
        null_sig = replace(sp0, "Signature", [("Signature", sig), ("Signature", NULL)])
        add(tag + "_signature_null_resets", base, replace(rc, "MembershipProofs", [("MembershipProofs", ("arr", [
            replace(m0, "SignatureProofs", [("SignatureProofs", ("arr", [null_sig] + sps[1][1:]))])] + mps[1][1:]))]))

    # public parameters: *RangeProofParams and its []*pssign.Signature
    outer = J.parse(g["pp"].encode())
    raw = J.parse(J.dec_bytes(J.field(outer, "Raw")))
    rpp = get(raw, "RangeProofParams")
    sv = get(rpp, "SignedValues")

    def pp_case(name, doc):
        js = J.enc_struct([("Identifier", J.enc_str("zkatdlog")),
                           ("Raw", J.enc_bytes(dump(doc).encode()))]).encode()
        return {"name": name, "pp": js.decode(), "error": Z.validate_json(js)}

    pps = [
        pp_case("pp_rpp_split_merges", replace(raw, "RangeProofParams", [
            ("RangeProofParams", only(rpp, ("SignPK", "Q"))),
            ("RangeProofParams", without(rpp, ("SignPK", "Q")))])),
        pp_case("pp_rpp_null_between_loses_q", replace(raw, "RangeProofParams", [
            ("RangeProofParams", only(rpp, ("SignPK", "Q"))), ("RangeProofParams", NULL),
            ("RangeProofParams", without(rpp, ("SignPK", "Q")))])),
        pp_case("pp_signed_values_fieldwise", replace(raw, "RangeProofParams", [("RangeProofParams", replace(
            rpp, "SignedValues", [("SignedValues", ("arr", [only(s, ("R",)) for s in sv[1]])),
                                  ("SignedValues", ("arr", [only(s, ("S",)) for s in sv[1]]))]))])),
        pp_case("pp_signed_values_null_element", replace(raw, "RangeProofParams", [("RangeProofParams", replace(
            rpp, "SignedValues", [("SignedValues", sv), ("SignedValues", ("arr", [NULL] + [("obj", [])] * (len(sv[1]) - 1)))]))])),
    ]
    out = {"generator": "tests/golden/make_merge.py", "oracle": "ftsoracle.gojson.resolve + zkat.transfer_verify / "
           "issue_verify / validate_json (PP-A)", "pp": g["pp"], "proofs": rows, "pp_validate": pps}
    with open(os.path.join(HERE, "json_merge_cases.json"), "w") as f:
        json.dump(out, f, indent=0)
    for r in rows:
        print("%-40s %d" % (r["name"], r["expect"]))
    for p in pps:
        print("%-40s %r" % (p["name"], p["error"]))


if __name__ == "__main__":
    main()

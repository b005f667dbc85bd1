#!/usr/bin/env python3
"""Fixture maker for the raw token-request path (tests/golden/token_requests.json).

Requests are asn1.Marshal(driver.TokenRequest) built from the golden proof
corpus (zkatdlog_golden.json, PP-A): issue / transfer actions are Go
json.Marshal of issue.IssueAction / transfer.TransferAction, ledger inputs are
json.Marshal(token.Token).  Expected verdicts come from the oracle's
ftsoracle.request.verify_token_request, with the action ZK checks answered by
the corpus's own (oracle-made) verdicts so that the maker runs in seconds;
tests/test_requests.py re-runs the oracle with real ZK on a few requests.

    python tests/golden/make_requests.py
"""
import base64
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle", "py"))
from ftsoracle import bn254 as C  # noqa: E402
from ftsoracle import gojson as J  # noqa: E402
from ftsoracle import request as R  # noqa: E402
from ftsoracle import zkat as Z  # noqa: E402

OWNER = b"owner-identity"


def elem(raw, curve=1):
    return J.enc_elem(raw, curve)


def token_json(raw, curve=1, owner=OWNER):
    return J.enc_struct([("Owner", J.enc_bytes(owner)), ("Data", elem(raw, curve))])


def transfer_json(keys, in_raw, out_raws, proof, out_override=None, in_coms=None, metadata="null"):
    outs = out_override if out_override is not None else [token_json(r) for r in out_raws]
    ic = in_coms if in_coms is not None else [elem(r) for r in in_raw]
    return J.enc_struct([("Inputs", J.enc_list(keys, J.enc_str)), ("InputCommitments", "[" + ",".join(ic) + "]"),
                         ("OutputTokens", "[" + ",".join(outs) + "]"), ("Proof", J.enc_bytes(proof)),
                         ("Metadata", metadata)]).encode()


def issue_json(out_raws, proof, anonymous, out_override=None, key="outputs"):
    outs = out_override if out_override is not None else [token_json(r) for r in out_raws]
    return J.enc_struct([("Issuer", J.enc_bytes(b"issuer")), (key, "[" + ",".join(outs) + "]"),
                         ("Proof", J.enc_bytes(proof)), ("Anonymous", "true" if anonymous else "false"),
                         ("Metadata", "{}")]).encode()


def split(h):
    b = bytes.fromhex(h)
    return [b[64 * i:64 * i + 64] for i in range(len(b) // 64)]


def compress(raw):
    x, y = C.g1_from_bytes(raw)
    flag = 0xC0 if y > (-y) % C.P else 0x80
    return bytes([flag | (x >> 248)]) + (x % (1 << 248)).to_bytes(31, "big")


def main():
    g = json.load(open(os.path.join(HERE, "zkatdlog_golden.json")))["pp_a"]
    pp = Z.PublicParams.from_json(g["pp"].encode())
    cases = {c["name"]: c for c in g["cases"]}
    memo = {}  # (kind, ins, outs, proof, anon) -> corpus verdict
    for c in g["cases"]:
        outs = tuple(C.g1_from_bytes(r) for r in split(c["outputs"]))
        proof = base64.b64decode(c["proof"])
        if c["kind"] == "transfer":
            ins = tuple(C.g1_from_bytes(r) for r in split(c["inputs"]))
            memo[("transfer", ins, outs, proof, False)] = c["expect"]
        else:
            memo[("issue", (), outs, proof, bool(c["anonymous"]))] = c["expect"]

    def zk(_pp, kind, ins, outs, proof, anonymous):
        key = (kind, tuple(ins), tuple(outs), proof, bool(anonymous))
        if key not in memo:  # not a corpus proof (e.g. an empty action): the real oracle
            memo[key] = R._zk(_pp, kind, ins, outs, proof, anonymous)
        return memo[key]

    ledger = {}
    counter = [0]

    def tr(name, **kw):
        c = cases[name]
        ins = split(c["inputs"])
        keys = []
        for r in ins:
            k = "tx%04d:%d" % (counter[0], len(keys))
            counter[0] += 1
            ledger[k] = token_json(r).encode()
            keys.append(k)
        return transfer_json(keys, ins, split(c["outputs"]), base64.b64decode(c["proof"]), **kw), keys

    def iss(name, **kw):
        c = cases[name]
        return issue_json(split(c["outputs"]), base64.b64decode(c["proof"]), c["anonymous"], **kw)

    enc = R.der_encode_token_request
    reqs = []

    def add(name, raw, note=""):
        reqs.append({"name": name, "raw": base64.b64encode(raw).decode(), "note": note})

    t0, _ = tr("valid_2in_2out")
    t1, _ = tr("valid_3in_1out")
    t2, _ = tr("valid_1in_3out")
    t3, _ = tr("valid_ownership_1in_1out")
    i0, i1, i2 = iss("issue_valid_0"), iss("issue_valid_1"), iss("issue_valid_2_anon")
    sigs = [b"sig-0", b"sig-1"]
    add("valid_mixed", enc([[i0, i1], [t0, t1, t2], sigs, [b"auditor-sig"]]))
    add("valid_issues_only", enc([[i2], [], [], []]))
    add("valid_transfers_only", enc([[], [t3, t0], sigs, []]))
    add("valid_empty", enc([[], [], [], []]), "no actions: nothing to verify")
    tw, _ = tr("wf_challenge_bitflip")
    add("transfer_wf_fails_at_2", enc([[i0], [t0, tw, t1], [], []]))
    add("first_failure_issue_wins", enc([[i0, iss("issue_range_challenge")], [tw], [], []]))
    tm, _ = tr("membership_challenge_bitflip")
    add("transfer_membership", enc([[], [tm], [], []]))
    tp, _ = tr("range_null_sigproof_panics")
    add("transfer_panics", enc([[], [t0, tp], [], []]))
    add("issue_anonymous_mismatch", enc([[iss("issue_as_anonymous_mismatch")], [], [], []]))
    # ledger failures
    tmiss = transfer_json(["no-such-key"], split(cases["valid_2in_2out"]["inputs"])[:1],
                          split(cases["valid_2in_2out"]["outputs"]), base64.b64decode(cases["valid_2in_2out"]["proof"]))
    add("input_missing", enc([[i0], [t0, tmiss], [], []]))
    ledger["bad-json-token"] = b"{not json"
    ledger["off-curve-token"] = token_json(b"\x00" * 63 + b"\x05").encode()
    ledger["nil-data-token"] = b'{"Owner":"b3duZXI=","Data":null}'
    ledger["foreign-data-token"] = token_json(split(cases["valid_2in_2out"]["inputs"])[0], curve=0).encode()
    for key, nm in (("bad-json-token", "input_not_json"), ("off-curve-token", "input_off_curve"),
                    ("nil-data-token", "input_nil_data_panics"), ("foreign-data-token", "input_foreign_curve_panics")):
        c = cases["valid_ownership_1in_1out"]
        raw = transfer_json([key], split(c["inputs"]), split(c["outputs"]), base64.b64decode(c["proof"]))
        add(nm, enc([[], [raw], [], []]))
    # output-token shapes
    c = cases["valid_2in_2out"]
    outs = split(c["outputs"])
    good = [token_json(r) for r in outs]
    t_nil_tok, _ = tr("valid_2in_2out", out_override=[good[0], "null"])
    add("transfer_nil_output_token_panics", enc([[], [t_nil_tok], [], []]))
    t_nil_data, _ = tr("valid_2in_2out", out_override=[good[0], '{"Owner":"eA==","Data":null}'])
    add("transfer_nil_output_data_panics", enc([[], [t_nil_data], [], []]))
    t_foreign, _ = tr("valid_2in_2out", out_override=[good[0], token_json(outs[1], curve=2)])
    add("transfer_foreign_output_panics", enc([[], [t_foreign], [], []]))
    t_comp, _ = tr("valid_2in_2out", out_override=[good[0], token_json(compress(outs[1]))])
    add("transfer_compressed_output_accepts", enc([[], [t_comp], [], []]))
    off = bytearray(outs[1])
    off[63] ^= 1
    t_off, _ = tr("valid_2in_2out", out_override=[good[0], token_json(bytes(off))])
    add("transfer_off_curve_output_rejects_request", enc([[iss("issue_wrong_type_in_clear")], [t0, t_off], [], []]),
        "an undecodable math.G1 fails unmarshalTransferActions before any verification")
    t_short, _ = tr("valid_2in_2out", out_override=[good[0], token_json(outs[1][:40])])
    add("transfer_short_output_rejects_request", enc([[], [t_short], [], []]))
    t_foreign_ic, _ = tr("valid_2in_2out", in_coms=[elem(split(c["inputs"])[0], curve=0), elem(split(c["inputs"])[1])])
    add("transfer_foreign_input_commitment_ignored", enc([[], [t_foreign_ic], [], []]),
        "InputCommitments are decoded but the verifier uses the ledger's tokens")
    bad_ic = bytearray(split(c["inputs"])[0])
    bad_ic[63] ^= 1
    t_bad_ic, _ = tr("valid_2in_2out", in_coms=[elem(bytes(bad_ic)), elem(split(c["inputs"])[1])])
    add("transfer_off_curve_input_commitment_rejects_request", enc([[], [t_bad_ic], [], []]))
    i_nil = iss("issue_valid_0", out_override=[token_json(split(cases["issue_valid_0"]["outputs"])[0]), "null"])
    add("issue_nil_output_malformed", enc([[i_nil], [], [], []]))
    i_upper = iss("issue_valid_0", key="OUTPUTS")
    add("issue_outputs_key_case_insensitive", enc([[i_upper], [], [], []]))
    t_meta, _ = tr("valid_2in_2out", metadata='{"k":"dmFsdWU=","n":null}')
    add("transfer_metadata_ok", enc([[], [t_meta], [], []]))
    t_meta_bad, _ = tr("valid_2in_2out", metadata='{"k":"!!"}')
    add("transfer_metadata_bad_base64", enc([[], [t_meta_bad], [], []]))
    add("transfer_action_null_json", enc([[], [b"null"], [], []]), "null leaves the action empty: Verify(nil) fails")
    add("transfer_action_not_json", enc([[i0], [b"{", t0], [], []]))
    add("transfer_action_array", enc([[], [b"[]"], [], []]))
    add("transfer_inputs_not_list", enc([[], [b'{"Inputs":"x"}'], [], []]))
    add("issue_anonymous_not_bool", enc([[b'{"Anonymous":1}'], [], [], []]))
    # ASN.1 shapes
    ok = enc([[i2], [], [], []])
    add("asn1_empty", b"")
    add("asn1_trailing_bytes_after_sequence_ignored", ok + b"\x00\x01garbage")
    body = ok[2:] if ok[1] < 0x80 else ok[2 + (ok[1] & 0x7F):]
    add("asn1_extra_field_inside_sequence_ignored", b"\x30" + R._der_len(len(body) + 5) + body + b"\x04\x03abc")
    add("asn1_wrong_outer_tag", b"\x31" + ok[1:])
    add("asn1_indefinite_length", b"\x30\x80" + body + b"\x00\x00")
    add("asn1_truncated", ok[:-3])
    add("asn1_long_form_small_length", b"\x30\x81\x08" + b"\x30\x00" * 4)
    add("asn1_leading_zero_length", b"\x30\x82\x00\x08" + b"\x30\x00" * 4)
    add("asn1_minimal_empty", b"\x30\x08" + b"\x30\x00" * 4)
    add("asn1_missing_field", b"\x30\x06" + b"\x30\x00" * 3)
    add("asn1_constructed_octet_string", b"\x30\x0b" + b"\x30\x05\x24\x03\x04\x01x" + b"\x30\x00" * 3)
    add("asn1_wrong_element_tag", b"\x30\x0b" + b"\x30\x05\x0c\x03abc" + b"\x30\x00" * 3)
    add("asn1_high_tag_form", b"\x30\x09" + b"\x3f\x10\x00" + b"\x30\x00" * 3)
    add("asn1_element_overruns_sequence", b"\x30\x0b" + b"\x30\x03\x04\x05abc" + b"\x30\x00" * 3 + b"de")
    # duplicate []*token.Token keys: Go decodes the later array INTO the tokens
    # already there (gojson.resolve), so fields the later occurrence omits survive
    own = '{"Owner":"eA=="}'

    def dup(raw, key, before):
        k = ('"%s":[' % key).encode()
        assert raw.count(k) == 1
        return raw.replace(k, before.encode() + k)
    t_full, _ = tr("valid_2in_2out")
    # the full array first, then owner-only tokens: Data survives -> accept
    add("transfer_output_tokens_dup_merges_accepts",
        enc([[], [t_full.replace(b'"Proof":', ('"OutputTokens":[%s,%s],"Proof":' % (own, own)).encode())], [], []]))
    add("transfer_output_tokens_dup_null_resets_panics",
        enc([[], [t_full.replace(b'"Proof":', ('"OutputTokens":null,"OutputTokens":[%s,%s],"Proof":'
                                               % (own, own)).encode())], [], []]))
    # [full0, full1] -> [owner] truncates to 1 -> [{}, {}] re-exposes full1
    add("transfer_output_tokens_truncated_then_reexposed_accepts",
        enc([[], [t_full.replace(b'"Proof":', ('"OutputTokens":[%s],"outputtokens":[{},{}],"Proof":' % own).encode())],
             [], []]))
    add("transfer_output_tokens_empty_array_resets_panics",
        enc([[], [t_full.replace(b'"Proof":', b'"OutputTokens":[],"OutputTokens":[{},{}],"Proof":')], [], []]))
    i_dup = iss("issue_valid_1")
    n_iss = len(split(cases["issue_valid_1"]["outputs"]))
    add("issue_outputs_dup_merges_accepts",
        enc([[i_dup.replace(b'"Proof":', ('"OUTPUTS":[%s],"Proof":' % ",".join(["{}"] * n_iss)).encode())],
             [], [], []]))
    add("issue_outputs_dup_partial_first_accepts",
        enc([[dup(i_dup, "outputs", '"outputs":[%s],' % ",".join([own] * n_iss))], [], [], []]))

    get = ledger.get
    for r in reqs:
        code, at = R.verify_token_request(pp, base64.b64decode(r["raw"]), get, zk=zk)
        r["expect"], r["failed_action"] = code, at
    out = {"generator": "tests/golden/make_requests.py (oracle/py/ftsoracle/request.py, corpus verdicts for the ZK "
                        "checks)",
           "pp": g["pp"], "ledger": {k: base64.b64encode(v).decode() for k, v in ledger.items()}, "requests": reqs}
    with open(os.path.join(HERE, "token_requests.json"), "w") as f:
        json.dump(out, f, indent=1)
    for r in reqs:
        print("%-52s %d %d" % (r["name"], r["expect"], r["failed_action"]))


if __name__ == "__main__":
    main()

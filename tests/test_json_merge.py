"""Duplicate struct-typed JSON keys (tests/golden/json_merge_cases.json, made by
make_merge.py with the oracle's verdicts).

Go 1.18 encoding/json decodes a repeated *T / []*T key INTO the value already
there (decode.go indirect()/object()/array()): two partial EqualityProofs
objects merge, a later shorter MembershipProofs array re-exposes the earlier
elements past its length, null / [] reset.  The product decoder (go_merge in
csrc/host/gojson.cpp) must give the oracle's verdict on every case: host
emulation and ftz_pp_validate on the CPU, the C ABI on the GPU.  The
TransferAction / IssueAction OutputTokens cases live in token_requests.json
(test_requests.py)."""
import base64
import ctypes
import json
import os

import pytest
from conftest import ROOT

GOLD = os.path.join(ROOT, "tests", "golden", "json_merge_cases.json")


@pytest.fixture(scope="module")
def merge():
    with open(GOLD) as f:
        return json.load(f)


def _split(rows):
    tr = [(r, (bytes.fromhex(r["inputs"]), bytes.fromhex(r["outputs"]), base64.b64decode(r["proof"])))
          for r in rows if r["kind"] == "transfer"]
    iss = [(r, (bytes.fromhex(r["outputs"]), base64.b64decode(r["proof"]), r["anonymous"]))
           for r in rows if r["kind"] == "issue"]
    return tr, iss


def _check(rows, got):
    bad = {r["name"]: (v, r["expect"]) for (r, _), v in zip(rows, got) if v != r["expect"]}
    assert not bad, bad


def test_corpus_shape(merge):
    codes = [r["expect"] for r in merge["proofs"]]
    # merges that only Go's semantics accept, resets that reject, type errors
    assert codes.count(0) >= 12 and 1 in codes and 2 in codes
    assert {p["error"] == "" for p in merge["pp_validate"]} == {True, False}


def test_oracle_reproduces_a_sample(merge):
    from ftsoracle import bn254 as C
    from ftsoracle import zkat as Z
    pp = Z.PublicParams.from_json(merge["pp"].encode())
    for r in merge["proofs"][:6]:
        outs = [C.g1_from_bytes(bytes.fromhex(r["outputs"])[64 * i:64 * i + 64])
                for i in range(len(r["outputs"]) // 128)]
        ins = [C.g1_from_bytes(bytes.fromhex(r["inputs"])[64 * i:64 * i + 64]) for i in range(len(r["inputs"]) // 128)]
        assert Z.transfer_verify(pp, ins, outs, base64.b64decode(r["proof"]))[1] == r["expect"], r["name"]
    for p in merge["pp_validate"]:
        assert Z.validate_json(p["pp"].encode()) == p["error"], p["name"]


def test_pp_validate_merges(merge):
    import zkatdlog
    for p in merge["pp_validate"]:
        assert zkatdlog.validate_public_params(p["pp"].encode()) == p["error"], p["name"]


def test_emu_matches_oracle(emu, merge):
    from zkatdlog import _abi as A
    js = merge["pp"].encode()
    err = ctypes.create_string_buffer(256)
    ctx = emu.emu_ctx_create(js, len(js), err, 256)
    assert ctx, err.value
    try:
        tr, iss = _split(merge["proofs"])
        arr, keep = A.pack_transfers([t for _, t in tr])
        codes = (ctypes.c_int32 * len(tr))()
        emu.emu_verify_transfers(ctx, len(tr), arr, codes)
        _check(tr, list(codes))
        arr, keep = A.pack_issues([t for _, t in iss])
        codes = (ctypes.c_int32 * len(iss))()
        emu.emu_verify_issues(ctx, len(iss), arr, codes)
        _check(iss, list(codes))
    finally:
        emu.emu_ctx_destroy(ctx)


@pytest.mark.gpu
def test_gpu_matches_oracle(merge):
    import zkatdlog
    tr, iss = _split(merge["proofs"])
    with zkatdlog.Context(merge["pp"].encode(), device=0) as ctx:
        _check(tr, ctx.verify_transfers([t for _, t in tr]))
        _check(iss, ctx.verify_issues([t for _, t in iss]))

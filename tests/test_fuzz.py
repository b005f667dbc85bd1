"""Mutation fuzz corpus (tests/golden/fuzz_cases.json, made by make_fuzz.py with
the oracle's verdicts): 400 seeded mutations of valid PP-A and PP-B transfers and issues -- outer
bytes, inner document bytes, and single-bit flips inside well-formed base64
elements, which reach the curve checks, transcripts and pairings.  The host
emulation (CPU tier) and the GPU path (gpu tier) must return the oracle's
verdict for every case."""
import base64
import ctypes
import json
import os
import sys

import pytest
from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from fuzzmut import mutate  # noqa: E402


@pytest.fixture(scope="module")
def fuzz(golden):
    """{pp: (transfer rows, issue rows)}, each row (case record, verifier input)"""
    with open(os.path.join(ROOT, "tests", "golden", "fuzz_cases.json")) as f:
        fz = json.load(f)
    out = {}
    for r in fz["cases"]:
        c = {x["name"]: x for x in golden[r["pp"]]["cases"]}[r["base"]]
        tr, iss = out.setdefault(r["pp"], ([], []))
        proof = mutate(base64.b64decode(c["proof"]), r["mode"], r["pos"], r["xor"])
        if r["kind"] == "issue":
            iss.append((r, (bytes.fromhex(c["outputs"]), proof, c["anonymous"])))
        else:
            tr.append((r, (bytes.fromhex(c["inputs"]), bytes.fromhex(c["outputs"]), proof)))
    return out


def _check(rows, got):
    bad = {r["name"]: (v, r["expect"]) for (r, _), v in zip(rows, got) if v != r["expect"]}
    assert not bad, bad


def test_fuzz_corpus_shape(fuzz):
    rows = [r for tr, iss in fuzz.values() for r, _ in tr + iss]
    assert len(rows) >= 400 and set(fuzz) == {"pp_a", "pp_b"}
    assert len({r["expect"] for r in rows}) >= 6  # accept, parse, malformed, WF, range, membership, panic


def test_fuzz_emu_matches_oracle(emu, golden, fuzz):
    from zkatdlog import _abi as A
    for pp, (tr, iss) in fuzz.items():
        js = golden[pp]["pp"].encode()
        err = ctypes.create_string_buffer(256)
        ctx = emu.emu_ctx_create(js, len(js), err, 256)
        assert ctx, err.value
        try:
            if tr:
                arr, keep = A.pack_transfers([t for _, t in tr])
                codes = (ctypes.c_int32 * len(tr))()
                emu.emu_verify_transfers(ctx, len(tr), arr, codes)
                _check(tr, list(codes))
            if iss:
                arr, keep = A.pack_issues([t for _, t in iss])
                codes = (ctypes.c_int32 * len(iss))()
                emu.emu_verify_issues(ctx, len(iss), arr, codes)
                _check(iss, list(codes))
        finally:
            emu.emu_ctx_destroy(ctx)


@pytest.mark.gpu
def test_fuzz_gpu_matches_oracle(golden, fuzz):
    import zkatdlog
    for pp, (tr, iss) in fuzz.items():
        with zkatdlog.Context(golden[pp]["pp"].encode(), device=0) as ctx:
            if tr:
                _check(tr, ctx.verify_transfers([t for _, t in tr]))
            if iss:
                _check(iss, ctx.verify_issues([t for _, t in iss]))

"""Mutation fuzz corpus (tests/golden/fuzz_cases.json, made by make_fuzz.py with
the oracle's verdicts): 240 seeded mutations of valid PP-A transfers -- outer
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
    with open(os.path.join(ROOT, "tests", "golden", "fuzz_cases.json")) as f:
        fz = json.load(f)
    base = {c["name"]: c for c in golden["pp_a"]["cases"]}
    rows = []
    for r in fz["cases"]:
        c = base[r["base"]]
        rows.append((bytes.fromhex(c["inputs"]), bytes.fromhex(c["outputs"]),
                     mutate(base64.b64decode(c["proof"]), r["mode"], r["pos"], r["xor"])))
    return fz["cases"], rows


def test_fuzz_corpus_shape(fuzz):
    cases, _ = fuzz
    assert len(cases) >= 200
    assert len({c["expect"] for c in cases}) >= 5  # parse, malformed, WF, range, membership, panic classes


def test_fuzz_emu_matches_oracle(emu, golden, fuzz):
    from zkatdlog import _abi as A
    cases, rows = fuzz
    pp = golden["pp_a"]["pp"].encode()
    err = ctypes.create_string_buffer(256)
    ctx = emu.emu_ctx_create(pp, len(pp), err, 256)
    assert ctx, err.value
    try:
        arr, keep = A.pack_transfers(rows)
        codes = (ctypes.c_int32 * len(rows))()
        emu.emu_verify_transfers(ctx, len(rows), arr, codes)
    finally:
        emu.emu_ctx_destroy(ctx)
    bad = {c["name"]: (v, c["expect"]) for c, v in zip(cases, codes) if v != c["expect"]}
    assert not bad, bad


@pytest.mark.gpu
def test_fuzz_gpu_matches_oracle(golden, fuzz):
    import zkatdlog
    cases, rows = fuzz
    with zkatdlog.Context(golden["pp_a"]["pp"].encode(), device=0) as ctx:
        got = ctx.verify_transfers(rows)
    bad = {c["name"]: (v, c["expect"]) for c, v in zip(cases, got) if v != c["expect"]}
    assert not bad, bad

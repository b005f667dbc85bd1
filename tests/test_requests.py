"""Raw token requests: asn1 TokenRequest decoding, the
action / ledger-token JSON and the request-level verdict order of
Validator.VerifyTokenRequestFromRaw (crypto/validator/validator.go:45-108,
minus the Go-side signature / HTLC / metadata checks).

Fixtures: tests/golden/token_requests.json (tests/golden/make_requests.py, from
the oracle ftsoracle.request over the golden proof corpus).  CPU tier: the
oracle against the fixtures (structure everywhere, real ZK on a sample), the
library's host-side ASN.1 decoder, and the host build of the whole request
path (TEST-ONLY tests/native); GPU tier: ftz_verify_token_requests."""
import base64
import ctypes
import json
import os

import pytest

from ftsoracle import request as R
from ftsoracle import zkat as Z

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def fx():
    with open(os.path.join(HERE, "golden", "token_requests.json")) as f:
        d = json.load(f)
    d["ledger_b"] = {k: base64.b64decode(v) for k, v in d["ledger"].items()}
    for r in d["requests"]:
        r["raw_b"] = base64.b64decode(r["raw"])
    return d


def test_fixture_covers_classes(fx):
    codes = {r["expect"] for r in fx["requests"]}
    assert codes >= {Z.OK, Z.ERR_PARSE, Z.ERR_MALFORMED, Z.ERR_WF, Z.ERR_RANGE, Z.ERR_MEMBERSHIP, Z.ERR_PANIC,
                     R.ERR_INPUT}
    assert len(fx["requests"]) >= 40


def test_oracle_asn1_round_trip(fx):
    """der_encode -> der_token_request is the identity; the library's decoder
    (host code, no GPU) accepts / rejects exactly as the oracle and returns
    the same fields."""
    import zkatdlog
    fields = [[b"a", b""], [b"x" * 200], [], [b"\x00" * 70000]]
    raw = R.der_encode_token_request(fields)
    assert R.der_token_request(raw) == fields
    assert zkatdlog.decode_token_request(raw) == fields
    for r in fx["requests"]:
        try:
            want = R.der_token_request(r["raw_b"])
        except R.Asn1Error:
            want = None
        try:
            got = zkatdlog.decode_token_request(r["raw_b"])
        except ValueError:
            got = None
        assert got == want, r["name"]


def test_oracle_verdicts_real_zk_sample(fx):
    """the oracle with its real ZK verifiers (not the corpus memo the maker
    used) on requests with one cheap action each"""
    pp = Z.PublicParams.from_json(fx["pp"].encode())
    pick = {"issue_anonymous_mismatch", "input_missing", "transfer_action_null_json", "asn1_extra_field_inside_sequence_ignored",
            "issue_nil_output_malformed"}
    seen = 0
    for r in fx["requests"]:
        if r["name"] in pick:
            got = R.verify_token_request(pp, r["raw_b"], fx["ledger_b"].get)
            assert list(got) == [r["expect"], r["failed_action"]], r["name"]
            seen += 1
    assert seen == len(pick)


@pytest.mark.parametrize("batched", [False, True])
@pytest.mark.parametrize("chunk,inflight,threads", [(1, 1, 0), (3, 2, 3), (7, 4, 4), (8192, 4, 2)])
def test_emu_request_pipeline_knobs(emu, fx, batched, chunk, inflight, threads):
    """the pipelined request path (chunks decoded on a thread pool while earlier
    chunks are being verified, lookups one key at a time or one call per chunk)
    gives every fixture verdict and failing index, whatever the chunking; the
    fixture's requests tiled 3x so that chunks straddle request kinds"""
    from zkatdlog import _abi as A
    emu.emu_verify_token_requests_ex.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(A.Bytes),
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                                 ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_int32),
                                                 ctypes.POINTER(ctypes.c_int32)]
    pp = fx["pp"].encode()
    ctx = emu.emu_ctx_create(pp, len(pp), ctypes.create_string_buffer(256), 256)
    rq = fx["requests"] * 3
    try:
        arr, keep = A.pack_bytes([r["raw_b"] for r in rq])
        cb = (A.get_states_callback if batched else A.get_state_callback)(fx["ledger_b"])
        fn = ctypes.cast(cb, ctypes.c_void_p)
        n = len(rq)
        codes = (ctypes.c_int32 * n)()
        failed = (ctypes.c_int32 * n)()
        assert emu.emu_verify_token_requests_ex(ctx, n, arr, None if batched else fn, fn if batched else None, None,
                                                chunk, inflight, threads, codes, failed) == 0
    finally:
        emu.emu_ctx_destroy(ctx)
    assert [(codes[k], failed[k]) for k in range(n)] == [(r["expect"], r["failed_action"]) for r in rq]


def test_emu_request_path_matches_fixture(emu, fx):
    """the product's request orchestration (host/request.cpp) over the host
    build of the job code reproduces every fixture verdict and failing index"""
    from zkatdlog import _abi as A
    emu.emu_verify_token_requests.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(A.Bytes),
                                              A.GET_STATE_FN, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32),
                                              ctypes.POINTER(ctypes.c_int32)]
    pp = fx["pp"].encode()
    ctx = emu.emu_ctx_create(pp, len(pp), ctypes.create_string_buffer(256), 256)
    try:
        reqs = [r["raw_b"] for r in fx["requests"]]
        arr, keep = A.pack_bytes(reqs)
        cb = A.get_state_callback(fx["ledger_b"])
        n = len(reqs)
        codes = (ctypes.c_int32 * n)()
        failed = (ctypes.c_int32 * n)()
        assert emu.emu_verify_token_requests(ctx, n, arr, cb, None, codes, failed) == 0
    finally:
        emu.emu_ctx_destroy(ctx)
    got = {r["name"]: (codes[k], failed[k]) for k, r in enumerate(fx["requests"])}
    want = {r["name"]: (r["expect"], r["failed_action"]) for r in fx["requests"]}
    assert got == want


@pytest.fixture(scope="module")
def gctx(fx):
    import zkatdlog
    c = zkatdlog.Context(fx["pp"].encode(), device=0)
    yield c
    c.close()


def pipeline_chunks(n, ch=4096, ramp=8):
    """chunks of host/request.cpp verify_token_requests: ch/8, ch/4, ch/2, then ch"""
    k, c = 0, max(ch // ramp, 1)
    while n > 0:
        n -= c
        k += 1
        c = min(ch, 2 * c)
    return k


def test_pipeline_chunks():
    assert [pipeline_chunks(n) for n in (0, 1, 512, 513, 3584, 3585, 20043)] == [0, 1, 1, 2, 3, 4, 8]


@pytest.mark.gpu
@pytest.mark.parametrize("batched", [False, True])
def test_gpu_requests_native_ledger_tiled(gctx, fx, batched):
    """ftz_verify_token_requests(_batched) with a native ledger callback over the
    fixture tiled past several 8192-request pipeline chunks: every verdict and
    failing index at its position, and every key looked up on the calling
    thread (one callback per pipeline chunk when batched: 512, 1024, 2048, then
    4096 requests)"""
    import zkatdlog
    rq = fx["requests"] * (20000 // len(fx["requests"]) + 1)
    led = zkatdlog.NativeLedger(fx["ledger_b"])
    try:
        codes, failed = gctx.verify_token_requests([r["raw_b"] for r in rq], led, batched=batched)
        calls, keys = led.counts()
    finally:
        led.close()
    assert list(zip(codes, failed)) == [(r["expect"], r["failed_action"]) for r in rq]
    if batched:
        assert calls <= pipeline_chunks(len(rq))
    else:
        assert calls == keys


@pytest.mark.gpu
def test_gpu_requests_match_fixture(gctx, fx):
    codes, failed = gctx.verify_token_requests([r["raw_b"] for r in fx["requests"]], fx["ledger_b"])
    got = {r["name"]: (codes[k], failed[k]) for k, r in enumerate(fx["requests"])}
    want = {r["name"]: (r["expect"], r["failed_action"]) for r in fx["requests"]}
    assert got == want


@pytest.mark.gpu
def test_gpu_requests_many(gctx, fx):
    """2000 requests (the fixture tiled, ~5 actions per valid request): every
    verdict as expected; prints the request rate end to end (ASN.1 + action
    JSON + ledger callbacks + device batches)."""
    import time
    reqs = fx["requests"] * 44
    t0 = time.perf_counter()
    codes, failed = gctx.verify_token_requests([r["raw_b"] for r in reqs], fx["ledger_b"])
    dt = time.perf_counter() - t0
    assert codes == [r["expect"] for r in reqs]
    assert failed == [r["failed_action"] for r in reqs]
    print("%d token requests in %.3f s: %.0f requests/s" % (len(reqs), dt, len(reqs) / dt), flush=True)


def test_asn1_decoder_mutation_fuzz(fx):
    """2000 seeded byte / length mutations of the fixture requests: the
    library's DER TokenRequest decoder (host code) accepts exactly what the
    oracle restatement of Go encoding/asn1 accepts, with the same fields."""
    import random

    import zkatdlog
    rng = random.Random(20261017)
    raws = [r["raw_b"] for r in fx["requests"] if len(r["raw_b"]) > 4]
    agree = 0
    for k in range(2000):
        b = bytearray(rng.choice(raws))
        mode = k % 4
        if mode == 0:  # flip a byte anywhere
            i = rng.randrange(len(b))
            b[i] ^= rng.randrange(1, 256)
        elif mode == 1:  # perturb a header byte near the front (identifiers, lengths)
            i = rng.randrange(min(len(b), 12))
            b[i] = rng.randrange(256)
        elif mode == 2:  # truncate
            del b[rng.randrange(1, len(b)):]
        else:  # trailing garbage (FromBytes ignores it)
            b += bytes(rng.randrange(256) for _ in range(rng.randrange(1, 8)))
        raw = bytes(b)
        try:
            want = R.der_token_request(raw)
        except R.Asn1Error:
            want = None
        try:
            got = zkatdlog.decode_token_request(raw)
        except ValueError:
            got = None
        assert got == want, (k, mode, raw[:16].hex())
        agree += 1
    assert agree == 2000


def test_bench_request_workload_encoding(fx, emu):
    """zkatdlog.workload.RequestSet (the bench's block-level leg) writes requests
    the oracle decodes as TokenRequest / TransferAction with the intended keys,
    commitments and proofs, and whose verdicts through the product's request
    orchestration (host emulation) are the ones it expects, including the
    missing-input rows"""
    import base64

    from ftsoracle import request as R
    from zkatdlog import _abi as A
    from zkatdlog import workload as W
    g = json.load(open(os.path.join(HERE, "golden", "zkatdlog_golden.json")))["pp_a"]
    good = [c for c in g["cases"] if c["kind"] == "transfer" and c["expect"] == 0 and len(c["inputs"]) == 256
            and len(c["outputs"]) == 256][:2]
    items = [(bytes.fromhex(c["inputs"]), bytes.fromhex(c["outputs"]), base64.b64decode(c["proof"])) for c in good]
    vs = W.TransferSet.from_items(items, [0] * len(items))
    rs = W.RequestSet(vs, 7, per=2, missing_every=3)
    raw0 = bytes(rs.buf[rs.off[0]:rs.off[1]])
    f = R.der_token_request(raw0)
    assert [len(x) for x in f] == [0, 2, 2, 0]
    a = R.decode_transfer_action(f[1][1])
    assert a is not None
    assert json.loads(f[1][1])["Inputs"] == ["blk0000000:1:0", "blk0000000:1:1"]
    assert base64.b64decode(json.loads(f[1][1])["Proof"]) == items[1][2]
    assert list(rs.expect) == [0, 0, 8, 0, 0, 8, 0] and list(rs.failed) == [-1, -1, 1, -1, -1, 1, -1]
    emu.emu_verify_token_requests.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(A.Bytes),
                                              A.GET_STATE_FN, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32),
                                              ctypes.POINTER(ctypes.c_int32)]
    pp = g["pp"].encode()
    ctx = emu.emu_ctx_create(pp, len(pp), ctypes.create_string_buffer(256), 256)
    try:
        cb = A.get_state_callback({k: v for k, v in rs.ledger.items()})
        codes = (ctypes.c_int32 * rs.n)()
        failed = (ctypes.c_int32 * rs.n)()
        assert emu.emu_verify_token_requests(ctx, rs.n, rs.ptr(), cb, None, codes, failed) == 0
    finally:
        emu.emu_ctx_destroy(ctx)
    assert list(codes) == list(rs.expect) and list(failed) == list(rs.failed)

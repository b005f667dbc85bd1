"""Batch prover (include/ftsamd.h ftz_prove_*).

The prover's randomness is rand(tag) = SHA-256(seed||tag||0)||SHA-256(seed||tag||1)
mod r per proof (the oracle's ``Rand``), so its proofs must equal the oracle's
``transfer_prove`` / ``issue_prove`` (tags "tx" / "issue") byte for byte.

CPU tier: the planner + device job code compiled for the host (TEST-ONLY
tests/native) against the oracle.  GPU tier: the same through the C ABI on the
MI355X, plus GPU-verify of a batch of GPU-made proofs."""
import ctypes
import hashlib
import random

import pytest

from ftsoracle import bn254 as C
from ftsoracle import zkat as Z
from zkatdlog import _abi as A


@pytest.fixture(scope="module")
def pp_a(golden):
    js = golden["pp_a"]["pp"].encode()
    return js, Z.PublicParams.from_json(js)


def witness(pp, seed_i, n_in, n_out, ttype="ABC", bound=None):
    rng = random.Random(seed_i)
    top = bound or pp.base ** pp.exponent
    ins_v = [rng.randrange(top) for _ in range(n_in)]
    outs_v = list(ins_v) if n_in == n_out else [rng.randrange(top) for _ in range(n_out)]
    in_bf = [rng.randrange(C.R) for _ in range(n_in)]
    out_bf = [rng.randrange(C.R) for _ in range(n_out)]
    ins = [Z.token_commitment(pp, ttype, v, b) for v, b in zip(ins_v, in_bf)]
    outs = [Z.token_commitment(pp, ttype, v, b) for v, b in zip(outs_v, out_bf)]
    seed = hashlib.sha256(b"prover-seed-%d" % seed_i).digest()
    return {"inputs": b"".join(C.g1_bytes(p) for p in ins), "outputs": b"".join(C.g1_bytes(p) for p in outs),
            "in_values": ins_v, "in_bfs": in_bf, "out_values": outs_v, "out_bfs": out_bf, "type": ttype,
            "seed": seed, "_ins": ins, "_outs": outs}


def oracle_transfer(pp, w):
    return Z.transfer_prove(pp, Z.Rand(w["seed"]), w["_ins"], w["_outs"],
                            list(zip(w["in_values"], w["in_bfs"])), list(zip(w["out_values"], w["out_bfs"])),
                            w["type"], tag="tx")


def issue_witness(pp, seed_i, n, ttype="ABC", anonymous=False):
    w = witness(pp, seed_i, 0, n, ttype)
    return {"outputs": w["outputs"], "values": w["out_values"], "bfs": w["out_bfs"], "type": ttype,
            "anonymous": anonymous, "seed": w["seed"], "_outs": w["_outs"]}


def oracle_issue(pp, w):
    return Z.issue_prove(pp, Z.Rand(w["seed"]), w["_outs"], list(zip(w["values"], w["bfs"])), w["type"],
                         anonymous=w["anonymous"], tag="issue")


def emu_prove(emu, pp_json, ws, issue=False):
    ctx = emu.emu_ctx_create(pp_json, len(pp_json), ctypes.create_string_buffer(256), 256)
    assert ctx
    try:
        arr, keep = (A.pack_issue_witnesses if issue else A.pack_transfer_witnesses)(ws)
        fn = emu.emu_prove_issues if issue else emu.emu_prove_transfers
        fn.restype = ctypes.c_long
        fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t,
                       ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p,
                       ctypes.c_size_t]
        cap = 1 << 22
        buf = ctypes.create_string_buffer(cap)
        offs = (ctypes.c_size_t * (len(ws) + 1))()
        codes = (ctypes.c_int32 * max(1, len(ws)))()
        err = ctypes.create_string_buffer(512)
        r = fn(ctx, len(ws), arr, buf, cap, offs, codes, err, 512)
        if r < 0:
            raise ValueError(err.value.decode())
        return [buf.raw[offs[i]:offs[i + 1]] for i in range(len(ws))], list(codes)[:len(ws)]
    finally:
        emu.emu_ctx_destroy(ctx)


@pytest.mark.parametrize("n_in,n_out", [(2, 2), (1, 1), (1, 2), (3, 1)])
def test_emu_transfer_proofs_match_oracle(emu, pp_a, n_in, n_out):
    js, pp = pp_a
    ws = [witness(pp, 10 * n_in + n_out, n_in, n_out)]
    if n_in != n_out:  # keep the sum balanced: outputs split the inputs' value
        v = sum(ws[0]["in_values"]) % (pp.base ** pp.exponent)
        ws[0]["out_values"] = [v // 3, v - v // 3][:n_out] if n_out == 2 else [v]
        ws[0]["_outs"] = [Z.token_commitment(pp, "ABC", a, b) for a, b in zip(ws[0]["out_values"], ws[0]["out_bfs"])]
        ws[0]["outputs"] = b"".join(C.g1_bytes(p) for p in ws[0]["_outs"])
    got, codes = emu_prove(emu, js, ws)
    assert codes == [0]
    want = oracle_transfer(pp, ws[0])
    assert got[0] == want
    # and the oracle verifier accepts it
    assert Z.transfer_verify(pp, ws[0]["_ins"], ws[0]["_outs"], got[0])[1] == Z.OK


@pytest.mark.parametrize("anonymous", [False, True])
def test_emu_issue_proofs_match_oracle(emu, pp_a, anonymous):
    js, pp = pp_a
    w = issue_witness(pp, 77 + anonymous, 2, ttype="tok<&>\"x\"", anonymous=anonymous)
    got, codes = emu_prove(emu, js, [w], issue=True)
    assert codes == [0]
    assert got[0] == oracle_issue(pp, w)


def test_emu_shape_templates_mixed_batch(emu, pp_a):
    """One planning call over interleaved shapes (the planner plans each shape
    once and appends the relocated template per proof, patching in the witness
    bytes): every proof -- different values, hence different digits, signature
    points and digit hashes per proof -- byte-identical to the oracle's; issues
    with two TypeInTheClear strings keep their own templates."""
    js, pp = pp_a
    shapes = [(2, 2), (1, 1), (2, 2), (1, 2), (2, 2), (1, 1)]
    ws = []
    for i, (ni, no) in enumerate(shapes):
        w = witness(pp, 900 + i, ni, no)
        if ni != no:
            v = sum(w["in_values"]) % (pp.base ** pp.exponent)
            w["out_values"] = [v // 3, v - v // 3]
            w["_outs"] = [Z.token_commitment(pp, "ABC", a, b) for a, b in zip(w["out_values"], w["out_bfs"])]
            w["outputs"] = b"".join(C.g1_bytes(p) for p in w["_outs"])
        ws.append(w)
    got, codes = emu_prove(emu, js, ws)
    assert codes == [0] * len(ws)
    for g, w in zip(got, ws):
        assert g == oracle_transfer(pp, w)
    iw = [issue_witness(pp, 950 + i, 2, ttype=t, anonymous=a)
          for i, (t, a) in enumerate([("ABC", False), ("XY", False), ("ABC", False), ("Q", True)])]
    got, codes = emu_prove(emu, js, iw, issue=True)
    assert codes == [0] * len(iw)
    for g, w in zip(got, iw):
        assert g == oracle_issue(pp, w)


def test_emu_value_out_of_range(emu, pp_a):
    js, pp = pp_a
    w = witness(pp, 5, 2, 2)
    w["out_values"] = [pp.base ** pp.exponent, 0]
    with pytest.raises(ValueError, match="outside authorized range"):
        emu_prove(emu, js, [w])


def test_emu_bad_commitment_code(emu, pp_a):
    js, pp = pp_a
    w = witness(pp, 6, 1, 1)
    bad = bytearray(w["inputs"])
    bad[63] ^= 1
    w["inputs"] = bytes(bad)
    _, codes = emu_prove(emu, js, [w])
    assert codes == [A.FTZ_ERR_PARSE]


# ---------------------------------------------------------------- GPU tier
@pytest.fixture(scope="module")
def gctx(golden):
    import zkatdlog
    c = zkatdlog.Context(golden["pp_a"]["pp"].encode(), device=0)
    yield c
    c.close()


@pytest.mark.gpu
def test_gpu_transfer_proofs_match_oracle(gctx, pp_a):
    _, pp = pp_a
    ws = [witness(pp, 300 + i, 2, 2) for i in range(3)] + [witness(pp, 310, 1, 1)]
    proofs, codes = gctx.prove_transfers(ws)
    assert codes == [0] * len(ws)
    for w, p in zip(ws, proofs):
        assert p == oracle_transfer(pp, w)


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["one_lane", "sextet"])
def test_gpu_proofs_match_oracle_every_layout(golden, pp_a, layout):
    """the prover's t / pair-2 line stage in either kernel layout
    (ftz_ctx_set_layout) gives byte-identical proofs"""
    import zkatdlog
    _, pp = pp_a
    ws = [witness(pp, 320 + i, 2, 2) for i in range(2)]
    with zkatdlog.Context(golden["pp_a"]["pp"].encode(), device=0) as c:
        c.set_layout("prover_g2lines", layout)
        proofs, codes = c.prove_transfers(ws)
    assert codes == [0, 0]
    for w, p in zip(ws, proofs):
        assert p == oracle_transfer(pp, w)


@pytest.mark.gpu
def test_gpu_proofs_without_prover_tables_match_oracle(golden, pp_a):
    """ftz_options.prover_tables = 0 (the fallback a context takes
    when the digit-signature table set cannot be allocated): the variable-base
    R_d / S_d path with G2 jobs gives the same bytes as the oracle, for
    transfers and issues"""
    import zkatdlog
    _, pp = pp_a
    ws = [witness(pp, 330 + i, 2, 2) for i in range(2)]
    iw = [issue_witness(pp, 430, 2)]
    with zkatdlog.Context(golden["pp_a"]["pp"].encode(), device=0, prover_tables=0) as c:
        assert c.options["prover_tables"] == 0
        proofs, codes = c.prove_transfers(ws)
        iproofs, icodes = c.prove_issues(iw)
    assert codes == [0, 0] and icodes == [0]
    for w, p in zip(ws, proofs):
        assert p == oracle_transfer(pp, w)
    assert iproofs[0] == oracle_issue(pp, iw[0])


@pytest.mark.gpu
def test_gpu_issue_proofs_match_oracle(gctx, pp_a):
    _, pp = pp_a
    ws = [issue_witness(pp, 400, 2), issue_witness(pp, 401, 1, ttype="USD", anonymous=True)]
    proofs, codes = gctx.prove_issues(ws)
    assert codes == [0, 0]
    for w, p in zip(ws, proofs):
        assert p == oracle_issue(pp, w)


@pytest.mark.gpu
def test_gpu_prove_then_verify_batch(gctx, pp_a):
    """A batch of GPU-made proofs is accepted by the GPU verifier; a proof
    checked against swapped outputs is rejected."""
    _, pp = pp_a
    base = [witness(pp, 500 + i, 2, 2) for i in range(8)]
    ws = [base[i % 8] | {"seed": hashlib.sha256(b"b%d" % i).digest()} for i in range(256)]
    proofs, codes = gctx.prove_transfers(ws)
    assert codes == [0] * len(ws)
    assert len(set(proofs)) == len(proofs)  # fresh randomness per proof
    tx = [(w["inputs"], w["outputs"], p) for w, p in zip(ws, proofs)]
    tx.append((ws[0]["inputs"], ws[1]["outputs"], proofs[0]))
    got = gctx.verify_transfers(tx)
    assert list(got[:-1]) == [0] * len(ws) and got[-1] != 0


@pytest.mark.gpu
def test_gpu_prover_rejects_out_of_range(gctx, pp_a):
    import zkatdlog
    _, pp = pp_a
    w = witness(pp, 7, 2, 2)
    w["out_values"] = [pp.base ** pp.exponent + 1, 0]
    with pytest.raises(zkatdlog.DeviceError, match="outside authorized range"):
        gctx.prove_transfers([w])


@pytest.mark.gpu
def test_gpu_prove_verify_pp_b(golden):
    """PP-B (b=16, e=16: 16 membership proofs per output): GPU proofs accepted
    by the GPU verifier, and tampering with one output rejects."""
    import zkatdlog
    if "pp_b" not in golden:
        pytest.skip("no PP-B fixtures")
    js = golden["pp_b"]["pp"].encode()
    pp = Z.PublicParams.from_json(js)
    ws = [witness(pp, 600 + i, 2, 2, bound=1 << 40) for i in range(4)]
    with zkatdlog.Context(js, device=0) as c:
        proofs, codes = c.prove_transfers(ws)
        assert codes == [0] * 4
        tx = [(w["inputs"], w["outputs"], p) for w, p in zip(ws, proofs)]
        tx.append((ws[0]["inputs"], ws[1]["outputs"], proofs[0]))
        assert list(c.verify_transfers(tx)) == [0, 0, 0, 0, A.FTZ_ERR_WF]


# ------------------------------------------- PP-B (64-bit values) vs the oracle
# tests/golden/ppb_prover_cases.json (make_ppb_prover.py): oracle proofs under
# the seeded Rand for values at the edges of the 64-bit range -- 0, 1, 15,
# 2^63 - 1, 2^63, 2^64 - 2, 2^64 - 1 and a split summing to 2^64 - 1 -- each
# accepted by the oracle verifier when the fixture was made.  This is where the
# reference's float64 digit code (range/proof.go:303-310) stops being exact and
# the library's integer decomposition takes over; the prover must reproduce the
# oracle byte for byte.
PPB_FIXTURE = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "ppb_prover_cases.json")


@pytest.fixture(scope="module")
def ppb_cases(golden):
    import json
    with open(PPB_FIXTURE) as f:
        cases = json.load(f)["cases"]
    js = golden["pp_b"]["pp"].encode()
    return js, Z.PublicParams.from_json(js), cases


def ppb_witness(c):
    import base64
    ints = lambda xs: [int(x) for x in xs]  # noqa: E731
    if c["kind"] == "transfer":
        w = {"inputs": bytes.fromhex(c["inputs"]), "outputs": bytes.fromhex(c["outputs"]),
             "in_values": ints(c["in_values"]), "in_bfs": ints(c["in_bfs"]),
             "out_values": ints(c["out_values"]), "out_bfs": ints(c["out_bfs"])}
    else:
        w = {"outputs": bytes.fromhex(c["outputs"]), "values": ints(c["values"]), "bfs": ints(c["bfs"]),
             "anonymous": c["anonymous"]}
    w.update(type=c["type"], seed=bytes.fromhex(c["seed"]))
    return w, base64.b64decode(c["proof"])


def test_ppb_fixture_covers_the_64bit_edges(ppb_cases):
    _, _, cases = ppb_cases
    vals = set()
    for c in cases:
        assert c["oracle_verdict"] == Z.OK
        vals.update(int(v) for v in c.get("out_values", c.get("values", [])))
    assert {0, 1, 15, (1 << 63) - 1, 1 << 63, (1 << 64) - 2, (1 << 64) - 1} <= vals
    split = [c for c in cases if c["name"] == "split_to_max"][0]
    assert sum(int(v) for v in split["in_values"]) == (1 << 64) - 1


def test_ppb_oracle_accepts_max_value_proof(ppb_cases):
    """the oracle verifier re-run on one fixture proof (values 2^64 - 1 and 0)"""
    _, pp, cases = ppb_cases
    c = [c for c in cases if c["name"] == "max_zero"][0]
    w, proof = ppb_witness(c)
    ins = [C.g1_from_bytes(w["inputs"][i:i + 64]) for i in range(0, len(w["inputs"]), 64)]
    outs = [C.g1_from_bytes(w["outputs"][i:i + 64]) for i in range(0, len(w["outputs"]), 64)]
    assert Z.transfer_verify(pp, ins, outs, proof)[1] == Z.OK


def test_emu_ppb_proofs_match_oracle(emu, ppb_cases):
    js, _, cases = ppb_cases
    tw = [ppb_witness(c) for c in cases if c["kind"] == "transfer"]
    got, codes = emu_prove(emu, js, [w for w, _ in tw])
    assert codes == [0] * len(tw)
    assert got == [p for _, p in tw]
    iw = [ppb_witness(c) for c in cases if c["kind"] == "issue"]
    got, codes = emu_prove(emu, js, [w for w, _ in iw], issue=True)
    assert codes == [0] * len(iw)
    assert got == [p for _, p in iw]


@pytest.mark.gpu
def test_gpu_ppb_proofs_match_oracle(ppb_cases):
    """GPU PP-B transfer and issue proofs byte-identical to the oracle's at the
    64-bit edges, and accepted by the GPU verifier"""
    import zkatdlog
    js, _, cases = ppb_cases
    tw = [ppb_witness(c) for c in cases if c["kind"] == "transfer"]
    iw = [ppb_witness(c) for c in cases if c["kind"] == "issue"]
    with zkatdlog.Context(js, device=0) as c:
        proofs, codes = c.prove_transfers([w for w, _ in tw])
        assert codes == [0] * len(tw)
        assert proofs == [p for _, p in tw]
        iproofs, icodes = c.prove_issues([w for w, _ in iw])
        assert icodes == [0] * len(iw)
        assert iproofs == [p for _, p in iw]
        got = c.verify_transfers([(w["inputs"], w["outputs"], p) for (w, _), p in zip(tw, proofs)])
        assert list(got) == [0] * len(tw)
        got = c.verify_issues([(w["outputs"], p, w["anonymous"]) for (w, _), p in zip(iw, iproofs)])
        assert list(got) == [0] * len(iw)

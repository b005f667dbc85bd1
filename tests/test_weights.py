"""Range-proof digit weights as the reference computes them.

The reference weighs digit i by int64(math.Pow(float64(Base), float64(i)))
(range/proof.go:428; the prover's decomposition and blinding factor use the
same expression, :303-311, :327).  Go's math.Pow (src/math/pow.go, go1.18 per
go.mod:3) is exact only while Base^i is a float64, and int64() of a float64 at
or above 2^63 is -2^63 on amd64.  The oracle restates both (zkat.go_pow /
go_int64), the product too (host/planner.cpp go_pow_int / go_int64), and
tests/golden/ppc_golden.json (make_ppc.py) holds PP-C (b = 7, e = 22: four
inexact weights) and PP-D (b = 1000, e = 8: w_7 = -2^63) proofs with the
oracle's verdicts under the reference's weights and under exact ones.

CPU tier: the weights and the prover's digits of the product's planner
(through the TEST-ONLY emulation library) against the oracle; every PP-C/PP-D
verdict and prover byte through the host build of the device code.  GPU tier:
the same verdicts through the C ABI, tiled past the small-pass size, and the
GPU prover's PP-C proofs byte for byte."""
import base64
import ctypes
import json
import os
import random

import pytest

from conftest import case_tuple
from ftsoracle import zkat as Z
from zkatdlog import _abi as A

FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "ppc_golden.json")
INT64_MIN = -(1 << 63)


@pytest.fixture(scope="module")
def ppc():
    with open(FIXTURE) as f:
        return json.load(f)


def _emu_fns(emu):
    emu.emu_digit_weight.restype = ctypes.c_int64
    emu.emu_digit_weight.argtypes = [ctypes.c_uint32, ctypes.c_int64]
    emu.emu_prover_digits.restype = ctypes.c_int
    emu.emu_prover_digits.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                      ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int64)]
    return emu


# ------------------------------------------------------------------ the weights
def test_go_pow_inexact_and_overflowing_weights():
    """Go's repeated-squaring Pow is not the correctly rounded power: 13^17
    comes out 1203 above it (the nearest float64 is 179 above), 7^21 25 above;
    at or above 2^63 the int64 conversion gives -2^63."""
    w = Z.digit_weight
    assert [w(7, i) - 7 ** i for i in (18, 19, 20, 21, 22)] == [0, 1, -1, 25, 239]
    assert w(13, 17) - 13 ** 17 == 1203 and int(float(13 ** 17)) - 13 ** 17 == 179
    assert w(3, 38) - 3 ** 38 == -89
    assert w(100, 2) == 10000 and w(16, 15) == 1 << 60
    assert w(16, 16) == INT64_MIN and w(2, 63) == INT64_MIN and w(1000, 7) == INT64_MIN
    assert w(2, 62) == 1 << 62 and w(10, 18) == 10 ** 18 and w(10, 19) == INT64_MIN
    assert w(7, 0) == 1 and w(7, 1) == 7 and w(5, 10 ** 6) == INT64_MIN  # Ldexp overflow -> +Inf
    # exact while base^i < 2^53
    rng = random.Random(3)
    for _ in range(2000):
        b = rng.randrange(2, 5000)
        i = rng.randrange(0, 60)
        if b ** i < 1 << 53:
            assert w(b, i) == b ** i


def test_product_weights_match_oracle(emu):
    e = _emu_fns(emu)
    rng = random.Random(5)
    pairs = [(b, i) for b in (2, 3, 7, 10, 11, 13, 16, 100, 255, 1000, 65535) for i in range(0, 70)]
    pairs += [(rng.randrange(2, 1 << 20), rng.randrange(0, 80)) for _ in range(3000)]
    pairs += [(3, 10 ** 6), (2, 1 << 40)]
    bad = [(b, i) for b, i in pairs if e.emu_digit_weight(b, i) != Z.digit_weight(b, i)]
    assert not bad, bad[:10]


def test_fixture_weights_are_the_oracles(ppc):
    for key in ("pp_c", "pp_d"):
        s = ppc[key]
        assert [int(x) for x in s["weights"]] == [Z.digit_weight(s["base"], i) for i in range(s["exponent"] + 1)]
    assert int(ppc["pp_c"]["weights"][21]) == 7 ** 21 + 25
    assert int(ppc["pp_d"]["weights"][7]) == INT64_MIN


def test_product_prover_digits_match_oracle(emu, ppc):
    """preProcess's decomposition (range/proof.go:297-311): quotient and
    remainder by the Go weights, values[0] = v % b of the original v; refusals
    and the digit >= b panic included"""
    e = _emu_fns(emu)
    rng = random.Random(9)
    for key, b, n in (("pp_c", 7, 22), ("pp_d", 1000, 8)):
        js = ppc[key]["pp"].encode()
        top = Z.digit_weight(b, n)
        vals = [0, 1, b - 1, b, b ** 18 + 3, (1 << 63) - 1, 1 << 63, (1 << 64) - 1, 1 << 70]
        vals += [top - 1, top, top + 1] if top > 0 else []
        vals += [rng.randrange(b ** 19 if b == 7 else 1, 7 ** 22) for _ in range(400)]
        vals += [int(r["value"]) for r in ppc["prover_refusals"] if r["pp"] == key[-1].upper()]
        for v in vals:
            d = (ctypes.c_uint32 * n)()
            w = (ctypes.c_int64 * (n + 1))()
            r = e.emu_prover_digits(js, len(js), (v % (1 << 256)).to_bytes(32, "big"), d, w)
            assert list(w) == [Z.digit_weight(b, i) for i in range(n + 1)]
            try:
                want, code = Z.digits(v, b, n), 0
            except Z.Panic:
                want, code = None, 2
            except ValueError:
                want, code = None, 1
            assert r == code, (key, v)
            if code == 0:
                assert list(d) == want, (key, v)


# ------------------------------------------------------------------ fixture shape
def test_fixture_shows_the_weights_change_verdicts(ppc):
    """The reference's weights accept proofs exact weights reject, and the
    reverse (a proof made with exact weights), and its own prover's proof can
    be rejected by its own verifier (inconsistent float64 digits)."""
    by = {c["name"]: c for c in ppc["cases"]}
    hi = by["ppc_high_digits_go_weights"]
    assert hi["expect"] == Z.OK and hi["expect_exact_weights"] == Z.ERR_RANGE
    ex = by["ppc_crafted_exact_digits"]
    assert ex["expect"] == Z.ERR_RANGE and ex["expect_exact_weights"] == Z.OK
    assert by["ppc_reference_prover_inconsistent_digits"]["expect"] == Z.ERR_RANGE
    # the blinding factor weighs every digit: exact weights reject even all-low-digit proofs
    assert by["ppc_low_values"]["expect"] == Z.OK and by["ppc_low_values"]["expect_exact_weights"] == Z.ERR_RANGE
    neg = by["ppd_weight_minus_2_63"]
    assert neg["expect"] == Z.OK and neg["expect_exact_weights"] == Z.ERR_RANGE
    assert by["ppc_issue_high_digits"]["expect"] == Z.OK
    assert {c["expect"] for c in ppc["cases"]} >= {Z.OK, Z.ERR_RANGE, Z.ERR_MEMBERSHIP}
    outcomes = {r["outcome"] for r in ppc["prover_refusals"]}
    assert outcomes == {"refused", "panic", "proves"}


# ------------------------------------------------------------------ CPU tier (host build)
def _emu_run(emu, pp_json, cases):
    err = ctypes.create_string_buffer(256)
    ctx = emu.emu_ctx_create(pp_json, len(pp_json), err, 256)
    assert ctx, err.value
    try:
        got = {}
        for kind, pack, fn in (("transfer", A.pack_transfers, emu.emu_verify_transfers),
                               ("issue", A.pack_issues, emu.emu_verify_issues)):
            cs = [c for c in cases if c["kind"] == kind]
            if cs:
                arr, keep = pack([case_tuple(c) for c in cs])
                codes = (ctypes.c_int32 * len(cs))()
                fn(ctx, len(cs), arr, codes)
                got.update({c["name"]: v for c, v in zip(cs, codes)})
        return got
    finally:
        emu.emu_ctx_destroy(ctx)


@pytest.mark.parametrize("key", ["pp_c", "pp_d"])
def test_emu_verdicts(emu, ppc, key):
    cases = [c for c in ppc["cases"] if c["pp"] == key[-1].upper()]
    got = _emu_run(emu, ppc[key]["pp"].encode(), cases)
    assert got == {c["name"]: c["expect"] for c in cases}


def prover_witness(c):
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


def _prover_cases(ppc, kind):
    return [prover_witness(c) for c in ppc["cases"] if c["pp"] == "C" and not c["crafted"] and c["kind"] == kind]


def _refusal_witness(v):
    from ftsoracle import bn254 as C
    g = C.g1_bytes(C.G1_GEN)  # the commitments' bytes do not matter to the value checks
    return {"inputs": g * 2, "outputs": g * 2, "in_values": [v, 5], "in_bfs": [1, 2],
            "out_values": [5, v], "out_bfs": [3, 4], "type": "PPC", "seed": bytes(32)}


def test_emu_prover_matches_oracle(emu, ppc):
    from test_prover import emu_prove
    js = ppc["pp_c"]["pp"].encode()
    tw = _prover_cases(ppc, "transfer")
    got, codes = emu_prove(emu, js, [w for w, _ in tw])
    assert codes == [0] * len(tw) and got == [p for _, p in tw]
    iw = _prover_cases(ppc, "issue")
    got, codes = emu_prove(emu, js, [w for w, _ in iw], issue=True)
    assert codes == [0] * len(iw) and got == [p for _, p in iw]


def test_emu_prover_refusals(emu, ppc):
    from test_prover import emu_prove
    for r in ppc["prover_refusals"]:
        js = ppc["pp_" + r["pp"].lower()]["pp"].encode()
        w = _refusal_witness(int(r["value"]))
        if r["outcome"] == "proves":
            _, codes = emu_prove(emu, js, [w])
            assert codes == [0]
            continue
        msg = "outside authorized range" if r["outcome"] == "refused" else "digit index out of range"
        with pytest.raises(ValueError, match=msg):
            emu_prove(emu, js, [w])


# ------------------------------------------------------------------ GPU tier
@pytest.mark.gpu
@pytest.mark.parametrize("key", ["pp_c", "pp_d"])
def test_gpu_verdicts(ppc, key):
    """Every PP-C/PP-D verdict through the C ABI, once alone and once tiled into
    a pass above the small-pass size (the batch path's layouts)."""
    import zkatdlog
    cases = [c for c in ppc["cases"] if c["pp"] == key[-1].upper()]
    tr = [c for c in cases if c["kind"] == "transfer"]
    iss = [c for c in cases if c["kind"] == "issue"]
    with zkatdlog.Context(ppc[key]["pp"].encode(), device=0) as c:
        assert list(c.verify_transfers([case_tuple(x) for x in tr])) == [x["expect"] for x in tr]
        if iss:
            assert list(c.verify_issues([case_tuple(x) for x in iss])) == [x["expect"] for x in iss]
        reps = -(-4200 // (22 * 2 * len(tr)))  # pairing jobs past small_pass (4096)
        tiled = [case_tuple(tr[i % len(tr)]) for i in range(len(tr) * reps)]
        got = list(c.verify_transfers(tiled))
        assert got == [tr[i % len(tr)]["expect"] for i in range(len(tiled))]


@pytest.mark.gpu
def test_gpu_prover_matches_oracle(ppc):
    import zkatdlog
    js = ppc["pp_c"]["pp"].encode()
    tw, iw = _prover_cases(ppc, "transfer"), _prover_cases(ppc, "issue")
    with zkatdlog.Context(js, device=0) as c:
        proofs, codes = c.prove_transfers([w for w, _ in tw])
        assert codes == [0] * len(tw) and proofs == [p for _, p in tw]
        iproofs, icodes = c.prove_issues([w for w, _ in iw])
        assert icodes == [0] * len(iw) and iproofs == [p for _, p in iw]
        for r in ppc["prover_refusals"]:
            if r["pp"] != "C" or r["outcome"] == "proves":
                continue
            msg = "outside authorized range" if r["outcome"] == "refused" else "digit index out of range"
            with pytest.raises(zkatdlog.DeviceError, match=msg):
                c.prove_transfers([_refusal_witness(int(r["value"]))])

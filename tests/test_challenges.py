"""Device parity beyond the verdict class: the recomputed Fiat-Shamir
challenges of every golden case, tampered ones included.

The oracle records every challenge its verifier recomputes (the HashToZr of
each well-formedness, membership and range transcript; zkat.CHALLENGE_TRACE)
in tests/golden/challenge_traces.json (make_traces.py).  The library keeps the
same values when a context is in debug mode (ftz_ctx_set_debug
FTZ_DEBUG_CHALLENGES) and returns them per proof (ftz_batch_challenges).  The
membership transcript holds the recomputed GT bytes (sigproof/pok.go:199-203,
membership.go:260-277), so equal challenges mean equal pairing values too.

Comparison per class (WF / membership / range): the oracle's values are a
prefix of the device's.  The device may hold more -- it plans every transcript
of a proof it can parse, while the oracle stops at the first error the
reference would return -- or none of a class, when the planner found the
structural failure before planning those transcripts (the oracle may still
hash the other digits of a range proof one of whose digits is malformed).
Accepted proofs must match in full.

CPU tier: the host build of the planner and device code (tests/native) on
every case; GPU tier: the same through the C ABI on the MI355X."""
import ctypes
import json
import os

import pytest

from conftest import case_tuple
from ftsoracle import zkat as Z
from zkatdlog import _abi as A

HERE = os.path.dirname(__file__)
SETS = ["pp_a", "pp_b", "pp_c", "pp_d"]


@pytest.fixture(scope="module")
def traces():
    with open(os.path.join(HERE, "golden", "challenge_traces.json")) as f:
        return json.load(f)["traces"]


@pytest.fixture(scope="module")
def corpus(golden):
    with open(os.path.join(HERE, "golden", "ppc_golden.json")) as f:
        pc = json.load(f)
    out = {k: (golden[k]["pp"].encode(), golden[k]["cases"]) for k in ("pp_a", "pp_b")}
    for k in ("pp_c", "pp_d"):
        out[k] = (pc[k]["pp"].encode(), [c for c in pc["cases"] if c["pp"] == k[-1].upper()])
    return out


def compare(name, expect, dev, ora):
    """dev / ora: [(class, 32-byte value)]; returns the number of values compared"""
    n = 0
    for kind in (Z.ERR_WF, Z.ERR_MEMBERSHIP, Z.ERR_RANGE):
        d = [v for k, v in dev if k == kind]
        o = [v for k, v in ora if k == kind]
        if expect == Z.OK:
            assert d == o, (name, kind)
        if d:
            assert d[:len(o)] == o, (name, kind, len(d), len(o))
            n += len(o)
    return n


def oracle_list(t):
    return [(k, bytes.fromhex(h)) for k, h in t["challenges"]]


def test_fixture_covers_every_case_and_class(traces, corpus):
    for key in SETS:
        names = {c["name"] for c in corpus[key][1]}
        assert set(traces[key]) == names, key
    kinds = {k for key in SETS for t in traces[key].values() for k, _ in t["challenges"]}
    assert kinds == {Z.ERR_WF, Z.ERR_MEMBERSHIP, Z.ERR_RANGE}
    # tampered proofs carry challenges too (the point of the check)
    rejected = [t for key in SETS for t in traces[key].values() if t["expect"] != Z.OK and t["challenges"]]
    assert len(rejected) >= 85


def test_oracle_trace_spot_check(traces, corpus):
    """re-derive two PP-A traces with the oracle (the fixture is the oracle's)"""
    from ftsoracle import bn254 as C
    pp_json, cases = corpus["pp_a"]
    pp = Z.PublicParams.from_json(pp_json)
    by = {c["name"]: c for c in cases}
    for name in ("valid_2in_2out", "membership_value"):
        c = by[name]
        ins, outs, proof = case_tuple(c)
        dec = lambda b: [C.g1_from_bytes(b[i:i + 64]) for i in range(0, len(b), 64)]  # noqa: E731
        Z.CHALLENGE_TRACE = []
        try:
            Z.transfer_verify(pp, dec(ins), dec(outs), proof)
            got = [[k, "%064x" % h] for k, h in Z.CHALLENGE_TRACE]
        finally:
            Z.CHALLENGE_TRACE = None
        assert got == traces["pp_a"][name]["challenges"]


def _emu_lib(emu):
    emu.emu_challenges.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p,
                                   ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p,
                                   ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
    return emu


@pytest.mark.parametrize("key", SETS)
def test_emu_challenges_match_oracle(emu, traces, corpus, key):
    lib = _emu_lib(emu)
    pp_json, cases = corpus[key]
    ctx = lib.emu_ctx_create(pp_json, len(pp_json), ctypes.create_string_buffer(256), 256)
    assert ctx
    compared = 0
    cap = 128
    try:
        for kind, pack in ((0, A.pack_transfers), (1, A.pack_issues)):
            cs = [c for c in cases if c["kind"] == ("transfer" if kind == 0 else "issue")]
            if not cs:
                continue
            arr, keep = pack([case_tuple(c) for c in cs])
            n = len(cs)
            codes = (ctypes.c_int32 * n)()
            kinds = (ctypes.c_int32 * (n * cap))()
            vals = ctypes.create_string_buffer(32 * n * cap)
            counts = (ctypes.c_size_t * n)()
            lib.emu_challenges(ctx, kind, n, ctypes.cast(arr, ctypes.c_void_p), codes, kinds, vals, cap, counts)
            for i, c in enumerate(cs):
                assert codes[i] == c["expect"], c["name"]
                assert counts[i] <= cap
                dev = [(kinds[i * cap + k], vals.raw[32 * (i * cap + k):32 * (i * cap + k + 1)])
                       for k in range(counts[i])]
                compared += compare(c["name"], c["expect"], dev, oracle_list(traces[key][c["name"]]))
    finally:
        lib.emu_ctx_destroy(ctx)
    assert compared > 0


# ------------------------------------------------------------------ GPU tier
@pytest.mark.gpu
@pytest.mark.parametrize("key", SETS)
def test_gpu_challenges_match_oracle(traces, corpus, key):
    """every golden case of the set in one debug batch per kind; the recomputed
    WF, membership and range challenges against the oracle's"""
    import zkatdlog
    pp_json, cases = corpus[key]
    compared = 0
    with zkatdlog.Context(pp_json, device=0) as ctx:
        ctx.set_debug(challenges=True)
        for kind in ("transfer", "issue"):
            cs = [c for c in cases if c["kind"] == kind]
            if not cs:
                continue
            b = (ctx.load_transfers if kind == "transfer" else ctx.load_issues)([case_tuple(c) for c in cs])
            try:
                b.run()
                codes = list(b.codes())
                for i, c in enumerate(cs):
                    assert codes[i] == c["expect"], c["name"]
                    compared += compare(c["name"], c["expect"], b.challenges(i),
                                        oracle_list(traces[key][c["name"]]))
            finally:
                b.close()
    assert compared > 0


# ------------------------------------------------- t' at infinity in shared trees
@pytest.fixture(scope="module")
def zero_norm():
    with open(os.path.join(HERE, "golden", "zero_norm_cases.json")) as f:
        return json.load(f)["cases"]


def test_zero_norm_fixture(zero_norm):
    """membership proofs with Challenge = Value = Hash = 0 (t' = O): the oracle
    still hashes their transcripts (the infinity pair contributes 1) and
    rejects on the challenge; the unmodified base proof is accepted"""
    by = {c["name"]: c for c in zero_norm}
    assert by["valid_2in_2out"]["expect"] == Z.OK
    for name in ("t_prime_infinity_digit_0_0", "t_prime_infinity_digit_1_1", "t_prime_infinity_every_digit"):
        assert by[name]["expect"] == Z.ERR_MEMBERSHIP
        assert sum(1 for k, _ in by[name]["challenges"] if k == Z.ERR_MEMBERSHIP) == 4


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["dense", "sparse"])
def test_gpu_zero_norm_shares_inversion_trees(golden, zero_norm, layout):
    """t' = O proofs tiled into a 4096-transfer pass (above small_pass: the
    one-lane line stage with its 256-job k_g2_binv trees, and k_fexp_binv):
    dense -- every fourth transfer, so every tree holds zero norms --, or
    sparse -- two among valid ones.  Every verdict and every recomputed
    challenge of the zero-norm proofs and their neighbours must be the
    oracle's; the engine path (default options) gives the same verdicts."""
    import zkatdlog
    n = 4096
    valid = next(i for i, c in enumerate(zero_norm) if c["name"] == "valid_2in_2out")
    if layout == "dense":
        sel = [k % len(zero_norm) for k in range(n)]
    else:
        sel = [valid] * n
        sel[1000] = next(i for i, c in enumerate(zero_norm) if c["name"] == "t_prime_infinity_digit_0_0")
        sel[3001] = next(i for i, c in enumerate(zero_norm) if c["name"] == "t_prime_infinity_every_digit")
    want = [zero_norm[k]["expect"] for k in sel]
    with zkatdlog.Context(golden["pp_a"]["pp"].encode(), device=0) as ctx:
        assert ctx.options["small_pass"] <= 4096  # 4 line-stage jobs per transfer: 16384 in this pass
        assert list(ctx.verify_transfers([case_tuple(zero_norm[k]) for k in sel])) == want
        ctx.set_debug(challenges=True)
        b = ctx.load_transfers([case_tuple(zero_norm[k]) for k in sel])
        try:
            b.run()
            assert b.codes() == want
            check = sorted(set(range(0, n, 97)) | ({999, 1000, 1001, 3000, 3001, 3002} if layout == "sparse" else set()))
            for i in check:
                c = zero_norm[sel[i]]
                dev = b.challenges(i)
                assert compare(c["name"], c["expect"], dev, oracle_list(c)) > 0
        finally:
            b.close()

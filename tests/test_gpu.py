"""GPU parity tests: the HIP path (through the C ABI) against the oracle's golden
verdicts, plus size-independent properties at larger batch sizes."""
import random

import pytest

from conftest import case_tuple

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def zk():
    import zkatdlog
    return zkatdlog


@pytest.fixture(scope="module")
def ctx_a(zk, golden):
    c = zk.Context(golden["pp_a"]["pp"].encode(), device=0)
    yield c
    c.close()


def _codes(ctx, cases):
    tr = [c for c in cases if c["kind"] == "transfer"]
    iss = [c for c in cases if c["kind"] == "issue"]
    got = {}
    if tr:
        for c, code in zip(tr, ctx.verify_transfers([case_tuple(c) for c in tr])):
            got[c["name"]] = code
    if iss:
        for c, code in zip(iss, ctx.verify_issues([case_tuple(c) for c in iss])):
            got[c["name"]] = code
    return got


def test_golden_pp_a_verdicts(ctx_a, golden):
    cases = golden["pp_a"]["cases"]
    got = _codes(ctx_a, cases)
    bad = {c["name"]: (got[c["name"]], c["expect"]) for c in cases if got[c["name"]] != c["expect"]}
    assert not bad, bad
    assert sum(1 for c in cases if c["expect"] == 0) >= 10


@pytest.mark.parametrize("g2lines", ["sextet", "one_lane"])
@pytest.mark.parametrize("pp", ["pp_a", "pp_b"])
def test_golden_verdicts_every_layout(zk, golden, pp, g2lines):
    """every kernel layout (ftz_ctx_set_layout) gives the golden verdicts: the
    t' / pair-2 line stage writes the same bytes whichever layout runs it"""
    with zk.Context(golden[pp]["pp"].encode(), device=0) as c:
        c.set_layout("g2lines", g2lines)
        cases = golden[pp]["cases"]
        got = _codes(c, cases)
        assert got == {c_["name"]: c_["expect"] for c_ in cases}


@pytest.mark.parametrize("pp", ["pp_a", "pp_b"])
def test_golden_tiled_past_small_pass_default_layout(zk, golden, pp):
    """the default layout path of production-size passes: the golden transfer
    cases tiled to > ftz_options.small_pass G2 jobs per device pass (so the
    one-lane k_g2_part + k_g2lines1 stage runs, not the small-pass sextet one),
    no set_layout call, every verdict at its position"""
    cases = [c for c in golden[pp]["cases"] if c["kind"] == "transfer"]
    with zk.Context(golden[pp]["pp"].encode(), device=0) as c:
        assert c.options["small_pass"] == 4096
        n = 4096 if pp == "pp_a" else 1024  # PP-A 8, PP-B 64 G2 jobs per transfer that reaches the pairings
        sel = [k % len(cases) for k in range(n)]
        got = c.verify_transfers([case_tuple(cases[k]) for k in sel])
        assert list(got) == [cases[k]["expect"] for k in sel]


def test_set_layout_rejects_unknown_values(zk, ctx_a):
    """ftz_ctx_set_layout: unknown stage or layout -> FTZ_E_INVALID, the context unchanged"""
    lib = ctx_a._lib
    assert lib.ftz_ctx_set_layout(ctx_a._h, 7, 1) != 0
    assert lib.ftz_ctx_set_layout(ctx_a._h, 0, 2) != 0
    assert lib.ftz_ctx_set_layout(None, 0, 1) != 0
    with pytest.raises(KeyError):
        ctx_a.set_layout("pairing", "one_lane")


def test_golden_pp_b_verdicts(zk, golden):
    if "pp_b" not in golden:
        pytest.skip("no PP-B fixtures")
    with zk.Context(golden["pp_b"]["pp"].encode(), device=0) as c:
        cases = golden["pp_b"]["cases"]
        got = _codes(c, cases)
        assert {k: v for k, v in got.items()} == {c_["name"]: c_["expect"] for c_ in cases}


def test_verifier_api_messages(zk, ctx_a, golden):
    byname = {c["name"]: c for c in golden["pp_a"]["cases"]}
    ins, outs, proof = case_tuple(byname["valid_2in_2out"])
    v = zk.TransferVerifier([ins[:64], ins[64:]], [outs[:64], outs[64:]], ctx_a)
    v.verify(proof)
    ins, outs, proof = case_tuple(byname["ref_wrong_sum"])
    with pytest.raises(zk.ZKError) as e:
        zk.transfer_zkproof_validate(ctx_a, ins, outs, proof)
    assert "invalid zero-knowledge transfer" in str(e.value)
    outs, proof, anon = case_tuple(byname["issue_valid_0"])
    zk.IssueVerifier([outs[:64], outs[64:]], anon, ctx_a).verify(proof)


def test_batch_4096_verdict_positions(zk, ctx_a, golden):
    """A 4096-proof batch mixing valid and tampered proofs at random positions:
    the verdict bitmap must flag exactly the tampered positions."""
    cases = [c for c in golden["pp_a"]["cases"] if c["kind"] == "transfer"]
    good = [case_tuple(c) for c in cases if c["expect"] == 0]
    bad = [(case_tuple(c), c["expect"]) for c in cases if c["expect"] != 0]
    rng = random.Random(4096)
    items, expect = [], []
    for i in range(4096):
        if rng.random() < 1 / 64:
            t, code = rng.choice(bad)
        else:
            t, code = rng.choice(good), 0
        items.append(t)
        expect.append(code)
    b = ctx_a.load_transfers(items)
    b.run()
    assert b.codes() == expect
    bits = b.bitmap()
    acc = [(bits[i // 8] >> (i % 8)) & 1 for i in range(4096)]
    assert acc == [1 if e == 0 else 0 for e in expect]
    b.run()  # re-running on resident inputs is idempotent
    assert b.codes() == expect
    st = b.stats()
    assert st["total"][0] > 0 and st["miller"][1] > 0
    # two batches in flight on their own streams (ftz_batch_submit / wait):
    # same verdicts as the synchronous runs, each batch resubmitted once
    b2 = ctx_a.load_transfers(items[::-1])
    for _ in range(2):
        b.submit()
        b2.submit()
        b.wait()
        b2.wait()
    assert b.codes() == expect and b2.codes() == expect[::-1]
    b2.close()
    b.close()


def test_fp_multiplier_self_check():
    """Inline-asm FIPS Montgomery product == C CIOS product on 2 x 4M random
    inputs per field (p and r), including (m-1)^2."""
    import ctypes
    import os
    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                   "fabric-token-sdk_amd", "zkatdlog", "_lib", "libftsfpcheck.so"))
    lib.ftz_fpcheck.argtypes = [ctypes.c_int, ctypes.c_uint32]
    assert lib.ftz_fpcheck(0, 12345) == 0


def test_binv_tree_device_check():
    """dev/binv.h binv_tree256 (the 256-job batched inversion of k_fexp_binv /
    k_g2_binv) on the device against each lane's own fp_inv_var: random values,
    zeros alone and in runs (a t' at infinity; every lane of a block zero),
    and a partial last block whose inactive lanes write nothing"""
    import ctypes
    import os
    import random
    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                   "fabric-token-sdk_amd", "zkatdlog", "_lib", "libftsfpcheck.so"))
    lib.ftz_binvcheck.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32]
    rng = random.Random(5)
    for n in (256, 1000, 4096 + 37, 255, 1):
        z = bytearray(n)
        for _ in range(max(1, n // 50)):
            z[rng.randrange(n)] = 1
        if n >= 512:
            z[256:512] = b"\x01" * 256  # a block of zeros only
        assert lib.ftz_binvcheck(0, n, bytes(z), 1000 + n) == 0, n


def test_row29_device_check():
    """dev/row29.h (one field element per 16-lane DPP row: the MSM Horner
    chain's arithmetic) against dev/fp29.h on the device: products, carry
    normalisation, reduction, zero tests and four products at once through
    row_level, for normalised and signed-limb operands (1024 waves x 16 rounds
    x 4 rows): every limb identical"""
    import ctypes
    import os
    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                   "fabric-token-sdk_amd", "zkatdlog", "_lib", "libftsfpcheck.so"))
    out = (ctypes.c_uint32 * 3)()
    lib.ftz_rowcheck.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    assert lib.ftz_rowcheck(0, 777, out) == 0, list(out)


def test_safegcd_inverse_device_check():
    """dev/safegcd.h (fp_inv_var: Bernstein-Yang divsteps) against the binary
    Euclid fp_inv_eea on the device: 262,144 random Montgomery elements plus
    1, 2 and p - 1, each inverse equal and times its value one"""
    import ctypes
    import os
    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                   "fabric-token-sdk_amd", "zkatdlog", "_lib", "libftsfpcheck.so"))
    lib.ftz_invcheck.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32]
    assert lib.ftz_invcheck(0, 1024, 4242) == 0

"""GPU: the job engine behind ftz_verify_* (pipelined device batches,
micro-batching of concurrent callers), the final-exponentiation variants, and
the untested BASELINE configs at N = 1: a 1M-transfer sharded job (configs[3])
and a 1M-token transfer + issue prover run (configs[4]).

Parity anchors: the golden fixtures (oracle verdicts), GPU-made proofs whose
bytes equal the oracle prover's on a fixed sample, and the expected codes of
golden tampered cases placed at known rows."""
import ctypes
import hashlib
import threading
import time

import numpy as np
import pytest

from conftest import case_tuple

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def zk():
    import zkatdlog
    return zkatdlog


@pytest.fixture(scope="module")
def ctx(zk, golden):
    c = zk.Context(golden["pp_a"]["pp"].encode(), device=0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def valid_set(ctx):
    from zkatdlog import workload as W
    t0 = time.time()
    vs = W.prove_distinct(ctx, 16384, tag=b"engine-test")
    print("proved %d distinct transfers in %.2f s" % (vs.n, time.time() - t0), flush=True)
    return vs


@pytest.fixture(scope="module")
def bad_set():
    from zkatdlog import workload as W
    return W.golden_tampered()


def _fuentes_cases(golden):
    return golden["pp_a_fuentes"]["cases"]


def test_fexp_variants_end_to_end(zk, golden):
    """Both final-exponentiation kernels reproduce the oracle's GT bytes: a
    proof verifies only if every membership transcript (GT bytes included) is
    byte-identical.  Exact-variant golden proofs verify on an exact context,
    Fuentes-variant proofs on a Fuentes context, and each is rejected by the
    other variant exactly as the oracle predicts."""
    pp = golden["pp_a"]["pp"].encode()
    cases = _fuentes_cases(golden)
    valid_exact = [c for c in golden["pp_a"]["cases"] if c["kind"] == "transfer" and c["expect"] == 0][:3]
    for variant in ("exact", "fuentes"):
        with zk.Context(pp, device=0, fexp=variant) as c:
            for case in cases:
                want = case["expect"] if variant == "fuentes" else case["expect_exact"]
                if case["kind"] == "transfer":
                    got = c.verify_transfers([case_tuple(case)])[0]
                else:
                    got = c.verify_issues([case_tuple(case)])[0]
                assert got == want, (variant, case["name"], got, want)
            got = c.verify_transfers([case_tuple(x) for x in valid_exact])
            if variant == "exact":
                assert got == [0] * len(valid_exact)
            else:
                assert all(g == zk.FTZ_ERR_MEMBERSHIP for g in got)


def test_fuentes_prover_matches_oracle(zk, golden):
    """The Fuentes context's prover equals the oracle's under FE_FUENTES."""
    import random
    from ftsoracle import bn254 as C
    from ftsoracle import zkat as Z
    js = golden["pp_a"]["pp"].encode()
    pp = Z.PublicParams.from_json(js)
    rng = random.Random(99)
    iv = [rng.randrange(5000), rng.randrange(5000)]
    ov = [iv[0] + iv[1] - 7, 7]
    ib, ob = [rng.randrange(C.R) for _ in range(2)], [rng.randrange(C.R) for _ in range(2)]
    ins = [Z.token_commitment(pp, "ABC", v, b) for v, b in zip(iv, ib)]
    outs = [Z.token_commitment(pp, "ABC", v, b) for v, b in zip(ov, ob)]
    seed = hashlib.sha256(b"fuentes-prover").digest()
    w = {"inputs": b"".join(C.g1_bytes(p) for p in ins), "outputs": b"".join(C.g1_bytes(p) for p in outs),
         "in_values": iv, "in_bfs": ib, "out_values": ov, "out_bfs": ob, "type": "ABC", "seed": seed}
    old = C.FE_VARIANT
    C.FE_VARIANT = C.FE_FUENTES
    try:
        want = Z.transfer_prove(pp, Z.Rand(seed), ins, outs, list(zip(iv, ib)), list(zip(ov, ob)), "ABC", tag="tx")
    finally:
        C.FE_VARIANT = old
    with zk.Context(js, device=0, fexp="fuentes") as c:
        proofs, codes = c.prove_transfers([w])
        assert codes == [0] and proofs[0] == want
        assert c.verify_transfers([(w["inputs"], w["outputs"], want)]) == [0]


def test_engine_chunks_and_mixes(ctx, valid_set, bad_set, golden):
    """One call of 3 x 4096 + 123 proofs (one full 8192 device batch + a partial one): every row's code
    equals its expected code, while another thread's issue verifications share
    the engine (transfers and issues mix in device batches) and get their own
    results."""
    from zkatdlog import workload as W
    job = W.mixed_job(valid_set, bad_set, 3 * 4096 + 123, seed=5)
    issues = [c for c in golden["pp_a"]["cases"] if c["kind"] == "issue"]
    got_i = []

    def issue_worker():
        for _ in range(20):
            got_i.append(ctx.verify_issues([case_tuple(c) for c in issues]))

    th = threading.Thread(target=issue_worker)
    th.start()
    codes = ctx.verify_transfers_packed(job.ptr(), job.n)
    th.join()
    assert np.array_equal(codes, job.expect)
    assert (job.expect != 0).sum() > 100
    assert all(g == [c["expect"] for c in issues] for g in got_i)


@pytest.mark.parametrize("opts", [{"first_pass": 1000}, {"first_pass": 0}, {"first_pass": 2048, "tail_split": 1024},
                                  {"first_pass": 0, "tail_split": 3000}])
def test_engine_first_pass_and_tail_split(zk, golden, valid_set, bad_set, opts):
    """ftz_options.first_pass (the job's first pass smaller than the batch, so
    one request's items straddle two passes) and tail_split (the queue's last
    pass cut in two halves): every code at its row equals the single-pass
    result and the expected code, for one request of 8192 + 777 rows and for
    one just above a first pass"""
    from zkatdlog import workload as W
    pp = golden["pp_a"]["pp"].encode()
    job = W.mixed_job(valid_set, bad_set, 8192 + 777, seed=31)
    small = W.mixed_job(valid_set, bad_set, 1001, seed=32)
    with zk.Context(pp, device=0, **opts) as c:
        for j in (job, small):
            codes = c.verify_transfers_packed(j.ptr(), j.n)
            assert np.array_equal(codes, j.expect), opts
        st = c.engine_stats(reset=True)
        assert st["batches"] >= 2, st
    with zk.Context(pp, device=0, first_pass=0, tail_split=0) as c:  # one pass per batch: the reference codes
        assert np.array_equal(c.verify_transfers_packed(job.ptr(), job.n), job.expect)


def test_engine_1m_transfer_job_sharded(ctx, valid_set, bad_set):
    """BASELINE configs[3] at N = 1 through the multi-GPU job path: a job of
    2^20 transfers cut with shard_range (world 1, and each half of world 2 run
    back to back on this GPU), each shard verified in ONE call that the engine
    splits into device batches (8192, the default); codes bit-exact vs expected."""
    from zkatdlog import workload as W
    from zkatdlog.dist import bitmap_of, verify_shard
    n = 1 << 20
    job = W.mixed_job(valid_set, bad_set, n, seed=11)
    t0 = time.time()
    start, stop, codes = verify_shard(ctx, job.rows, n, 0, 1)
    dt = time.time() - t0
    print("1M-transfer job: %.2f s, %.0f transfers/s end to end" % (dt, n / dt), flush=True)
    assert (start, stop) == (0, n)
    assert np.array_equal(codes, job.expect)
    halves = [verify_shard(ctx, job.rows, n, r, 2) for r in range(2)]
    assert halves[0][1] == halves[1][0]
    joined = np.concatenate([h[2] for h in halves])
    assert np.array_equal(joined, job.expect)
    assert bitmap_of(joined) == bitmap_of(codes)


def test_microbatch_256_threads(ctx, valid_set, bad_set):
    """256 caller threads each verifying single transfers (n = 1 per call, as
    the Go shim's TransferZKProofValidate does): every call gets its own code;
    the engine coalesces them into shared device batches."""
    from zkatdlog import workload as W
    job = W.mixed_job(valid_set, bad_set, 256 * 16, seed=21)
    got = np.full(job.n, -99, dtype=np.int32)
    errs = []

    def worker(t):
        try:
            for k in range(16):
                i = t * 16 + k
                got[i] = ctx.verify_transfers_packed(job.ptr(i), 1)[0]
        except Exception as e:  # pragma: no cover - reported below
            errs.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(256)]
    t0 = time.time()
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.time() - t0
    assert not errs, errs[:3]
    assert np.array_equal(got, job.expect)
    t1 = time.time()
    staged = ctx.verify_transfers_packed(job.ptr(), job.n)
    dt1 = time.time() - t1
    assert np.array_equal(staged, job.expect)
    print("micro-batched: %d single-proof calls from 256 threads in %.2f s (%.0f/s); one %d-proof call: %.0f/s"
          % (job.n, dt, job.n / dt, job.n, job.n / dt1), flush=True)


def test_engine_errors_do_not_wedge(ctx, zk, valid_set):
    """A bad argument fails fast and the engine keeps serving."""
    assert ctx._lib.ftz_verify_transfers(ctx._h, 3, None, None) == -1  # FTZ_E_INVALID
    assert b"null" in ctx._lib.ftz_last_error()
    assert ctx.verify_transfers([valid_set.item(0)]) == [0]
    assert ctx.verify_transfers([]) == []


def test_engine_failure_isolation_requeue(zk, golden, valid_set, bad_set):
    """ADVICE r03 (engine.hip requeue_solo): a device pass that fails to plan --
    here an item poisoned with ftz_ctx_debug_poison, as a planner limit would --
    is handed back and every request in it re-planned solo.  16 concurrent
    callers (5..150 items, valid and tampered rows at known positions) share
    64-item passes; one caller's 150-item request carries the poisoned item at
    position 100, so that request is split across passes that plan fine
    (in flight or done) and the failing one.  The poisoned caller gets the error,
    every other caller its exact codes, and the engine keeps serving."""
    from zkatdlog import _abi as A
    rng = np.random.default_rng(64)
    reqs = []
    for k in range(16):
        n = 150 if k == 5 else int(rng.integers(5, 150))
        its, want = [], []
        for i in range(n):
            if rng.random() < 0.1:
                j = int(rng.integers(bad_set.n))
                its.append(bad_set.item(j))
                want.append(int(bad_set.expect[j]))
            else:
                its.append(valid_set.item(int(rng.integers(valid_set.n))))
                want.append(0)
        arr, keep = A.pack_transfers(its)
        reqs.append((arr, keep, n, want))
    with zk.Context(golden["pp_a"]["pp"].encode(), device=0, batch=64, slots=3, window_us=20000,
                    hold_inflight=0) as c:
        for rnd in range(2):
            poison = reqs[5][0][100].proof
            assert c._lib.ftz_ctx_debug_poison(c._h, poison) == 0
            go = threading.Barrier(len(reqs))
            res = [None] * len(reqs)

            def call(k):
                arr, keep, n, want = reqs[k]
                go.wait()
                try:
                    res[k] = list(c.verify_transfers_packed(arr, n))
                except zk.DeviceError as e:
                    res[k] = e
            th = [threading.Thread(target=call, args=(k,)) for k in range(len(reqs))]
            for t in th:
                t.start()
            for t in th:
                t.join(timeout=120)
            assert not any(t.is_alive() for t in th), "a caller is wedged"
            assert isinstance(res[5], zk.DeviceError) and "poisoned item" in str(res[5]), res[5]
            for k, (arr, keep, n, want) in enumerate(reqs):
                if k != 5:
                    assert res[k] == want, (rnd, k)
        assert c._lib.ftz_ctx_debug_poison(c._h, None) == 0
        arr, keep, n, want = reqs[5]
        assert list(c.verify_transfers_packed(arr, n)) == want


def test_prove_repeatedly_no_leak(ctx):
    """ftz_prove_transfers reuses the context's prover slots: 40 one-shot calls
    (no stream/event growth) and each result verifies."""
    from zkatdlog import _abi as A
    from zkatdlog import workload as W
    bases = W.witness_bases()[:4]
    for k in range(40):
        sel = np.arange(8) % 4
        p, n, keep = A.pack_transfer_witnesses_tiled(bases, sel, W.seeds(8, b"leak/%d" % k))
        blob, offs, codes = ctx.prove_packed("transfer", p, n)
        assert (codes == 0).all()
    ts = W.TransferSet.from_flat(np.frombuffer(b"".join(bases[i]["inputs"] for i in sel), dtype=np.uint8),
                                 np.arange(9) * 128,
                                 np.frombuffer(b"".join(bases[i]["outputs"] for i in sel), dtype=np.uint8),
                                 np.arange(9) * 128, blob, offs, np.zeros(8))
    assert (ctx.verify_transfers_packed(ctypes.cast(ts.rows.ctypes.data, ctypes.POINTER(A.Transfer)), 8) == 0).all()


def test_prover_1m_tokens(ctx, golden):
    """BASELINE configs[4] at N = 1: 2^20 output tokens -- 2^18 2-in/2-out
    transfers (2^19 tokens) and 2^18 2-output issues (2^19 tokens) -- proved
    on the GPU, every proof re-verified by the GPU verifier, and a fixed sample
    of 32 proofs byte-compared with the oracle prover (same seeds)."""
    from ftsoracle import bn254 as C
    from ftsoracle import zkat as Z
    from zkatdlog import _abi as A
    from zkatdlog import workload as W
    nt = ni = 1 << 18
    bases = W.witness_bases()
    t0 = time.time()
    tseeds = W.seeds(nt, b"1m-transfer")
    tsel = np.arange(nt) % len(bases)
    wp, n, keep = A.pack_transfer_witnesses_tiled(bases, tsel, tseeds)
    tblob, toffs, tcodes = ctx.prove_packed("transfer", wp, n)
    t1 = time.time()
    ibases = [{"outputs": b["outputs"], "values": b["out_values"], "bfs": b["out_bfs"], "type": b["type"],
               "anonymous": (k % 3 == 0)} for k, b in enumerate(bases)]
    iseeds = W.seeds(ni, b"1m-issue")
    isel = np.arange(ni) % len(ibases)
    ip, n2, keep2 = A.pack_issue_witnesses_tiled(ibases, isel, iseeds)
    iblob, ioffs, icodes = ctx.prove_packed("issue", ip, n2)
    t2 = time.time()
    assert (tcodes == 0).all() and (icodes == 0).all()
    print("proved %d transfers in %.2f s, %d issues in %.2f s (%d tokens)" % (nt, t1 - t0, ni, t2 - t1, 2 * nt + 2 * ni),
          flush=True)
    # every proof verified on the GPU
    ins = np.frombuffer(b"".join(b["inputs"] for b in bases), dtype=np.uint8)
    outs = np.frombuffer(b"".join(b["outputs"] for b in bases), dtype=np.uint8)
    rows = np.zeros(nt, dtype=A.transfer_dtype())
    ia, ik = A.buffer_address(ins)
    oa, ok_ = A.buffer_address(outs)
    pa, pk = A.buffer_address(tblob)
    rows["inputs"], rows["n_in"] = ia + 128 * tsel, 2
    rows["outputs"], rows["n_out"] = oa + 128 * tsel, 2
    rows["proof"], rows["proof_len"] = pa + toffs[:-1], toffs[1:] - toffs[:-1]
    tv = ctx.verify_transfers_packed(ctypes.cast(rows.ctypes.data, ctypes.POINTER(A.Transfer)), nt)
    assert (tv == 0).all(), np.unique(tv, return_counts=True)
    iout = np.frombuffer(b"".join(b["outputs"] for b in ibases), dtype=np.uint8)
    ioff = np.arange(len(ibases) + 1) * 128
    irows_out = ioff[isel]
    ia2, ik2 = A.buffer_address(iout)
    ib, ibk = A.buffer_address(iblob)
    idt = A._np_struct([("outputs", "<u8"), ("n_out", "<u4"), ("proof", "<u8"), ("proof_len", "<u8"),
                        ("anonymous", "u1")], A.Issue)
    irows = np.zeros(ni, dtype=idt)
    irows["outputs"], irows["n_out"] = ia2 + irows_out, 2
    irows["proof"], irows["proof_len"] = ib + ioffs[:-1], ioffs[1:] - ioffs[:-1]
    irows["anonymous"] = np.asarray([ibases[k]["anonymous"] for k in range(len(ibases))], dtype=np.uint8)[isel]
    codes = np.zeros(ni, dtype=np.int32)
    rc = ctx._lib.ftz_verify_issues(ctx._h, ni, ctypes.cast(irows.ctypes.data, ctypes.POINTER(A.Issue)),
                                    codes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    assert rc == 0 and (codes == 0).all(), np.unique(codes, return_counts=True)
    print("verified all %d proofs in %.2f s" % (nt + ni, time.time() - t2), flush=True)
    # oracle byte-equality on a fixed sample
    pp = Z.PublicParams.from_json(golden["pp_a"]["pp"].encode())
    dec = lambda b: [C.g1_from_bytes(b[64 * i:64 * i + 64]) for i in range(len(b) // 64)]
    for i in [0, 1, 63, 64, 4095, 4096, 65537, nt - 1] + [int(x) for x in np.linspace(5, nt - 2, 8)]:
        b = bases[tsel[i]]
        want = Z.transfer_prove(pp, Z.Rand(tseeds[32 * i:32 * i + 32]), dec(b["inputs"]), dec(b["outputs"]),
                                list(zip(b["in_values"], b["in_bfs"])), list(zip(b["out_values"], b["out_bfs"])),
                                b["type"], tag="tx")
        assert bytes(tblob[toffs[i]:toffs[i + 1]]) == want, i
    for i in [0, 2, 100, 4097, ni - 1] + [int(x) for x in np.linspace(7, ni - 3, 11)]:
        b = ibases[isel[i]]
        want = Z.issue_prove(pp, Z.Rand(iseeds[32 * i:32 * i + 32]), dec(b["outputs"]),
                             list(zip(b["values"], b["bfs"])), b["type"], anonymous=b["anonymous"], tag="issue")
        assert bytes(iblob[ioffs[i]:ioffs[i + 1]]) == want, i

"""The standalone G1 MSM (BASELINE configs[2]; dev/msm.h, k_msm.hip).

CPU tier: the pipeline's device functions run on the host (TEST-ONLY
tests/native/msm_emu.cpp) against the oracle's sum_i k_i P_i, at small window
sizes so that many windows, carries, empty and shared buckets occur.
GPU tier: ftz_msm_* through the C ABI, bit-exact against the oracle: explicit
points at small n, and at 2^16 / 2^20 the known-log points P_i = (i + off) G,
whose MSM is (sum_i k_i (i + off) mod r) G -- a size-independent check."""
import ctypes
import random

import pytest

from ftsoracle import bn254 as C


def rnd_case(n, seed, special=True):
    rng = random.Random(seed)
    pts = [C.g1_mul(C.G1_GEN, rng.randrange(1, C.R)) for _ in range(n)]
    ks = [rng.randrange(1 << 256) for _ in range(n)]
    if special and n >= 6:
        pts[1] = pts[0]                 # repeated point: bucket doubling
        ks[1] = ks[0]
        pts[2] = C.g1_neg(pts[3])       # P + (-P) in one bucket
        ks[2] = ks[3]
        ks[4] = 0                       # zero scalar
        ks[5] = C.R - 1                 # -1
    return pts, ks


def pack(pts, ks):
    return b"".join(C.g1_bytes(p) for p in pts), b"".join(k.to_bytes(32, "big") for k in ks)


def emu_msm(emu, pts, ks, c, cap, seg_len, glv=1, pre=0):
    pb, kb = pack(pts, ks)
    out = ctypes.create_string_buffer(64)
    emu.emu_msm_ex.argtypes = [ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p]
    assert emu.emu_msm_ex(len(pts), pb, kb, c, cap, seg_len, glv, pre, out) == 0
    return out.raw


@pytest.mark.parametrize("n,c,cap,seg", [(1, 4, 1, 1), (7, 2, 1, 1), (33, 5, 2, 3), (40, 8, 0, 0), (64, 3, 3, 2),
                                         (20, 1, 1, 1), (48, 6, 4, 5)])
@pytest.mark.parametrize("glv", [1, 0])
@pytest.mark.parametrize("pre", [0, 1])
def test_emu_pipeline(emu, n, c, cap, seg, glv, pre):
    """pre = 1: resident-point mode (window multiples 2^(c w) P, one bucket set,
    zero digits on the identity in bucket 0)"""
    pts, ks = rnd_case(n, 100 + n * 7 + c)
    assert emu_msm(emu, pts, ks, c, cap, seg, glv, pre) == C.g1_bytes(C.g1_msm(pts, ks))


@pytest.mark.parametrize("pre", [0, 1])
def test_emu_skewed_scalars(emu, pre):
    # small scalars pile into few buckets: heavy buckets are split over slots
    # (with pre the zero digits of every upper window land in bucket 0)
    rng = random.Random(77)
    pts, _ = rnd_case(60, 78, special=False)
    ks = [rng.randrange(1, 6) for _ in pts]
    assert emu_msm(emu, pts, ks, 4, 4, 3, 1, pre) == C.g1_bytes(C.g1_msm(pts, ks))


@pytest.mark.parametrize("pre", [0, 1])
def test_emu_cancelling_sum(emu, pre):
    pts, ks = rnd_case(8, 5, special=False)
    pts2 = pts + [C.g1_neg(p) for p in pts]
    assert emu_msm(emu, pts2, ks + ks, 4, 3, 2, 1, pre) == C.g1_bytes(None)


def test_emu_pre_identity_points(emu):
    """identity points among the resident points (all their multiples stay the
    identity) and all-zero scalars (every entry on the identity)"""
    pts, ks = rnd_case(12, 9, special=False)
    pts[3] = None
    pts[7] = None
    assert emu_msm(emu, pts, ks, 5, 2, 2, 1, 1) == C.g1_bytes(C.g1_msm(pts, ks))
    assert emu_msm(emu, pts, [0] * len(pts), 5, 2, 2, 1, 1) == C.g1_bytes(None)


def window_bits_var(nv):
    """dev/msm.h msm_window_bits_var: the variable-base planner's window bits for
    nv virtual points (GLV: 2n) -- 13 up to 2^19, then floor(log2 nv / 2) + 7
    clamped to [8, 20] except 17 at 2^22 and 19 at 2^23 (round-6 sweeps)."""
    lg = nv.bit_length() - 1
    if lg <= 19:
        return 13
    return {22: 17, 23: 19}.get(lg, min(20, max(8, lg // 2 + 7)))


def test_window_plan():
    assert [window_bits_var(2 << k) for k in (10, 16, 18, 19, 20, 21, 22, 23, 28)] == \
        [13, 13, 13, 17, 17, 17, 19, 19, 20]


@pytest.fixture(scope="module")
def ctx(golden):
    import zkatdlog
    c = zkatdlog.Context(golden["pp_a"]["pp"].encode(), device=0)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 5, 200, 1000])
def test_gpu_msm_explicit(ctx, n):
    pts, ks = rnd_case(n, 900 + n)
    pb, kb = pack(pts, ks)
    assert ctx.msm_g1(pb, kb) == C.g1_bytes(C.g1_msm(pts, ks))


@pytest.mark.gpu
def test_gpu_msm_without_glv(golden):
    import zkatdlog
    pts, ks = rnd_case(300, 901)
    pb, kb = pack(pts, ks)
    with zkatdlog.Context(golden["pp_a"]["pp"].encode(), device=0, msm_glv=0, msm_window_bits=9) as c:
        assert c.msm_g1(pb, kb) == C.g1_bytes(C.g1_msm(pts, ks))


@pytest.mark.gpu
def test_gpu_msm_precompute_explicit(golden):
    """resident-point mode through the C ABI: explicit points (identity and
    repeated points included), then new scalars on the same resident points"""
    import zkatdlog
    pts, ks = rnd_case(500, 902)
    pts[9] = None
    pb, kb = pack(pts, ks)
    with zkatdlog.Context(golden["pp_a"]["pp"].encode(), device=0, msm_precompute=1) as c:
        assert c.msm_g1(pb, kb) == C.g1_bytes(C.g1_msm(pts, ks))
        m = zkatdlog.Msm(c, pb, kb)
        try:
            assert m.run() == C.g1_bytes(C.g1_msm(pts, ks))
            ks2 = [random.Random(3).randrange(1 << 256) for _ in pts]
            m.set_scalars(b"".join(k.to_bytes(32, "big") for k in ks2))
            assert m.run() == C.g1_bytes(C.g1_msm(pts, ks2))
            m.set_scalars(bytes(32 * len(pts)))
            assert m.run() == C.g1_bytes(None)
        finally:
            m.close()


@pytest.mark.gpu
@pytest.mark.parametrize("lg,bits", [(20, 256), (16, 3)])
def test_gpu_msm_precompute_known_logs(golden, lg, bits):
    import zkatdlog
    n, off = 1 << lg, 999
    rng = random.Random(lg * 77 + bits)
    ks = [rng.randrange(1 << bits) for _ in range(n)]
    kb = b"".join(k.to_bytes(32, "big") for k in ks)
    with zkatdlog.Context(golden["pp_a"]["pp"].encode(), device=0, msm_precompute=1) as c:
        m = zkatdlog.Msm(c, scalars=kb, gen_offset=off)
        try:
            got = m.run()
            again = m.run()
            info = m.info()
        finally:
            m.close()
    assert got == C.g1_bytes(C.g1_mul(C.G1_GEN, _known_log_sum(kb, n, off)))
    assert again == got
    print("MSM 2^%d resident-point mode: %.3f ms device, window %d bits" % (lg, info["last_ms"], info["window_bits"]))


@pytest.mark.gpu
def test_gpu_msm_rejects_bad_point(ctx):
    import zkatdlog
    pts, ks = rnd_case(4, 3, special=False)
    pb, kb = pack(pts, ks)
    bad = bytearray(pb)
    bad[63] ^= 1
    with pytest.raises(zkatdlog.DeviceError, match="not a canonical"):
        ctx.msm_g1(bytes(bad), kb)


@pytest.mark.gpu
@pytest.mark.parametrize("pinned", [False, True])
def test_gpu_msm_run_scalars_from_host(ctx, pinned):
    """ftz_msm_run_scalars (chunked host copies overlapped with the fused key
    kernel): the known-log sum for new scalars, from pageable and page-locked
    memory, with n not a multiple of the chunk count; the scalars stay loaded
    for a following ftz_msm_run"""
    import zkatdlog
    n, off = (1 << 18) + 3, 777
    rng = random.Random(99 + pinned)
    k0 = [rng.randrange(C.R) for _ in range(n)]
    k1 = [rng.randrange(1 << 256) for _ in range(n)]  # unreduced: the device reduces mod r
    b0 = b"".join(k.to_bytes(32, "big") for k in k0)
    b1 = b"".join(k.to_bytes(32, "big") for k in k1)
    m = zkatdlog.Msm(ctx, scalars=b0, gen_offset=off)
    buf = None
    try:
        if pinned:
            buf = zkatdlog.HostBuffer(ctx, len(b1))
            buf.write(b1)
            got = m.run_scalars(buf)
        else:
            got = m.run_scalars(b1)
        again = m.run()
    finally:
        m.close()
        if buf is not None:
            buf.close()
    want = C.g1_mul(C.G1_GEN, sum(k * (i + off) for i, k in enumerate(k1)) % C.R)
    assert got == C.g1_bytes(want) and again == got


@pytest.mark.gpu
@pytest.mark.parametrize("lg,bits", [(16, 256), (20, 256), (16, 3), (18, 64)])
def test_gpu_msm_known_logs(ctx, lg, bits):
    """bits < 256: skewed scalars (a few hot buckets, most windows empty)."""
    import zkatdlog
    n, off = 1 << lg, 12345
    rng = random.Random(lg * 1000 + bits)
    ks = [rng.randrange(1 << bits) for _ in range(n)]
    kb = b"".join(k.to_bytes(32, "big") for k in ks)
    m = zkatdlog.Msm(ctx, scalars=kb, gen_offset=off)
    try:
        got = m.run()
        again = m.run()
        info = m.info()
    finally:
        m.close()
    want = C.g1_mul(C.G1_GEN, sum(k * (i + off) for i, k in enumerate(ks)) % C.R)
    assert got == C.g1_bytes(want)
    assert again == got
    assert info["window_bits"] == window_bits_var(2 << lg) and info["last_ms"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("c,radix", [(19, 0), (19, 8), (17, 9), (12, 9)])
def test_gpu_msm_radix_digits(golden, c, radix):
    """The sort's digit width (ftz_options.msm_radix_bits: 0 = the planner's
    9 bits for 17-18-bit keys, else 8) changes only the number of passes: with
    bucket-within-window keys and a stable sort every setting gives the known
    discrete log, zero digits included (scalars with zero windows)."""
    import zkatdlog
    n, off = 1 << 18, 4242
    rng = random.Random(c * 10 + radix)
    ks = [rng.randrange(1 << 256) % C.R for _ in range(n)]
    ks[:64] = [0, 1, C.R - 1] + [(1 << (19 * w)) for w in range(7)] + [rng.randrange(1 << 40) for _ in range(54)]
    kb = b"".join(k.to_bytes(32, "big") for k in ks)
    with zkatdlog.Context(golden["pp_a"]["pp"].encode(), device=0, msm_window_bits=c, msm_radix_bits=radix) as cx:
        m = zkatdlog.Msm(cx, scalars=kb, gen_offset=off)
        try:
            got = m.run()
            assert m.info()["window_bits"] == c
        finally:
            m.close()
    want = C.g1_mul(C.G1_GEN, sum(k * (i + off) for i, k in enumerate(ks)) % C.R)
    assert got == C.g1_bytes(want)


@pytest.mark.gpu
def test_gpu_msm_radix_bits_rejected(golden):
    import zkatdlog
    with pytest.raises(zkatdlog.DeviceError, match="msm_radix_bits"):
        zkatdlog.Context(golden["pp_a"]["pp"].encode(), device=0, msm_radix_bits=7)


def _known_log_sum(kb, n, off):
    """sum_i k_i (i + off) mod r for n big-endian 32-byte scalars, in 16-bit
    chunks with numpy (each chunk's dot product with i fits in uint64 for
    n <= 2^24)."""
    import numpy as np
    k = np.frombuffer(kb, dtype=">u2").reshape(n, 16).astype(np.uint64)  # chunk 0 = most significant
    idx = np.arange(n, dtype=np.uint64)
    total = 0
    for j in range(16):
        c = k[:, j]
        s = int(np.dot(c, idx)) + off * int(c.sum())
        total += s << (16 * (15 - j))
    return total % C.R


@pytest.mark.gpu
def test_gpu_msm_known_logs_2_24(ctx):
    """BASELINE configs[2] at its largest size: 2^24 points P_i = (i + off) G
    generated on the device, 2^24 uniform 256-bit scalars; the result must be
    (sum_i k_i (i + off)) G exactly, and stable across runs."""
    import numpy as np

    import zkatdlog
    n, off = 1 << 24, 777
    kb = np.random.default_rng(24).bytes(32 * n)
    want = C.g1_bytes(C.g1_mul(C.G1_GEN, _known_log_sum(kb, n, off)))
    m = zkatdlog.Msm(ctx, scalars=kb, gen_offset=off)
    try:
        got = m.run()
        again = m.run()
        info = m.info()
    finally:
        m.close()
    assert got == want
    assert again == got
    print("MSM 2^24: %.2f ms device, window %d bits" % (info["last_ms"], info["window_bits"]), flush=True)


def test_known_log_sum_helper():
    """the numpy chunked sum equals the big-int sum (CPU)"""
    import numpy as np
    n, off = 1000, 5
    kb = np.random.default_rng(3).bytes(32 * n)
    ks = [int.from_bytes(kb[32 * i:32 * i + 32], "big") for i in range(n)]
    assert _known_log_sum(kb, n, off) == sum(k * (i + off) for i, k in enumerate(ks)) % C.R


@pytest.mark.gpu
def test_gpu_g1_sum_edge_cases(ctx):
    """ftz_g1_sum (the split MSM's final add): identity entries, P + P,
    P + (-P), the empty sum, and a rejected off-curve point."""
    import zkatdlog
    rng = random.Random(5)
    p = C.g1_mul(C.G1_GEN, rng.randrange(1, C.R))
    q = C.g1_mul(C.G1_GEN, rng.randrange(1, C.R))
    inf = bytes(64)
    cases = [[p, q], [p, p], [p, C.g1_neg(p)], [p, None, q, None], [None], []]
    for pts in cases:
        want = C.G1_INF
        for x in pts:
            want = C.g1_add(want, x)
        got = ctx.g1_sum(b"".join(inf if x is None else C.g1_bytes(x) for x in pts))
        assert got == (inf if want is None else C.g1_bytes(want))
    bad = bytearray(C.g1_bytes(p))
    bad[63] ^= 1
    with pytest.raises(zkatdlog.DeviceError, match="point 1"):
        ctx.g1_sum(C.g1_bytes(q) + bytes(bad))


@pytest.mark.gpu
def test_gpu_msm_point_split_2_20(ctx):
    """The configs[2] multi-GPU split on one device: 2^20 known-log points cut
    into 4 contiguous rank slices (zkatdlog.dist.shard_range), each slice's MSM
    staged with its own generator offset, the 4 partials added by ftz_g1_sum:
    equal to (sum_i k_i (i + off)) G."""
    import numpy as np

    import zkatdlog
    from zkatdlog.dist import shard_range
    n, off, world = 1 << 20, 4242, 4
    kb = np.random.default_rng(20).bytes(32 * n)
    parts = []
    for r in range(world):
        a, b = shard_range(n, r, world)
        m = zkatdlog.Msm(ctx, scalars=kb[32 * a:32 * b], gen_offset=off + a)
        try:
            parts.append(m.run())
        finally:
            m.close()
    got = ctx.g1_sum(b"".join(parts))
    assert got == C.g1_bytes(C.g1_mul(C.G1_GEN, _known_log_sum(kb, n, off)))


@pytest.mark.parametrize("n,c,threads", [(1, 0, 1), (6, 3, 2), (40, 5, 3), (300, 0, 4), (2000, 0, 8)])
def test_cpu_pippenger_baseline(n, c, threads):
    """oracle/cpu msm_pippenger.cpp (the bench's CPU MSM baseline: XYZZ buckets,
    signed windows over GLV halves, tasks of window x point slice) against the
    oracle's sum, with repeated / cancelling points and zero / -1 scalars"""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle", "cpu"))
    import build_cpu
    lib = ctypes.CDLL(build_cpu.build())
    lib.cpu_msm_pippenger.argtypes = [ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                      ctypes.c_uint32, ctypes.c_char_p]
    pts, ks = rnd_case(n, 100 + n)
    ks = [k % C.R for k in ks]
    pb, kb = pack(pts, ks)
    out = ctypes.create_string_buffer(64)
    assert lib.cpu_msm_pippenger(n, pb, kb, threads, c, out) == 0
    want = None
    for p, k in zip(pts, ks):
        want = C.g1_add(want, C.g1_mul(p, k))
    assert out.raw == C.g1_bytes(want)

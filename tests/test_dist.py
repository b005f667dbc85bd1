"""Multi-rank sharding + verdict gather on CPU (gloo, world_size 2), the same
code bench.py runs over RCCL on N GPUs."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))


def test_shard_range_partitions():
    from zkatdlog.dist import shard_range
    for n in (0, 1, 7, 4096, 1000003):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from zkatdlog.dist import gather_verdicts, max_elapsed, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_total = 13
    a, b = shard_range(n_total, rank, world)
    accept = [(i % 3) != 0 for i in range(a, b)]  # global verdict pattern
    bits = bytearray((b - a + 7) // 8)
    for i, ok in enumerate(accept):
        if ok:
            bits[i // 8] |= 1 << (i % 8)
    maps, n_acc, ok = gather_verdicts(bytes(bits), b - a, rank != 1 or world == 1, dist)
    t = max_elapsed(0.5 + rank, dist)
    glob = []
    for r, m in enumerate(maps):
        ra, rb = shard_range(n_total, r, world)
        glob += [bool((m[i // 8] >> (i % 8)) & 1) for i in range(rb - ra)]
    q.put((rank, glob, n_acc, ok, t))
    dist.destroy_process_group()


def test_gather_verdicts_gloo_world2():
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [(i % 3) != 0 for i in range(13)]
    for rank, glob, n_acc, ok, t in res:
        assert glob == want
        assert n_acc == sum(want)
        assert ok is False  # rank 1 reported a mismatch: the MIN reduce must see it
        assert t == pytest.approx(1.5)


class _EmuVerifier:
    """TEST-ONLY stand-in for zkatdlog.Context on a CPU rank: the host build of
    the same planner + job code (tests/native), behind the one method
    zkatdlog.dist.verify_shard calls."""

    def __init__(self, pp_json):
        import ctypes
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from conftest import build_emu
        from zkatdlog import _abi as A
        self._A = A
        self.lib = ctypes.CDLL(build_emu())
        self.lib.emu_ctx_create.restype = ctypes.c_void_p
        self.lib.emu_ctx_create.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
        self.lib.emu_verify_transfers.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(A.Transfer),
                                                  ctypes.POINTER(ctypes.c_int32)]
        self.lib.emu_set_threads.argtypes = [ctypes.c_int]
        self.lib.emu_set_threads(2)
        self.h = self.lib.emu_ctx_create(pp_json, len(pp_json), ctypes.create_string_buffer(256), 256)

    def verify_transfers_packed(self, ptr, n):
        import ctypes

        import numpy as np
        codes = np.zeros(max(1, n), dtype=np.int32)
        if n:
            self.lib.emu_verify_transfers(self.h, n, ptr, codes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        return codes[:n]


def _golden_job():
    import base64
    import json

    from zkatdlog import workload as W
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "zkatdlog_golden.json")))["pp_a"]
    cases = [c for c in g["cases"] if c["kind"] == "transfer"][:26]
    items = [(bytes.fromhex(c["inputs"]), bytes.fromhex(c["outputs"]), base64.b64decode(c["proof"])) for c in cases]
    return g["pp"].encode(), W.TransferSet.from_items(items, [c["expect"] for c in cases])


def _worker_real(rank, world, port, q):
    import numpy as np
    import torch.distributed as dist

    from zkatdlog.dist import bitmap_of, gather_verdicts, shard_range, verify_shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pp, ts = _golden_job()
    v = _EmuVerifier(pp)
    start, stop, codes = verify_shard(v, ts.rows, ts.n, rank, world)
    ok_local = bool(np.array_equal(codes, ts.expect[start:stop]))
    maps, n_acc, ok = gather_verdicts(bitmap_of(codes), stop - start, ok_local, dist)
    glob = []
    for r, m in enumerate(maps):
        ra, rb = shard_range(ts.n, r, world)
        glob += [bool((m[i // 8] >> (i % 8)) & 1) for i in range(rb - ra)]
    q.put((rank, (start, stop), glob, n_acc, ok))
    dist.destroy_process_group()


def test_verify_shards_real_proofs_gloo_world2():
    """configs[3]'s job path on two CPU ranks: each rank verifies its
    shard_range slice of real golden proofs (valid and tampered) with the host
    build of the verifier, and the gathered verdict bitmaps equal the oracle's
    verdicts for the whole job."""
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    _, ts = _golden_job()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker_real, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [int(e) == 0 for e in ts.expect]
    assert any(want) and not all(want)
    spans = sorted(r[1] for r in res)
    assert spans[0][0] == 0 and spans[0][1] == spans[1][0] and spans[1][1] == ts.n
    for rank, span, glob, n_acc, ok in res:
        assert ok is True
        assert glob == want
        assert n_acc == sum(want)


class _EmuMsm:
    """TEST-ONLY stand-in for zkatdlog.Context on a CPU rank for the
    point-split MSM: the host build of dev/msm.h (tests/native/msm_emu.cpp)
    behind the two methods zkatdlog.dist.msm_shard uses."""

    def __init__(self):
        import ctypes
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from conftest import build_emu
        self.lib = ctypes.CDLL(build_emu())
        self.lib.emu_msm.argtypes = [ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32,
                                     ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p]
        self.lib.emu_g1_sum.argtypes = [ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p]

    def msm_g1(self, points, scalars):
        import ctypes
        out = ctypes.create_string_buffer(64)
        assert self.lib.emu_msm(len(points) // 64, points, scalars, 4, 0, 0, 1, out) == 0
        return out.raw

    def g1_sum(self, points):
        import ctypes
        out = ctypes.create_string_buffer(64)
        assert self.lib.emu_g1_sum(len(points) // 64, points, out) == 0
        return out.raw


def _msm_case(n):
    import random
    sys.path.insert(0, os.path.join(ROOT, "oracle", "py"))
    from ftsoracle import bn254 as C
    rng = random.Random(99)
    pts = [C.g1_mul(C.G1_GEN, rng.randrange(1, C.R)) for _ in range(n)]
    ks = [rng.randrange(1 << 256) for _ in range(n)]
    if n > 3:
        ks[3] = 0
    pb = b"".join(C.g1_bytes(p) for p in pts)
    kb = b"".join(k.to_bytes(32, "big") for k in ks)
    want = C.G1_INF
    for p, k in zip(pts, ks):
        want = C.g1_add(want, C.g1_mul(p, k % C.R))
    return pb, kb, C.g1_bytes(want)


def _worker_msm(rank, world, port, q, n):
    import torch.distributed as dist

    from zkatdlog.dist import msm_shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pb, kb, _ = _msm_case(n)
    ctx = _EmuMsm()
    start, stop, out = msm_shard(ctx, n, rank, world, dist,
                                 lambda a, b: ctx.msm_g1(pb[64 * a:64 * b], kb[32 * a:32 * b]))
    q.put((rank, start, stop, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 21), (3, 2)])
def test_msm_point_split_gloo(world, n):
    """configs[2] split over ranks: each rank's partial MSM of
    its point slice, one all-gather of the 64-byte partials, the final add on
    every rank -- equal to the oracle's whole sum (world 3 with n = 2 leaves
    one rank with no points: its partial is the identity)."""
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    _, _, want = _msm_case(n)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker_msm, args=(r, world, port, q, n)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted((r[1], r[2]) for r in res)[-1][1] == n
    for rank, start, stop, out in res:
        assert out == want


@pytest.mark.gpu
def test_rccl_rank_path_on_one_gpu():
    """bench.py's N > 1 path in the order a torchrun rank runs it: torch
    initialises HIP and joins an RCCL ("nccl") group, then the library opens
    its context in the same process (one HIP runtime: torch's, which the
    library's code objects run on).  One rank on one GPU: the tx-sharded
    verification, the verdict-bitmap all-gather, the MIN / MAX reduces and
    the point-split MSM's 64-byte partial gather (tests/gpu_scripts/
    dist_world1.py, a child process so that torch loads first)."""
    import json
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, "-u", os.path.join(here, "gpu_scripts", "dist_world1.py")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out == {"verdicts_ok": True, "elapsed_max": 0.125, "msm_matches_single": True}

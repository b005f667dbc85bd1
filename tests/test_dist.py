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

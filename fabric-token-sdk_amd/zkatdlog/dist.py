"""Multi-GPU sharding of a verification job.

Transfers are independent, so a job of N transfers is cut into contiguous
slices, one per rank (one process per GPU).  There is no data-path collective:
each rank verifies its slice on its own GPU; the only exchange is the gather
of the per-rank verdict bitmaps (RCCL all-gather over xGMI when the process
group backend is "nccl", gloo on CPU in the tests) and a MIN all-reduce of the
per-rank "verdicts matched the expected codes" flag.  The standalone MSM is
split by points instead (msm_shard): one 64-byte partial per rank is gathered
and added.
"""


def shard_range(n_total, rank, world):
    """Contiguous [start, stop) slice of n_total transfers owned by rank."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def verify_shard(ctx, rows, n_total, rank, world):
    """BASELINE configs[3]: this rank's contiguous slice [start, stop) of an
    n_total-transfer job, verified through the context's job engine (which cuts
    it into device batches and pipelines them).  rows: the job as a packed
    numpy ftz_transfer array (_abi.pack_transfers_flat rows, or a selection of
    them).  Returns (start, stop, codes)."""
    import ctypes

    from . import _abi
    start, stop = shard_range(n_total, rank, world)
    part = rows[start:stop]
    codes = ctx.verify_transfers_packed(ctypes.cast(part.ctypes.data, ctypes.POINTER(_abi.Transfer)), stop - start)
    return start, stop, codes


def msm_shard(ctx, n_total, rank, world, dist, partial):
    """SURVEY 8(e) for the standalone MSM (BASELINE configs[2]): the n_total
    points are split into contiguous slices, rank r computes the partial MSM of
    its slice with partial(start, stop) -> 64-byte RawBytes (ctx.msm_g1 or a
    staged Msm), the partials are all-gathered (one 64-byte collective per
    rank, RCCL over xGMI) and every rank adds them on its own device
    (ctx.g1_sum).  Returns (start, stop, 64-byte RawBytes of the whole sum)."""
    import torch
    start, stop = shard_range(n_total, rank, world)
    part = partial(start, stop) if stop > start else bytes(64)
    dev = _device(dist)
    t = torch.frombuffer(bytearray(part), dtype=torch.uint8).to(dev)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return start, stop, ctx.g1_sum(b"".join(p.cpu().numpy().tobytes() for p in parts))


def bitmap_of(codes):
    """verdict bitmap (bit i <=> transfer i accepted, LSB first) of a code array"""
    import numpy as np
    return np.packbits(np.asarray(codes) == 0, bitorder="little").tobytes()


def _device(dist):
    import torch
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")


def gather_verdicts(bits, n_local, ok_local, dist):
    """All-gather rank-local verdict bitmaps (bit i of rank r <=> transfer
    shard_start(r)+i accepted).  Returns (list of per-rank bitmaps as bytes,
    total accepted, all ranks matched their expected codes)."""
    import torch
    dev = _device(dist)
    world = dist.get_world_size()
    # ranks may hold different slice sizes: exchange sizes first, pad to max
    nb = torch.tensor([len(bits), n_local], dtype=torch.int64, device=dev)
    sizes = [torch.empty_like(nb) for _ in range(world)]
    dist.all_gather(sizes, nb)
    width = max(int(s[0].item()) for s in sizes) or 1
    bt = torch.zeros(width, dtype=torch.uint8, device=dev)
    if bits:
        bt[:len(bits)] = torch.frombuffer(bytearray(bits), dtype=torch.uint8).to(dev)
    gathered = [torch.empty_like(bt) for _ in range(world)]
    dist.all_gather(gathered, bt)
    okt = torch.tensor([1 if ok_local else 0], dtype=torch.int64, device=dev)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    import numpy as np
    out, n_accept = [], 0
    for g, s in zip(gathered, sizes):
        arr = g.cpu().numpy()[:int(s[0].item())]
        n = int(s[1].item())
        n_accept += int(np.unpackbits(arr, bitorder="little")[:n].sum())  # vectorised popcount
        out.append(arr.tobytes())
    return out, n_accept, bool(okt.item())


def max_elapsed(elapsed, dist):
    """Max over ranks of a wall-clock interval (the job ends with the slowest rank)."""
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=_device(dist))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())

"""GPU check of bench.py's N > 1 code path on one GPU (tests/test_dist.py runs
it as a child process): torch initialises HIP first and joins an RCCL ("nccl")
process group of one rank, then the library opens its context in the same
process, as in a torchrun rank; a tx-sharded verification, the verdict-bitmap
all-gather, the MIN flag reduce, the max-time reduce and the point-split MSM
with its 64-byte partial gather must all run and agree with the expected
results.  Prints one JSON line."""
import base64
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    torch.cuda.set_device(0)
    import tempfile
    store = os.path.join(tempfile.mkdtemp(prefix="ftz_dist_"), "store")  # a file rendezvous: no port to collide on
    dist.init_process_group("nccl", init_method="file://" + store, rank=0, world_size=1)
    import numpy as np

    import zkatdlog
    from zkatdlog import workload as W
    from zkatdlog.dist import bitmap_of, gather_verdicts, max_elapsed, msm_shard, verify_shard
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "zkatdlog_golden.json")))["pp_a"]
    out = {}
    with zkatdlog.Context(g["pp"].encode(), device=0) as ctx:
        cases = [c for c in g["cases"] if c["kind"] == "transfer"]
        ts = W.TransferSet.from_items([(bytes.fromhex(c["inputs"]), bytes.fromhex(c["outputs"]),
                                        base64.b64decode(c["proof"])) for c in cases], [c["expect"] for c in cases])
        job = W.mixed_job(ts, None, 4 * ts.n)
        rows, expect = job.rows, job.expect
        start, stop, codes = verify_shard(ctx, rows, job.n, 0, 1)
        ok_local = bool(np.array_equal(codes, expect))
        maps, n_accept, ok_all = gather_verdicts(bitmap_of(codes), stop - start, ok_local, dist)
        out["verdicts_ok"] = ok_local and ok_all and n_accept == int((expect == 0).sum())
        out["elapsed_max"] = max_elapsed(0.125, dist)
        n = 4096
        scal = np.random.default_rng(5).bytes(32 * n)

        def partial(a, b):
            m = zkatdlog.Msm(ctx, scalars=scal[32 * a:32 * b], gen_offset=1 + a)
            try:
                return m.run()
            finally:
                m.close()
        _, _, whole = msm_shard(ctx, n, 0, 1, dist, partial)
        out["msm_matches_single"] = whole == partial(0, n)
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)
    return 0 if out["verdicts_ok"] and out["elapsed_max"] == 0.125 and out["msm_matches_single"] else 1


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Generate tests/golden/bench_transfers.json: distinct valid 2-in/2-out
zkatdlog transfers on the golden PP-A (b=100, e=2) for bench.py, produced by
the CPU oracle (the reference prover cannot run here).  Values are uniform in
[1, (b^e-1)/2] per input and re-split uniformly over the outputs
(SURVEY.md section 8d, config C1/C2)."""
import base64
import json
import os
import random
import sys
from concurrent.futures import ProcessPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle", "py"))
from ftsoracle import bn254 as C  # noqa: E402
from ftsoracle import zkat as Z  # noqa: E402

N = int(os.environ.get("BENCH_SET_N", "64"))


def witness(k, pp):
    """the witnesses of bench transfer k (cheap: no group operations)"""
    rnd = Z.Rand(b"bench-set/%d" % k)
    rng = random.Random(k)
    hi = (pp.base ** pp.exponent - 1) // 2
    iv = [rng.randint(1, hi), rng.randint(1, hi)]
    o0 = rng.randint(0, sum(iv))
    ov = [o0, sum(iv) - o0]
    inw = [(v, rnd.zr("in/%d" % i)) for i, v in enumerate(iv)]
    outw = [(v, rnd.zr("out/%d" % i)) for i, v in enumerate(ov)]
    return rnd, inw, outw


def one(args):
    k, ppjson = args
    pp = Z.PublicParams.from_json(ppjson.encode())
    rnd, inw, outw = witness(k, pp)
    ins = [Z.token_commitment(pp, "ABC", v, b) for v, b in inw]
    outs = [Z.token_commitment(pp, "ABC", v, b) for v, b in outw]
    proof = Z.transfer_prove(pp, rnd, ins, outs, inw, outw, "ABC", tag="b%d" % k)
    return {"inputs": b"".join(C.g1_bytes(p) for p in ins).hex(),
            "outputs": b"".join(C.g1_bytes(p) for p in outs).hex(),
            "proof": base64.b64encode(proof).decode(), "expect": 0, **witness_json(inw, outw)}


def witness_json(inw, outw):
    # prover inputs for bench.py's batch-prover leg (BASELINE configs[4])
    return {"type": "ABC", "in_values": [v for v, _ in inw], "in_bfs": [str(b) for _, b in inw],
            "out_values": [v for v, _ in outw], "out_bfs": [str(b) for _, b in outw]}


def add_witnesses():
    """--witnesses: add the witness fields to an existing bench_transfers.json"""
    g = json.load(open(os.path.join(HERE, "zkatdlog_golden.json")))
    pp = Z.PublicParams.from_json(g["pp_a"]["pp"].encode())
    path = os.path.join(HERE, "bench_transfers.json")
    d = json.load(open(path))
    for k, t in enumerate(d["transfers"]):
        _, inw, outw = witness(k, pp)
        t.update(witness_json(inw, outw))
    json.dump(d, open(path, "w"))
    print("updated", path)


def main():
    if "--witnesses" in sys.argv:
        return add_witnesses()
    g = json.load(open(os.path.join(HERE, "zkatdlog_golden.json")))
    ppjson = g["pp_a"]["pp"]
    with ProcessPoolExecutor(max_workers=os.cpu_count()) as ex:
        items = list(ex.map(one, [(k, ppjson) for k in range(N)]))
    out = os.path.join(HERE, "bench_transfers.json")
    json.dump({"pp": "pp_a", "transfers": items}, open(out, "w"))
    print("wrote", out, len(items))


if __name__ == "__main__":
    main()

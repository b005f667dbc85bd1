#!/usr/bin/env python3
"""Generate tests/golden/ppb_prover_cases.json: PP-B (b = 16, e = 16, 64-bit
values) prover vectors from the oracle restatement (oracle/py/ftsoracle).

Each case is a witness (values, blinding factors, type, 32-byte seed) and the
oracle's proof bytes under the seeded ``Rand`` (rand(tag) = SHA-256(seed || tag
|| 0) || SHA-256(seed || tag || 1) mod r, tags "tx" / "issue"), plus the
oracle verifier's verdict on those bytes (every case here must be accepted).
The values sit where the reference's float64 digit code stops being exact
(range/proof.go:303-310: math.Pow(16, 16) does not fit an int64, so Go's own
prover refuses or mis-decomposes values near 2^63 and above) -- the oracle and
the library decompose by exact integer division, and the verifier accepts the
proofs, which pins that choice on the verifier side.

The GPU prover (tests/test_prover.py, -m gpu) and the host emulation (CPU
tier) must reproduce every proof byte for byte.  Runs in ~4 minutes on 8
cores:  python tests/golden/make_ppb_prover.py
"""
import base64
import hashlib
import json
import os
import random
import sys
from multiprocessing import Pool

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle", "py"))

from ftsoracle import bn254 as C  # noqa: E402
from ftsoracle import zkat as Z  # noqa: E402

OUT = os.path.join(HERE, "ppb_prover_cases.json")
M64 = (1 << 64) - 1
# (name, input values, output values); issues: (name, output values, anonymous)
TRANSFERS = [
    ("zero_one", [0, 1], [1, 0]),
    ("digit_max_int63", [15, (1 << 63) - 1], [15, (1 << 63) - 1]),
    ("two63_max_minus1", [1 << 63, M64 - 1], [M64 - 1, 1 << 63]),
    ("max_zero", [M64, 0], [0, M64]),
    ("split_to_max", [1 << 63, (1 << 63) - 1], [M64 - 1, 1]),
    ("random", None, None),
]
ISSUES = [
    ("issue_max", [M64, 7], False),
    ("issue_anon_two63", [1 << 63], True),
]


def _pp():
    with open(os.path.join(HERE, "zkatdlog_golden.json")) as f:
        js = json.load(f)["pp_b"]["pp"]
    return js, Z.PublicParams.from_json(js.encode())


def _transfer(args):
    i, (name, ins_v, outs_v) = args
    js, pp = _pp()
    rng = random.Random(7000 + i)
    if ins_v is None:
        ins_v = [rng.randrange(1 << 64) for _ in range(2)]
        outs_v = [ins_v[1], ins_v[0]]
    in_bf = [rng.randrange(C.R) for _ in ins_v]
    out_bf = [rng.randrange(C.R) for _ in outs_v]
    ttype = "PPB"
    ins = [Z.token_commitment(pp, ttype, v, b) for v, b in zip(ins_v, in_bf)]
    outs = [Z.token_commitment(pp, ttype, v, b) for v, b in zip(outs_v, out_bf)]
    seed = hashlib.sha256(b"ppb-prover-%d" % i).digest()
    proof = Z.transfer_prove(pp, Z.Rand(seed), ins, outs, list(zip(ins_v, in_bf)), list(zip(outs_v, out_bf)),
                             ttype, tag="tx")
    verdict = Z.transfer_verify(pp, ins, outs, proof)[1]
    return {"name": name, "kind": "transfer", "type": ttype, "seed": seed.hex(),
            "in_values": [str(v) for v in ins_v], "in_bfs": [str(b) for b in in_bf],
            "out_values": [str(v) for v in outs_v], "out_bfs": [str(b) for b in out_bf],
            "inputs": b"".join(C.g1_bytes(p) for p in ins).hex(),
            "outputs": b"".join(C.g1_bytes(p) for p in outs).hex(),
            "proof": base64.b64encode(proof).decode(), "oracle_verdict": verdict}


def _issue(args):
    i, (name, vals, anon) = args
    js, pp = _pp()
    rng = random.Random(7100 + i)
    bfs = [rng.randrange(C.R) for _ in vals]
    ttype = "PPB"
    outs = [Z.token_commitment(pp, ttype, v, b) for v, b in zip(vals, bfs)]
    seed = hashlib.sha256(b"ppb-issue-%d" % i).digest()
    proof = Z.issue_prove(pp, Z.Rand(seed), outs, list(zip(vals, bfs)), ttype, anonymous=anon, tag="issue")
    verdict = Z.issue_verify(pp, outs, proof, anonymous=anon)[1]
    return {"name": name, "kind": "issue", "type": ttype, "seed": seed.hex(), "anonymous": anon,
            "values": [str(v) for v in vals], "bfs": [str(b) for b in bfs],
            "outputs": b"".join(C.g1_bytes(p) for p in outs).hex(),
            "proof": base64.b64encode(proof).decode(), "oracle_verdict": verdict}


def main():
    with Pool(min(8, len(TRANSFERS) + len(ISSUES))) as pool:
        ts = pool.map_async(_transfer, list(enumerate(TRANSFERS)))
        iss = pool.map_async(_issue, list(enumerate(ISSUES)))
        cases = ts.get() + iss.get()
    bad = [c["name"] for c in cases if c["oracle_verdict"] != Z.OK]
    if bad:
        raise SystemExit("oracle rejects its own PP-B proofs: %s" % bad)
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_ppb_prover.py", "pp": "zkatdlog_golden.json:pp_b",
                   "cases": cases}, f, indent=1)
    print("wrote", OUT, len(cases), "cases")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Generate tests/golden/challenge_traces.json: every Fiat-Shamir challenge the
oracle verifier (oracle/py/ftsoracle, TEST INFRASTRUCTURE) recomputes on each
golden case -- the HashToZr of each well-formedness, membership and range
transcript, valid or tampered -- as [class, hex] in the order the checks run
(zkat.CHALLENGE_TRACE).  The GPU parity test reads the device's recomputed
challenges back (ftz_ctx_set_debug / ftz_batch_challenges) and compares them
with these, so a rejected proof is checked on its bytes, not only its verdict
class.

    python tests/golden/make_traces.py     # ~2 minutes on 8 cores
"""
import base64
import json
import os
import sys
from multiprocessing import Pool

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle", "py"))

from ftsoracle import bn254 as C  # noqa: E402
from ftsoracle import zkat as Z  # noqa: E402

OUT = os.path.join(HERE, "challenge_traces.json")
_PP = {}


def _trace(args):
    key, pp_json, c = args
    pp = _PP.get(key)
    if pp is None:
        pp = _PP[key] = Z.PublicParams.from_json(pp_json.encode())
    dec = lambda h: [C.g1_from_bytes(bytes.fromhex(h)[64 * i:64 * i + 64]) for i in range(len(h) // 128)]  # noqa: E731
    proof = base64.b64decode(c["proof"])
    Z.CHALLENGE_TRACE = []
    try:
        if c["kind"] == "transfer":
            code = Z.transfer_verify(pp, dec(c["inputs"]), dec(c["outputs"]), proof)[1]
        else:
            code = Z.issue_verify(pp, dec(c["outputs"]), proof, c["anonymous"])[1]
        tr = [[k, "%064x" % h] for k, h in Z.CHALLENGE_TRACE]
    finally:
        Z.CHALLENGE_TRACE = None
    return key, c["name"], code, tr


def main():
    with open(os.path.join(HERE, "zkatdlog_golden.json")) as f:
        g = json.load(f)
    with open(os.path.join(HERE, "ppc_golden.json")) as f:
        pc = json.load(f)
    jobs = []
    for key in ("pp_a", "pp_b"):
        jobs += [(key, g[key]["pp"], c) for c in g[key]["cases"]]
    for c in pc["cases"]:
        key = "pp_" + c["pp"].lower()
        jobs.append((key, pc[key]["pp"], c))
    # longest first (PP-B / PP-C transcripts hold 32-44 membership proofs)
    jobs.sort(key=lambda j: -len(j[2]["proof"]))
    with Pool(8) as pool:
        res = pool.map(_trace, jobs, chunksize=1)
    out = {}
    for key, name, code, tr in res:
        out.setdefault(key, {})[name] = {"expect": code, "challenges": tr}
    for key, cs in out.items():
        print(key, len(cs), "cases,", sum(len(v["challenges"]) for v in cs.values()), "challenges")
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_traces.py (zkat.CHALLENGE_TRACE)", "traces": out}, f)
    print("wrote", OUT)


if __name__ == "__main__":
    main()

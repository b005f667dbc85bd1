#!/usr/bin/env python3
"""Generate tests/golden/zero_norm_cases.json: PP-A transfers whose
membership proofs make t' = c PK0 + v PK1 + h PK2 the point at infinity
(Challenge = Value = Hash = 0; sigproof/pok.go:175-183), with the oracle's
verdicts and recomputed challenges (oracle/py/ftsoracle, TEST INFRASTRUCTURE).

A t' at infinity has a zero norm in the line stage's batched Fp2 inversion
(k_g2_sum / k_g2_binv) and its pairing contributes 1 (gnark's MillerLoop
skips an infinity pair), so the GPU test tiles these proofs between valid ones
into passes above the small-pass size, where one 256-job inversion tree holds
the zero norm and its neighbours' norms (dev/binv.h).

    python tests/golden/make_zero_norm.py
"""
import base64
import copy
import json
import os
import sys
from multiprocessing import Pool

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle", "py"))
sys.path.insert(0, HERE)

from ftsoracle import bn254 as C  # noqa: E402
from ftsoracle import zkat as Z  # noqa: E402
from make_golden import join_transfer, split_transfer, zr_elem  # noqa: E402

OUT = os.path.join(HERE, "zero_norm_cases.json")


def _pp():
    with open(os.path.join(HERE, "zkatdlog_golden.json")) as f:
        js = json.load(f)["pp_a"]["pp"]
    return Z.PublicParams.from_json(js.encode())


def _verify(c):
    pp = _pp()
    dec = lambda h: [C.g1_from_bytes(bytes.fromhex(h)[64 * i:64 * i + 64]) for i in range(len(h) // 128)]  # noqa: E731
    Z.CHALLENGE_TRACE = []
    try:
        _, code, msg = Z.transfer_verify(pp, dec(c["inputs"]), dec(c["outputs"]), base64.b64decode(c["proof"]))
        tr = [[k, "%064x" % h] for k, h in Z.CHALLENGE_TRACE]
    finally:
        Z.CHALLENGE_TRACE = None
    return code, msg, tr


def main():
    with open(os.path.join(HERE, "zkatdlog_golden.json")) as f:
        cases = json.load(f)["pp_a"]["cases"]
    base = next(c for c in cases if c["name"] == "valid_2in_2out")
    top, wf, rc = split_transfer(base64.b64decode(base["proof"]))
    out = []

    def add(name, digits):
        r = copy.deepcopy(rc)
        for k, i in digits:
            sp = r["MembershipProofs"][k]["SignatureProofs"][i]
            sp["Challenge"] = zr_elem(0)
            sp["Value"] = zr_elem(0)
            sp["Hash"] = zr_elem(0)
        c = dict(base)
        c.update(name=name, proof=base64.b64encode(join_transfer(top, wf, r)).decode())
        out.append(c)

    add("t_prime_infinity_digit_0_0", [(0, 0)])
    add("t_prime_infinity_digit_1_1", [(1, 1)])
    add("t_prime_infinity_every_digit", [(0, 0), (0, 1), (1, 0), (1, 1)])
    out.append(dict(base))
    with Pool(4) as pool:
        res = pool.map(_verify, out)
    for c, (code, msg, tr) in zip(out, res):
        c["expect"], c["message"], c["challenges"] = code, msg, tr
        print("%-36s code=%d %s (%d challenges)" % (c["name"], code, msg, len(tr)))
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_zero_norm.py", "pp": "zkatdlog_golden.json:pp_a",
                   "cases": out}, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()

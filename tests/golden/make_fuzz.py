#!/usr/bin/env python3
"""Make tests/golden/fuzz_cases.json: seeded mutations (fuzzmut.mutate) of the
golden corpus's valid PP-A / PP-B transfers and issues, each with the verdict of the
oracle restatement (ftsoracle.zkat.transfer_verify / issue_verify).  Test data only; the cases are
stored as (base, mode, pos, xor), the proofs are rebuilt by the tests.

    python tests/golden/make_fuzz.py [scale]
"""
import base64
import json
import os
import random
import sys
from multiprocessing import Pool

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle", "py"))
sys.path.insert(0, HERE)

from fuzzmut import MODES, mutate  # noqa: E402

BASES = [("pp_a", b, 60) for b in ["valid_2in_2out", "valid_2in_2out_1", "valid_3in_1out", "valid_1in_3out",
                                   "issue_valid_0", "issue_valid_2_anon"]]
BASES += [("pp_b", b, 20) for b in ["ppb_valid_2in_2out_64bit_values", "ppb_issue_valid_2_anon"]]
SEED = 20261017


def _load():
    g = json.load(open(os.path.join(HERE, "zkatdlog_golden.json")))
    return ({k: g[k]["pp"] for k in ("pp_a", "pp_b")},
            {k: {c["name"]: c for c in g[k]["cases"]} for k in ("pp_a", "pp_b")})


def _verdict(job):
    from ftsoracle import bn254 as C
    from ftsoracle import zkat as Z
    pp_json, case, mode, pos, xor = job
    pp = Z.PublicParams.from_json(pp_json.encode())
    ins_b, outs_b = bytes.fromhex(case["inputs"]), bytes.fromhex(case["outputs"])
    ins = [C.g1_from_bytes(ins_b[64 * i:64 * i + 64]) for i in range(len(ins_b) // 64)]
    outs = [C.g1_from_bytes(outs_b[64 * i:64 * i + 64]) for i in range(len(outs_b) // 64)]
    proof = mutate(base64.b64decode(case["proof"]), mode, pos, xor)
    if case["kind"] == "issue":
        return Z.issue_verify(pp, outs, proof, case["anonymous"])[1]
    return Z.transfer_verify(pp, ins, outs, proof)[1]


def main():
    scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    pps, cases = _load()
    rng = random.Random(SEED)
    rows = []
    for pp, b, n in BASES:
        for k in range(int(n * scale)):
            mode = MODES[k % len(MODES)]
            rows.append({"name": "fz_%s_%03d" % (b, k), "pp": pp, "base": b, "kind": cases[pp][b]["kind"], "mode": mode,
                         "pos": rng.randrange(1 << 20),
                         "xor": rng.randrange(1, 256)})
    with Pool(min(8, os.cpu_count() or 1)) as pool:
        codes = pool.map(_verdict, [(pps[r["pp"]], cases[r["pp"]][r["base"]], r["mode"], r["pos"], r["xor"])
                                    for r in rows])
    for r, c in zip(rows, codes):
        r["expect"] = c
    out = {"generator": "tests/golden/make_fuzz.py", "mutations": "tests/golden/fuzzmut.py", "seed": SEED,
           "oracle": "ftsoracle.zkat.transfer_verify / issue_verify (PP-A and PP-B)", "cases": rows}
    with open(os.path.join(HERE, "fuzz_cases.json"), "w") as f:
        json.dump(out, f, indent=0)
    hist = {}
    for c in codes:
        hist[c] = hist.get(c, 0) + 1
    print(len(rows), "cases, verdicts", dict(sorted(hist.items())))


if __name__ == "__main__":
    main()

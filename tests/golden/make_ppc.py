#!/usr/bin/env python3
"""Generate tests/golden/ppc_golden.json: public parameters whose range-proof
digit weights are NOT the exact powers of the base, with the oracle's
verdicts and proofs (oracle/py/ftsoracle, TEST INFRASTRUCTURE).

The reference weighs digit i by int64(math.Pow(float64(Base), float64(i)))
(range/proof.go:428 verifier; :303-311, :327 prover).  Go's math.Pow
(src/math/pow.go) is exact only while Base^i is a float64, and int64() of a
float64 >= 2^63 is -2^63 on amd64.  Two parameter sets exercise both:

* PP-C (b = 7, e = 22): 7^19 .. 7^22 exceed 2^53, and math.Pow gives
  7^19 + 1, 7^20 - 1, 7^21 + 25, 7^22 + 239.  The reference's prover
  decomposes values with those weights (quotient / remainder, values[0] = v %
  7 on the original v), so
    - some values give digits whose Go-weighted sum is v but whose exact sum
      is not: accepted by the reference, rejected with exact weights;
    - some give digits whose Go-weighted sum is not v: the reference's
      verifier rejects its own prover's proof ("invalid range proof");
    - some make a digit 7, which indexes past Signatures: the prover panics;
    - a proof made with exact weights (base-7 digits, blinding factor
      sum_i bf_i 7^i) is rejected by the reference; every proof made with
      the reference's weights is rejected with exact ones, since its
      blinding factor weighs all 22 digits.
* PP-D (b = 1000, e = 8): 1000^7 >= 2^63, so w_7 = -2^63 (the build once
  refused such parameters).  The reference's prover refuses every value
  (v >= int64(math.Pow(1000, 8)) = -2^63), so the proofs here are crafted with
  explicit digits (range_prove's digit_rows); the reference's verifier
  accepts one whose tokens commit to sum_i d_i w_i mod r.

Each case carries the verdict under the reference's weights ("expect") and
under exact integer weights ("expect_exact_weights", the counterfactual the
parity tests use to show the weights matter).  Prover cases carry the witness
and seed so that the library's prover can be checked byte for byte.

    python tests/golden/make_ppc.py        # ~2 minutes on 8 cores
"""
import base64
import copy
import hashlib
import json
import os
import random
import sys
from multiprocessing import Pool

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle", "py"))
sys.path.insert(0, HERE)

from ftsoracle import bn254 as C  # noqa: E402
from ftsoracle import zkat as Z  # noqa: E402
from make_golden import join_transfer, split_transfer, zr_elem, zr_val, other_point  # noqa: E402

OUT = os.path.join(HERE, "ppc_golden.json")
B_C, E_C = 7, 22
B_D, E_D = 1000, 8
TTYPE = "PPC"


def _pp(which):
    if which == "C":
        return Z.setup(B_C, E_C, Z.Rand(b"golden-pp-C"))
    return Z.setup(B_D, E_D, Z.Rand(b"golden-pp-D"))


_PP = {}


def pp_of(which):
    if which not in _PP:
        _PP[which] = _pp(which)
    return _PP[which]


def categorize(v, b, e):
    """'panic' | 'refused' | (go-weighted sum == v, exact sum == v) of the reference prover's digits"""
    try:
        d = Z.digits(v, b, e)
    except Z.Panic:
        return "panic"
    except ValueError:
        return "refused"
    go = sum(x * Z.digit_weight(b, i) for i, x in enumerate(d)) == v
    ex = sum(x * b ** i for i, x in enumerate(d)) == v
    return (go, ex)


def pick_values():
    """Deterministic PP-C values of each category."""
    rng = random.Random(20261018)
    want = {(True, False): [], (False, False): [], (False, True): []}
    while any(len(x) < 4 for x in want.values()):
        v = rng.randrange(B_C ** 19, B_C ** 22)
        c = categorize(v, B_C, E_C)
        if c in want and len(want[c]) < 4:
            want[c].append(v)
    w21, w22 = Z.digit_weight(B_C, 21), Z.digit_weight(B_C, 22)
    panic = None
    for q in range(1, 7):
        for off in range(-300, 300):
            v = q * w21 + (B_C ** 21 - 7) + off
            if 0 <= v < w22 and categorize(v, B_C, E_C) == "panic":
                panic = v
                break
        if panic is not None:
            break
    above = B_C ** 22 + 5  # < w22 = 7^22 + 239: the reference proves it (exact bound refuses it)
    return want, panic, above


def witness_transfer(which, name, ins_v, outs_v, seed_tag, digit_rows=None):
    pp = pp_of(which)
    rng = random.Random(seed_tag)
    in_bf = [rng.randrange(C.R) for _ in ins_v]
    out_bf = [rng.randrange(C.R) for _ in outs_v]
    ins = [Z.token_commitment(pp, TTYPE, v % C.R, b) for v, b in zip(ins_v, in_bf)]
    outs = [Z.token_commitment(pp, TTYPE, v % C.R, b) for v, b in zip(outs_v, out_bf)]
    seed = hashlib.sha256(seed_tag.encode()).digest()
    proof = Z.transfer_prove(pp, Z.Rand(seed), ins, outs, list(zip(ins_v, in_bf)), list(zip(outs_v, out_bf)),
                             TTYPE, tag="tx", digit_rows=digit_rows)
    return {"name": name, "pp": which, "kind": "transfer", "type": TTYPE, "seed": seed.hex(),
            "crafted": digit_rows is not None, "anonymous": False,
            "in_values": [str(v) for v in ins_v], "in_bfs": [str(b) for b in in_bf],
            "out_values": [str(v) for v in outs_v], "out_bfs": [str(b) for b in out_bf],
            "inputs": b"".join(C.g1_bytes(p) for p in ins).hex(),
            "outputs": b"".join(C.g1_bytes(p) for p in outs).hex(),
            "proof": base64.b64encode(proof).decode()}


def witness_issue(which, name, vals, anon, seed_tag):
    pp = pp_of(which)
    rng = random.Random(seed_tag)
    bfs = [rng.randrange(C.R) for _ in vals]
    outs = [Z.token_commitment(pp, TTYPE, v, b) for v, b in zip(vals, bfs)]
    seed = hashlib.sha256(seed_tag.encode()).digest()
    proof = Z.issue_prove(pp, Z.Rand(seed), outs, list(zip(vals, bfs)), TTYPE, anonymous=anon, tag="issue")
    return {"name": name, "pp": which, "kind": "issue", "type": TTYPE, "seed": seed.hex(), "crafted": False,
            "anonymous": anon, "values": [str(v) for v in vals], "bfs": [str(b) for b in bfs],
            "inputs": "", "outputs": b"".join(C.g1_bytes(p) for p in outs).hex(),
            "proof": base64.b64encode(proof).decode()}


def _make(job):
    kind = job[0]
    if kind == "tx":  # a proof made with exact integer weights (digits and blinding factor)
        Z.EXACT_WEIGHTS = True
        try:
            return witness_transfer(*job[1:])
        finally:
            Z.EXACT_WEIGHTS = False
    if kind == "t":
        return witness_transfer(*job[1:])
    return witness_issue(*job[1:])


def _verify(c):
    """(go verdict, go message, exact-weights verdict) of one case"""
    pp = pp_of(c["pp"])
    proof = base64.b64decode(c["proof"])
    dec = lambda h: [C.g1_from_bytes(bytes.fromhex(h)[64 * i:64 * i + 64]) for i in range(len(h) // 128)]
    res = []
    for exact in (False, True):
        Z.EXACT_WEIGHTS = exact
        if c["kind"] == "transfer":
            _, code, msg = Z.transfer_verify(pp, dec(c["inputs"]), dec(c["outputs"]), proof)
        else:
            _, code, msg = Z.issue_verify(pp, dec(c["outputs"]), proof, c["anonymous"])
        res.append((code, msg))
    Z.EXACT_WEIGHTS = False
    return res[0][0], res[0][1], res[1][0]


def tamper(c, name, fn):
    top, wf, rc = split_transfer(base64.b64decode(c["proof"]))
    r = copy.deepcopy(rc)
    fn(r)
    t = dict(c)
    t.update(name=name, crafted=True, proof=base64.b64encode(join_transfer(top, wf, r)).decode())
    return t


def main():
    want, panic, above = pick_values()
    A, Bc, Cc = want[(True, False)], want[(False, False)], want[(False, True)]
    small = 12345
    jobs = [
        ("t", "C", "ppc_low_values", [B_C ** 18 + 3, small], [small, B_C ** 18 + 3], "ppc-t-low"),
        ("t", "C", "ppc_high_digits_go_weights", [A[0], A[1]], [A[1], A[0]], "ppc-t-high"),
        ("t", "C", "ppc_reference_prover_inconsistent_digits", [Bc[0], small], [small, Bc[0]], "ppc-t-incons"),
        ("t", "C", "ppc_value_above_exact_bound", [above, small], [small, above], "ppc-t-above"),
        ("i", "C", "ppc_issue_high_digits", [A[2], small], False, "ppc-i-high"),
        ("i", "C", "ppc_issue_anon_high_digits", [A[3]], True, "ppc-i-anon"),
        # exact base-7 digits and blinding weights: the reference rejects it
        ("tx", "C", "ppc_crafted_exact_digits", [Cc[0], small], [small, Cc[0]], "ppc-t-exact",
         [[(small // B_C ** i) % B_C for i in range(E_C)], [(Cc[0] // B_C ** i) % B_C for i in range(E_C)]]),
    ]
    # PP-D: digits (d_0..d_7) with d_7 = 1 weighted by -2^63; the token holds sum d_i w_i mod r
    dd = [5, 1, 0, 7, 0, 0, 9, 1]
    vd = sum(d * Z.digit_weight(B_D, i) for i, d in enumerate(dd)) % C.R
    low = [3, 0, 2, 0, 0, 0, 0, 0]
    vl = sum(d * B_D ** i for i, d in enumerate(low))
    jobs += [
        ("t", "D", "ppd_weight_minus_2_63", [vd, vl], [vl, vd], "ppd-t-neg", [low, dd]),
        ("t", "D", "ppd_low_digits", [vl, 7], [7, vl], "ppd-t-low", [[7, 0, 0, 0, 0, 0, 0, 0], low]),
    ]
    with Pool(8) as pool:
        cases = pool.map(_make, jobs, chunksize=1)
    by = {c["name"]: c for c in cases}
    mp = lambda r, k, i: r["MembershipProofs"][k]["SignatureProofs"][i]  # noqa: E731

    def flip_mp(k, i):
        def f(r):
            mp(r, k, i)["Challenge"] = zr_elem(zr_val(mp(r, k, i)["Challenge"]) ^ 1)
        return f

    def flip_range(r):
        r["Challenge"] = zr_elem(zr_val(r["Challenge"]) ^ 2)

    def swap_coms(r):
        cs = r["MembershipProofs"][0]["Commitments"]
        cs[20], cs[21] = cs[21], cs[20]

    def replace_com(r):
        r["MembershipProofs"][1]["Commitments"][21] = {"curve": 1, "element": base64.b64encode(other_point(4242)).decode()}

    hi = by["ppc_high_digits_go_weights"]
    cases += [
        tamper(hi, "ppc_membership_digit21_bitflip", flip_mp(0, 21)),
        tamper(hi, "ppc_range_challenge_bitflip", flip_range),
        tamper(hi, "ppc_commitments_20_21_swapped", swap_coms),
        tamper(hi, "ppc_commitment21_replaced", replace_com),
        tamper(by["ppd_weight_minus_2_63"], "ppd_membership_digit7_bitflip", flip_mp(1, 7)),
        tamper(by["ppd_weight_minus_2_63"], "ppd_range_challenge_bitflip", flip_range),
    ]
    with Pool(8) as pool:
        res = pool.map(_verify, cases, chunksize=1)
    for c, (code, msg, ex) in zip(cases, res):
        c["expect"], c["message"], c["expect_exact_weights"] = code, msg, ex
        print("%-44s go=%d exact=%d %s" % (c["name"], code, ex, msg), flush=True)
    # prover refusals: (pp, value, outcome) with outcome "refused" | "panic" | "proves"
    refusals = [
        ("C", Z.digit_weight(B_C, 22), "refused"),
        ("C", Z.digit_weight(B_C, 22) - 1, categorize(Z.digit_weight(B_C, 22) - 1, B_C, E_C)),
        ("C", 1 << 63, "refused"),
        ("C", panic, "panic"),
        ("C", above, "proves"),
        ("D", 5, "refused"),
    ]
    refusals = [{"pp": p, "value": str(v), "outcome": o if isinstance(o, str) else "proves"} for p, v, o in refusals]
    for r in refusals:
        print("refusal", r, flush=True)
    out = {
        "generator": "tests/golden/make_ppc.py (oracle/py/ftsoracle; weights int64(math.Pow) as Go computes them)",
        "pp_c": {"base": B_C, "exponent": E_C, "pp": pp_of("C").to_json().decode(),
                 "weights": [str(Z.digit_weight(B_C, i)) for i in range(E_C + 1)]},
        "pp_d": {"base": B_D, "exponent": E_D, "pp": pp_of("D").to_json().decode(),
                 "weights": [str(Z.digit_weight(B_D, i)) for i in range(E_D + 1)]},
        "cases": cases,
        "prover_refusals": refusals,
    }
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT, len(cases), "cases")


if __name__ == "__main__":
    main()

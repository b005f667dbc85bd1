#!/usr/bin/env python3
"""Generate tests/golden/pp_validate.json: the PP-A public parameters with
structural mutations and the oracle's PublicParams.Validate verdict for each
(setup.go:238-273 restated in oracle/py/ftsoracle/zkat.py validate_json).

    python tests/golden/make_pp_cases.py
"""
import base64
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle", "py"))
from ftsoracle import zkat as Z  # noqa: E402


def main():
    g = json.load(open(os.path.join(HERE, "zkatdlog_golden.json")))["pp_a"]
    outer = json.loads(g["pp"])
    raw = json.loads(base64.b64decode(outer["Raw"]))

    def wrap(r, ident="zkatdlog"):
        return json.dumps({"Identifier": ident, "Raw": base64.b64encode(json.dumps(r).encode()).decode()}).encode()

    def mut(f):
        r = json.loads(json.dumps(raw))
        f(r)
        return wrap(r)

    def setk(path, v):
        def f(r):
            o = r
            for k in path[:-1]:
                o = o[k]
            o[path[-1]] = v
        return f
    cases = [("valid", wrap(raw)),
             ("curve_3", mut(setk(["Curve"], 3))),
             ("curve_negative_passes", mut(setk(["Curve"], -1))),
             ("idemix_curve_5", mut(setk(["IdemixCurveID"], 5))),
             ("pedgen_null", mut(setk(["PedGen"], None))),
             ("pedparams_len2", mut(lambda r: r["PedParams"].pop())),
             ("pedparams_null_entry", mut(setk(["PedParams", 1], None))),
             ("rpp_null", mut(setk(["RangeProofParams"], None))),
             ("signpk_len2", mut(lambda r: r["RangeProofParams"]["SignPK"].pop())),
             ("signedvalues_len1", mut(lambda r: r["RangeProofParams"].__setitem__(
                 "SignedValues", r["RangeProofParams"]["SignedValues"][:1]))),
             ("q_null", mut(setk(["RangeProofParams", "Q"], None))),
             ("exponent_0", mut(setk(["RangeProofParams", "Exponent"], 0))),
             ("signedvalue_null_entry", mut(setk(["RangeProofParams", "SignedValues", 3], None))),
             ("signpk_null_entry", mut(setk(["RangeProofParams", "SignPK", 2], None))),
             ("precision_32", mut(setk(["QuantityPrecision"], 32))),
             ("precision_missing", mut(lambda r: r.pop("QuantityPrecision"))),
             ("idemix_pk_null", mut(setk(["IdemixIssuerPK"], None))),
             ("idemix_pk_empty", mut(setk(["IdemixIssuerPK"], ""))),
             ("wrong_identifier", wrap(raw, "fabtoken")),
             ("precision_negative", mut(setk(["QuantityPrecision"], -64)))]
    out = []
    for name, data in cases:
        msg = Z.validate_json(data)
        out.append({"name": name, "pp": data.decode(), "error": msg})
        print("%-28s %s" % (name, msg or "ok"))
    json.dump(out, open(os.path.join(HERE, "pp_validate.json"), "w"), indent=1)


if __name__ == "__main__":
    main()

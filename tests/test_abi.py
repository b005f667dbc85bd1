"""CPU: the C-ABI library loads and exports every symbol include/ftsamd.h
declares (no compute calls here -- there is no GPU in the CPU tier)."""
import ctypes
import os
import re

import pytest

from zkatdlog import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(ROOT, "include", "ftsamd.h")).read()
    return sorted(set(re.findall(r"\b(ftz_[a-z0-9_]+)\s*\(", src)))


def test_header_matches_binding_list():
    assert declared() == sorted(_abi.SYMBOLS)


def test_library_exports_all_symbols():
    if not os.path.exists(_abi.LIB_PATH):
        pytest.skip("libftsamd.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_abi.LIB_PATH)
    missing = [s for s in declared() if not hasattr(lib, s)]
    assert not missing


def test_codes_match_header():
    src = open(os.path.join(ROOT, "include", "ftsamd.h")).read()
    for name in ("FTZ_OK", "FTZ_ERR_PARSE", "FTZ_ERR_MALFORMED", "FTZ_ERR_WF", "FTZ_ERR_RANGE",
                 "FTZ_ERR_MEMBERSHIP", "FTZ_ERR_PANIC"):
        m = re.search(r"#define %s (\d+)" % name, src)
        assert m and int(m.group(1)) == getattr(_abi, name)
    from ftsoracle import zkat as Z
    assert (Z.OK, Z.ERR_PARSE, Z.ERR_MALFORMED, Z.ERR_WF, Z.ERR_RANGE, Z.ERR_MEMBERSHIP, Z.ERR_PANIC) == \
        (0, 1, 2, 3, 4, 5, 6)


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_abi, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_abi, "_lib", None)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _abi.load()


def test_pp_validate_matches_oracle():
    """ftz_pp_validate (host side of the product library, no GPU) reproduces
    PublicParams.Validate (setup.go:238-273) on every golden mutation: same
    accept/reject and the same error text as the oracle restatement."""
    import json
    import os

    import zkatdlog
    cases = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pp_validate.json")))
    for c in cases:
        got = zkatdlog.validate_public_params(c["pp"].encode())
        if c["error"].startswith("failed unmarshalling"):
            assert got.startswith("failed unmarshalling"), (c["name"], got)
        else:
            assert got == c["error"], (c["name"], got, c["error"])
    assert sum(1 for c in cases if not c["error"]) == 2


def test_pp_setup_reproduces_golden_public_params(golden):
    """ftz_pp_setup (native crypto.Setup + Serialize, setup.go:119-128,214-236) with
    the golden fixtures' seeds gives their PP-A / PP-B bytes exactly (the oracle's
    zkat.setup made those), and the result passes PublicParams.Validate."""
    import zkatdlog
    for key, base, exp, seed in (("pp_a", 100, 2, b"golden-pp-A"), ("pp_b", 16, 16, b"golden-pp-B")):
        got = zkatdlog.setup_public_params(base, exp, seed)
        assert got == golden[key]["pp"].encode(), key
        assert not zkatdlog.validate_public_params(got)
    other = zkatdlog.setup_public_params(10, 3, b"another", idemix_pk=None, idemix_curve=1)
    from ftsoracle import zkat as Z
    want = Z.setup(10, 3, Z.Rand(b"another"), idemix_pk=None, idemix_curve=1).to_json()
    assert other == want

"""The one-statement limb products of csrc/gen_oneasm.py, executed by a small
interpreter of the generated gfx950 instructions and compared with big-integer
arithmetic (the GPU tests check the compiled code end to end)."""
import importlib.util
import os
import random
import re

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GEN = os.path.join(HERE, "..", "fabric-token-sdk_amd", "csrc", "gen_oneasm.py")
P = 0x30644e72e131a029b85045b68181585d97816a916871ca8d3c208c16d87cfd47
R = 0x30644e72e131a029b85045b68181585d2833e84879b9709143e1f593f0000001
M32 = (1 << 32) - 1


def _gen():
    spec = importlib.util.spec_from_file_location("gen_oneasm", GEN)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _run(stmt, inputs):
    """inputs: operand-expression -> value.  Returns output-expression -> value."""
    ops = [e for _, e in stmt.outs] + [e for _, e in stmt.ins]
    reg, sreg = {}, {}
    for i, e in enumerate(ops):
        if e in inputs:
            reg["%%%d" % i] = inputs[e]

    def val(x):
        if x.startswith("v["):
            a, b = map(int, re.findall(r"\d+", x))
            assert b == a + 1 and a % 2 == 0
            return reg["v%d" % a] | (reg["v%d" % b] << 32)
        if re.fullmatch(r"-?\d+", x):
            return int(x)
        return reg[x]

    def put(x, v):
        if x.startswith("v["):
            a, _ = map(int, re.findall(r"\d+", x))
            reg["v%d" % a] = v & M32
            reg["v%d" % (a + 1)] = (v >> 32) & M32
        else:
            reg[x] = v & M32

    for line in stmt.body:
        op, rest = line.split(None, 1)
        a = [t.strip() for t in rest.split(",")]
        if op == "v_mad_u64_u32":
            s = val(a[2]) * val(a[3]) + val(a[4])
            put(a[0], s)
            sreg[a[1]] = s >> 64
        elif op == "v_addc_co_u32":
            s = val(a[2]) + val(a[3]) + sreg[a[4]]
            put(a[0], s)
            sreg[a[1]] = s >> 32
        elif op == "v_add_co_u32":
            s = val(a[2]) + val(a[3])
            put(a[0], s)
            sreg[a[1]] = s >> 32
        elif op == "v_mov_b32":
            put(a[0], val(a[1]))
        elif op == "v_mul_lo_u32":
            put(a[0], val(a[1]) * val(a[2]))
        else:
            raise AssertionError(op)
        for r in re.findall(r"\bv(\d+)\b", a[0]):
            assert int(r) <= 3 or a[0].startswith("%"), line  # only the clobbered registers
    return {e: reg["%%%d" % i] for i, e in enumerate(ops[: len(stmt.outs)]) if "%%%d" % i in reg}


def _limbs(x, n):
    return [(x >> (32 * i)) & M32 for i in range(n)]


def _join(vals):
    return sum(v << (32 * i) for i, v in enumerate(vals))


def _consts(m):
    d = {"p%d" % i: v for i, v in enumerate(_limbs(m, 8))}
    d["inv"] = (-pow(m, -1, 1 << 32)) % (1 << 32)
    return d


@pytest.mark.parametrize("m", [P, R])
def test_mont_mul_oneasm(m):
    g, rng = _gen(), random.Random(1)
    st = g.build("mont")
    for it in range(200):
        a, b = (m - 1, m - 1) if it == 0 else (rng.randrange(m), rng.randrange(m))
        inp = dict(_consts(m))
        inp.update({"a[%d]" % i: v for i, v in enumerate(_limbs(a, 8))})
        inp.update({"b[%d]" % i: v for i, v in enumerate(_limbs(b, 8))})
        out = _run(st, inp)
        r = _join([out["r[%d]" % i] for i in range(8)])
        assert r % m == a * b * pow(2, -256, m) % m and r < 2 * m


def test_mul_wide_oneasm():
    g, rng = _gen(), random.Random(2)
    st = g.build("mulw")
    for it in range(200):
        a, b = ((1 << 256) - 1, (1 << 256) - 1) if it == 0 else (rng.getrandbits(256), rng.getrandbits(256))
        inp = {"a[%d]" % i: v for i, v in enumerate(_limbs(a, 8))}
        inp.update({"b[%d]" % i: v for i, v in enumerate(_limbs(b, 8))})
        out = _run(st, inp)
        assert _join([out["r[%d]" % i] for i in range(16)]) == a * b


def test_redc_wide_oneasm():
    g, rng = _gen(), random.Random(3)
    st = g.build("redc")
    for it in range(200):
        t = 14 * P * P - 1 if it == 0 else rng.randrange(14 * P * P)
        inp = dict(_consts(P))
        inp.update({"t[%d]" % i: v for i, v in enumerate(_limbs(t, 16))})
        out = _run(st, inp)
        r = _join([out["r[%d]" % i] for i in range(8)])
        assert r % P == t * pow(2, -256, P) % P and r < t // (1 << 256) + P

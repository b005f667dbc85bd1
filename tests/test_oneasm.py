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


# ---- carry chains of dev/fp_asm.h (gen_fpasm.py), interpreted from the header text
FPASM = os.path.join(HERE, "..", "fabric-token-sdk_amd", "csrc", "dev", "fp_asm.h")


def _fpasm_statements(fn):
    src = open(FPASM).read()
    i = src.index("void %s(" % fn)
    end = src.index("\n}\n", i)
    out = []
    for m in re.finditer(r'asm\("(.*?)"\s*:(.*?):(.*?)(?::\s*"vcc")?\);', src[i:end], re.S):
        body = m.group(1).split("\\n\\t")
        outs = re.findall(r'(?:\[(\w+)\]\s*)?"([=&+]*[vs])"\(([^)]*\)?)\)', m.group(2))
        ins = re.findall(r'"([vs])"\(([^)]*)\)', m.group(3))
        out.append((body, outs, ins))
    return out


def _exec_chain(stmts, env):
    for body, outs, ins in stmts:
        ops, named = [], {}
        for name, cons, expr in outs:
            ops.append(expr)
            if name:
                named[name] = expr
        ops += [e for _, e in ins]

        def ref(x):
            x = x.strip()
            m = re.fullmatch(r"%(\d+)", x)
            if m:
                return ops[int(m.group(1))]
            m = re.fullmatch(r"%\[(\w+)\]", x)
            if m:
                return named[m.group(1)]
            return x

        def val(x):
            e = ref(x)
            if e == "vcc":
                return env["vcc"]
            if re.fullmatch(r"0x[0-9a-f]+u", e):
                return int(e[:-1], 16)
            if re.fullmatch(r"\d+", e):
                return int(e)
            return env[e]

        for line in body:
            op, rest = line.split(None, 1)
            a = [ref(t) for t in rest.split(",")]
            base = op.rsplit("_e", 1)[0]
            if base in ("v_add_co_u32", "v_sub_co_u32", "v_addc_co_u32", "v_subb_co_u32"):
                x, y = val(a[2]), val(a[3])
                c = val(a[4]) & 1 if len(a) > 4 else 0
                r = x + y + c if "add" in base else x - y - c
                env[a[0]] = r & M32
                env[a[1]] = 1 if (r >> 32) != 0 else 0
            elif base == "v_cndmask_b32":
                env[a[0]] = val(a[2]) if val(a[3]) & 1 else val(a[1])
            elif base == "s_mov_b64":
                env[a[0]] = val(a[1])
            else:
                raise AssertionError(op)
    return env


def _arr(env, name, n):
    return _join([env["%s[%d]" % (name, i)] for i in range(n)])


def _set(env, name, x, n):
    for i, v in enumerate(_limbs(x, n)):
        env["%s[%d]" % (name, i)] = v


@pytest.mark.parametrize("m,suffix", [(P, "p"), (R, "r")])
def test_fpasm_addmod_submod_condsub(m, suffix):
    rng = random.Random(4)
    add, sub, cs = (_fpasm_statements("%s_%s_asm" % (k, suffix)) for k in ("addmod", "submod", "condsub"))
    for it in range(300):
        a, b = (m - 1, m - 1) if it == 0 else ((0, m - 1) if it == 1 else (rng.randrange(m), rng.randrange(m)))
        env = {}
        _set(env, "a", a, 8)
        _set(env, "b", b, 8)
        assert _arr(_exec_chain(add, dict(env)), "r", 8) == (a + b) % m
        assert _arr(_exec_chain(sub, dict(env)), "r", 8) == (a - b) % m
        x = rng.randrange(2 * m) if it > 1 else (m if it == 0 else 2 * m - 1)
        e2 = {}
        _set(e2, "x", x, 8)
        assert _arr(_exec_chain(cs, e2), "x", 8) == x % m


def test_fpasm_condsub2_acc16():
    rng = random.Random(5)
    cs2 = _fpasm_statements("condsub2_p_asm")
    for it in range(200):
        x = rng.randrange(3 * P) if it else 3 * P - 1
        env = {}
        _set(env, "x", x, 8)
        assert _arr(_exec_chain(cs2, env), "x", 8) == x % P
    a16, s16 = _fpasm_statements("add16_asm"), _fpasm_statements("sub16_asm")
    for it in range(200):
        r, a = rng.getrandbits(512), rng.getrandbits(512)
        env = {}
        _set(env, "r", r, 16)
        _set(env, "a", a, 16)
        assert _arr(_exec_chain(a16, dict(env)), "r", 16) == (r + a) % (1 << 512)
        assert _arr(_exec_chain(s16, dict(env)), "r", 16) == (r - a) % (1 << 512)

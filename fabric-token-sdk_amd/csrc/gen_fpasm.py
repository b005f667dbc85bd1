#!/usr/bin/env python3
"""Generate csrc/dev/fp_asm.h: carry chains of the modular add / subtract, the
final conditional subtraction and the 16-limb accumulator add / subtract as
single inline-asm statements (device only).

hipcc pads every dependent v_addc/v_subb pair of its own carry chains with an
s_nop (1-2 wait states); one asm statement per chain issues the chain back to
back, the same form as the FIPS multiplier's v_mad -> v_addc carries.  Modulus
limbs are VOP2 literal operands (v_subrev / v_subbrev / v_addc with a literal
src0), so the statements need no SGPRs."""
import os
import re

# Carry flag of the chains: "vcc" (VOP2 _e32 encodings) or "sgpr" (an SGPR pair
# output operand, VOP3 _e64 encodings).
CARRY = os.environ.get("FTS_FPASM_CARRY", "vcc")  # sgpr measured neutral (393k vs 399k)


def sgpr_carry(body, names=("cy",), first_in=16):
    """Rewrite a vcc chain to use %[cy] (and %[cy2] after a marker).  The carry
    pairs are extra output operands, so input operands >= first_in move up."""
    body = [re.sub(r"%(\d+)", lambda g: "%%%d" % (int(g.group(1)) + (int(g.group(1)) >= first_in)), l) for l in body]
    out, cur = [], names[0]
    for line in body:
        if line == "@SWITCH@":
            cur = names[1]
            continue
        if line.startswith("s_mov_b64 %[bw], vcc"):
            continue
        line = line.replace("_e32", "_e64")
        line = re.sub(r"\bvcc\b", "%%[%s]" % cur, line)
        out.append(line)
    return out

P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617


def limbs(x):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)]


def fn_addmod(name, m):
    # r = a + b mod m  (a, b < m): t = a + b; u = t - m; r = borrow ? t : u
    L = limbs(m)
    body = ["v_add_co_u32_e32 %8, vcc, %16, %24"]
    body += ["v_addc_co_u32_e32 %%%d, vcc, %%%d, %%%d, vcc" % (8 + i, 16 + i, 24 + i) for i in range(1, 8)]
    # modulus limbs in VGPR operands 32..39 (a literal plus the VCC carry
    # would exceed the one-scalar constant bus of a VOP2 instruction)
    body += ["v_sub_co_u32_e32 %0, vcc, %8, %32"]
    body += ["v_subb_co_u32_e32 %%%d, vcc, %%%d, %%%d, vcc" % (i, 8 + i, 32 + i) for i in range(1, 8)]
    body += ["v_cndmask_b32_e32 %%%d, %%%d, %%%d, vcc" % (i, i, 8 + i) for i in range(8)]
    return emit(name, body, "a", "b", mod=m)


def fn_submod(name, m):
    # r = a - b mod m: d = a - b; t = d + m; r = borrow ? t : d
    L = limbs(m)
    # operand 16 is the saved borrow mask: a = 17.., b = 25..
    body = ["v_sub_co_u32_e32 %8, vcc, %17, %25"]
    body += ["v_subb_co_u32_e32 %%%d, vcc, %%%d, %%%d, vcc" % (8 + i, 17 + i, 25 + i) for i in range(1, 8)]
    # keep the borrow mask: t = d + m does not touch it if computed with the
    # carry in an SGPR pair; here: save vcc, add, restore by re-deriving
    body += ["s_mov_b64 %[bw], vcc", "@SWITCH@"]
    body += ["v_add_co_u32_e32 %0, vcc, %8, %33"]
    body += ["v_addc_co_u32_e32 %%%d, vcc, %%%d, %%%d, vcc" % (i, 8 + i, 33 + i) for i in range(1, 8)]
    body += ["v_cndmask_b32_e64 %%%d, %%%d, %%%d, %%[bw]" % (i, 8 + i, i) for i in range(8)]
    return emit(name, body, "a", "b", extra_sgpr=True, mod=m)


def emit(name, body, x, y, extra_sgpr=False, mod=None):
    outs = ", ".join(['"=&v"(r[%d])' % i for i in range(8)] + ['"=&v"(t[%d])' % i for i in range(8)])
    decl = []
    if CARRY == "sgpr":
        # submod: cy takes bw's place (operand 16) and cy2 is operand 17
        body = [l.replace("%[bw]", "%[cy]") for l in sgpr_carry(body, ("cy", "cy2"), 17 if extra_sgpr else 16)]
        outs += ', [cy] "=&s"(cy)'
        decl.append("  uint64_t cy;")
        if extra_sgpr:
            outs += ', [cy2] "=&s"(cy2)'
            decl.append("  uint64_t cy2;")
        clob = ""
    else:
        body = [l for l in body if l != "@SWITCH@"]
        if extra_sgpr:
            outs += ', [bw] "=&s"(bw)'
            decl.append("  uint64_t bw;")
        clob = '\n               : "vcc"'
    ins = ", ".join(['"v"(%s[%d])' % (x, i) for i in range(8)] + ['"v"(%s[%d])' % (y, i) for i in range(8)] +
                    ['"v"(0x%08xu)' % v for v in limbs(mod)])
    s = []
    s.append("__device__ __forceinline__ void %s(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {" % name)
    s.append("  uint32_t t[8];")
    s += decl
    s.append("  asm(\"%s\"" % "\\n\\t".join(body))
    s.append("               : %s" % outs)
    s.append("               : %s%s);" % (ins, clob))
    s.append("}")
    return "\n".join(s)


def fn_condsub(name, m, twice=False):
    # r = x >= m ? x - m : x   (x < 2m); twice: x < 3m, subtract 2m then m
    out = []
    for mm in ([2 * m, m] if twice else [m]):
        body = ["v_sub_co_u32_e32 %8, vcc, %0, %16"]
        body += ["v_subb_co_u32_e32 %%%d, vcc, %%%d, %%%d, vcc" % (8 + i, i, 16 + i) for i in range(1, 8)]
        body += ["v_cndmask_b32_e32 %%%d, %%%d, %%%d, vcc" % (i, 8 + i, i) for i in range(8)]
        out.append((body, limbs(mm)))
    s = ["__device__ __forceinline__ void %s(uint32_t x[8]) {" % name, "  uint32_t t[8];"]
    if CARRY == "sgpr":
        s.append("  uint64_t cy;")
    for body, L in out:
        sg = CARRY == "sgpr"
        if sg:
            body = sgpr_carry(body)
        s.append('  asm("%s"' % "\\n\\t".join(body))
        s.append("      : %s" % ", ".join(['"+v"(x[%d])' % i for i in range(8)] + ['"=&v"(t[%d])' % i for i in range(8)]
                                         + (['[cy] "=&s"(cy)'] if sg else [])))
        s.append("      : %s%s);" % (", ".join('"v"(0x%08xu)' % v for v in L), "" if sg else ': "vcc"'))
    s.append("}")
    return "\n".join(s)


def fn_acc16(name, op):
    first, rest = ("v_add_co_u32_e32", "v_addc_co_u32_e32") if op == "add" else ("v_sub_co_u32_e32",
                                                                                  "v_subb_co_u32_e32")
    body = ["%s %%0, vcc, %%0, %%16" % first]
    body += ["%s %%%d, vcc, %%%d, %%%d, vcc" % (rest, i, i, 16 + i) for i in range(1, 16)]
    s = ["__device__ __forceinline__ void %s(uint32_t r[16], const uint32_t a[16]) {" % name]
    sg = CARRY == "sgpr"
    if sg:
        body = sgpr_carry(body)
        s.append("  uint64_t cy;")
    s.append("  asm(\"%s\"" % "\\n\\t".join(body))
    s.append("               : %s" % ", ".join(['"+v"(r[%d])' % i for i in range(16)] + (['[cy] "=&s"(cy)'] if sg else [])))
    s.append("               : %s%s);" % (", ".join('"v"(a[%d])' % i for i in range(16)), "" if sg else ' : "vcc"'))
    s.append("}")
    return "\n".join(s)


def main():
    L = ["// Generated by gen_fpasm.py -- do not edit.",
         "// Device-only carry chains as single inline-asm statements (gfx950).",
         "#pragma once  // included from fp.h inside namespace fts",
         "#if defined(__HIP_DEVICE_COMPILE__)"]
    L.append(fn_addmod("addmod_p_asm", P))
    L.append(fn_addmod("addmod_r_asm", R))
    L.append(fn_submod("submod_p_asm", P))
    L.append(fn_submod("submod_r_asm", R))
    L.append(fn_condsub("condsub_p_asm", P))
    L.append(fn_condsub("condsub_r_asm", R))
    L.append(fn_condsub("condsub2_p_asm", P, twice=True))
    L.append(fn_acc16("add16_asm", "add"))
    L.append(fn_acc16("sub16_asm", "sub"))
    L.append("#endif")
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dev", "fp_asm.h")
    open(path, "w").write("\n\n".join(L) + "\n")


if __name__ == "__main__":
    main()

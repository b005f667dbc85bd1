#!/usr/bin/env python3
"""Generate csrc/dev/fp_oneasm.h: the 8-limb Montgomery product (FIPS), the
8x8 -> 16 limb product and the 16 -> 8 limb Montgomery reduction, each as ONE
inline-asm statement.

The per-column statements of gen_fips.py / gen_wide.py leave C glue between
columns (carry-word shifts, m_k = acc * inv, r_k = acc) and hipcc pads each
statement boundary with an s_nop.  Here the 96-bit column accumulator lives in
fixed, clobbered registers: the 64-bit sum in one of the pairs v[0:1] / v[2:3]
and the carry word in the odd register of the other pair, so that the shift
acc >>= 32 at a column end is ONE v_mov into the other pair's even register
and the roles swap:

  v_mad_u64_u32 v[0:1], s[c:c+1], x, y, v[0:1]    acc += x * y
  v_addc_co_u32 v3, s[c:c+1], v3, 0, s[c:c+1]      carry word (first of a column: 0, 0)
  v_mov_b32 v2, v1                                  acc = (v2, v3) = acc >> 32

The carry flag is an SGPR pair chosen by the compiler, not VCC, and the shift is
a plain v_mov, not v_pk_mov_b32: both measured faster on gfx950
(tools/fpvariants.py).
"""
import os


class Stmt:
    def __init__(self):
        self.outs, self.ins, self.body = [], [], []

    def out(self, expr, cons="=&v"):
        self.outs.append((cons, expr))
        return "%%%d" % (len(self.outs) - 1)

    def render(self, indent="  "):
        text = "\\n\\t".join(self.body)
        outs = ", ".join('"%s"(%s)' % o for o in self.outs)
        ins = ", ".join('"%s"(%s)' % i for i in self.ins)
        return (indent + 'asm volatile("%s"\n' % text + indent + "    : %s\n" % outs + indent + "    : %s\n" % ins
                + indent + '    : "v0", "v1", "v2", "v3");')


def build(kind):
    """kind: 'mont' (a*b*R^-1 mod M, FIPS), 'mulw' (a*b, 16 limbs), 'redc' (t*R^-1, 16 -> 8 limbs)."""
    s = Stmt()
    names = {}
    nr = 16 if kind == "mulw" else 8
    for k in range(nr):
        names["r%d" % k] = s.out("r[%d]" % k)
    if kind != "mulw":
        for k in range(8):
            names["m%d" % k] = s.out("m[%d]" % k)
    CY = s.out("cy", "=&s")

    def add_in(cons, expr):
        s.ins.append((cons, expr))
        return "%%%d" % (len(s.outs) + len(s.ins) - 1)

    if kind in ("mont", "mulw"):
        for i in range(8):
            names["a%d" % i] = add_in("v", "a[%d]" % i)
        for i in range(8):
            names["b%d" % i] = add_in("v", "b[%d]" % i)
    if kind == "redc":
        for i in range(16):
            names["t%d" % i] = add_in("v", "t[%d]" % i)
    if kind in ("mont", "redc"):
        for i in range(8):
            names["p%d" % i] = add_in("s", "p%d" % i)
        names["inv"] = add_in("s", "inv")

    B = s.body
    st = {"cur": 0, "first": True}  # cur 0: acc v[0:1], carry word v3;  cur 1: acc v[2:3], carry word v1

    def pair():
        return "v[0:1]" if st["cur"] == 0 else "v[2:3]"

    def lo():
        return "v0" if st["cur"] == 0 else "v2"

    def hiw():
        return "v3" if st["cur"] == 0 else "v1"

    def mac(x, y, fresh):
        src = "0" if st["first"] else pair()
        st["first"] = False
        B.append("v_mad_u64_u32 %s, %s, %s, %s, %s" % (pair(), CY, x, y, src))
        if fresh:
            B.append("v_addc_co_u32 %s, %s, 0, 0, %s" % (hiw(), CY, CY))
        else:
            B.append("v_addc_co_u32 %s, %s, %s, 0, %s" % (hiw(), CY, hiw(), CY))

    def shift(add=None):
        # acc = (acc >> 32) [+ add]: into the other pair, whose odd register is the carry word
        if st["cur"] == 0:
            src_hi, dst_lo, dst_hi = "v1", "v2", "v3"
        else:
            src_hi, dst_lo, dst_hi = "v3", "v0", "v1"
        if add is None:
            B.append("v_mov_b32 %s, %s" % (dst_lo, src_hi))
        else:
            B.append("v_add_co_u32 %s, %s, %s, %s" % (dst_lo, CY, src_hi, add))
            B.append("v_addc_co_u32 %s, %s, %s, 0, %s" % (dst_hi, CY, dst_hi, CY))
        st["cur"] ^= 1

    ncols = 16 if kind == "redc" else 15
    for k in range(ncols):
        if kind == "redc":
            if k == 0:
                B.append("v_mov_b32 v0, %s" % names["t0"])
                B.append("v_mov_b32 v1, 0")
                st["first"] = False
            else:
                shift(names["t%d" % k])
        elif k > 0:
            shift()
        fresh = True
        prods = []
        if kind in ("mont", "mulw"):
            prods += [(names["a%d" % i], names["b%d" % (k - i)]) for i in range(8) if 0 <= k - i < 8]
        if kind in ("mont", "redc"):
            prods += [(names["m%d" % i], names["p%d" % (k - i)]) for i in range(8) if i < k and 0 <= k - i < 8]
        for x, y in prods:
            mac(x, y, fresh)
            fresh = False
        if kind in ("mont", "redc") and k < 8:
            B.append("v_mul_lo_u32 %s, %s, %s" % (names["m%d" % k], lo(), names["inv"]))
            mac(names["m%d" % k], names["p0"], fresh)
            fresh = False
        else:
            B.append("v_mov_b32 %s, %s" % (names["r%d" % (k if kind == "mulw" else k - 8)], lo()))
        if fresh and not (kind == "redc" and k == 15):  # only REDC's top column has no products
            raise AssertionError(k)
    if kind != "redc":
        shift()
        B.append("v_mov_b32 %s, %s" % (names["r%d" % (nr - 1)], lo()))
    return s


def main():
    L = []
    w = L.append
    w("// Generated by gen_oneasm.py -- do not edit.")
    w("// One-statement limb products for gfx950 (see gen_oneasm.py for the register scheme).")
    w("#pragma once  // included from fp.h inside namespace fts")
    w("#if defined(__HIP_DEVICE_COMPILE__)")
    w("template <class M>")
    w("__device__ __forceinline__ void mont_mul_oneasm(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {")
    w("  uint32_t m[8];")
    w("  uint64_t cy;")
    w("  const uint32_t p0 = M::m[0], p1 = M::m[1], p2 = M::m[2], p3 = M::m[3], p4 = M::m[4], p5 = M::m[5],"
      " p6 = M::m[6], p7 = M::m[7], inv = M::inv;")
    w(build("mont").render())
    w("}")
    w("")
    w("// r[16] = a[8] * b[8]")
    w("__device__ __forceinline__ void mul_wide_oneasm(uint32_t r[16], const uint32_t a[8], const uint32_t b[8]) {")
    w("  uint64_t cy;")
    w(build("mulw").render())
    w("}")
    w("")
    w("// r = t / 2^256 mod M up to a multiple: r < t / 2^256 + M (caller finishes the subtraction)")
    w("template <class M>")
    w("__device__ __forceinline__ void redc_wide_oneasm(uint32_t r[8], const uint32_t t[16]) {")
    w("  uint32_t m[8];")
    w("  uint64_t cy;")
    w("  const uint32_t p0 = M::m[0], p1 = M::m[1], p2 = M::m[2], p3 = M::m[3], p4 = M::m[4], p5 = M::m[5],"
      " p6 = M::m[6], p7 = M::m[7], inv = M::inv;")
    w(build("redc").render())
    w("}")
    w("#endif")
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dev", "fp_oneasm.h")
    open(path, "w").write("\n".join(L) + "\n")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Measured integer-VALU ceilings of the GPU (csrc/tools/madpeak.hip
ftz_valu_rate): wave-instructions per ns for each instruction stream the hot
kernels issue, alone and in the kernels' static mixes, at 1 / 2 / 4 / 8 waves
per SIMD.  Writes one JSON document (stdout, or --out).

    python fabric-token-sdk_amd/tools/valupeak.py --out profiles/r03_valu_rates.json
"""
import argparse
import ctypes
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "..", "zkatdlog", "_lib", "libftsmadpeak.so")
OPS = ["v_mad_u64_u32", "v_mad_i64_i32", "v_add_co_u32+v_addc_co_u32", "v_lshl_add_u64", "v_cndmask_b32",
       "v_mov_b32", "v_bfe_i32", "v_ashrrev_i64", "v_sub_co_u32+v_subb_co_u32",
       "mix: k_fexp_expt (9 mad_i64 : 2 add64 : 1 bfe : 1 ashr64 : 2 sub/subb : 1 mov)",
       "mix: 32-bit Montgomery (3 mad_u64 : 4 add_co/addc : 1 cndmask)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--iters", type=int, default=20000)
    ap.add_argument("--out")
    a = ap.parse_args()
    lib = ctypes.CDLL(LIB)
    lib.ftz_valu_rate.restype = ctypes.c_double
    lib.ftz_valu_rate.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32]
    lib.ftz_clock_mhz.restype = ctypes.c_int
    lib.ftz_madpeak.restype = ctypes.c_double
    lib.ftz_madpeak.argtypes = [ctypes.c_int, ctypes.c_uint32]
    mhz = lib.ftz_clock_mhz(a.device)
    simds = 1024
    rows = []
    for op, name in enumerate(OPS):
        r = {"op": op, "stream": name}
        for w in (1, 2, 4, 8):
            rate = lib.ftz_valu_rate(a.device, op, w, a.iters)
            r["w%d_wave_inst_per_ns" % w] = round(rate / 1e9, 4)
            # cycles per wave-instruction per SIMD at the reported clock
            r["w%d_cycles_per_inst" % w] = round(simds * mhz * 1e6 / rate, 3) if rate > 0 else None
        rows.append(r)
        print(json.dumps(r), flush=True)
    doc = {"tool": "fabric-token-sdk_amd/tools/valupeak.py (csrc/tools/madpeak.hip ftz_valu_rate)",
           "clock_mhz": mhz, "simds": simds, "iters": a.iters,
           "madpeak_lane_mad_per_s": lib.ftz_madpeak(a.device, 4096),
           "note": "wave-instructions per ns over the whole chip; cycles_per_inst = SIMDs x clock / rate "
                   "(1 = one wave64 instruction per SIMD per clock)", "streams": rows}
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        json.dump(doc, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""TEST / BASELINE INFRASTRUCTURE ONLY -- builds oracle/cpu/libftscpu.so, the
C++ CPU restatement of the zkatdlog batch verifier that bench.py's
cpu_baseline leg times.

It is the host build of the same job functions the GPU runs (dev/*.h: BN254
Fp/Fr, G1/G2, optimal-ate Miller loop, final exponentiation, SHA-256 /
HashToZr) and the same planner (host/planner.cpp: Go encoding/json, the
reference's check order), driven by tests/native/emu_exec.cpp over a thread
pool -- one thread per core -- with the Montgomery product in 4 x 64-bit limbs
(FTS_HOST64, 128-bit multiplies as gnark-crypto's generic Go code does) instead
of the GPU's 8 x 32-bit limbs.  Its verdicts are checked against the golden
fixtures (tests/test_cpu_baseline.py).  The product library (libftsamd.so) has
no CPU path; nothing in the product loads this file.

    python oracle/cpu/build_cpu.py
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
LIB = os.path.join(HERE, "libftscpu.so")
PKG = os.path.join(ROOT, "fabric-token-sdk_amd", "csrc")
SRCS = [os.path.join(ROOT, "tests", "native", f) for f in ("emu.cpp", "emu_exec.cpp", "msm_emu.cpp", "sx_emu.cpp")] + \
       [os.path.join(HERE, "msm_pippenger.cpp")] + \
       [os.path.join(PKG, "host", f) for f in ("planner.cpp", "planner_prove.cpp", "gojson.cpp", "request.cpp")]


def build(force=False):
    deps = SRCS + [os.path.join(d, f) for d in (os.path.join(PKG, "dev"), os.path.join(PKG, "host"))
                   for f in os.listdir(d) if f.endswith(".h")]
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(p) for p in deps):
        return LIB
    cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-Wno-unknown-pragmas", "-pthread", "-DFTS_HOST64"] + SRCS + \
          ["-o", LIB]
    subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))

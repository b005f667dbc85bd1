#!/usr/bin/env python3
"""Build libftsamd.so (HIP kernels for gfx950 + C++ host planner + C ABI).

One hipcc process per translation unit, run in parallel, incremental on
source/header mtimes.  Output: zkatdlog/_lib/libftsamd.so (in-tree, so it
travels to the GPU box with the repo snapshot).

    python fabric-token-sdk_amd/build.py [-j N] [--force]
"""
import argparse
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build", "obj")
LIB = os.path.join(HERE, "zkatdlog", "_lib", "libftsamd.so")
MADPEAK = os.path.join(HERE, "zkatdlog", "_lib", "libftsmadpeak.so")
FPCHECK = os.path.join(HERE, "zkatdlog", "_lib", "libftsfpcheck.so")
CALLERS = os.path.join(HERE, "zkatdlog", "_lib", "libftscallers.so")  # bench: closed-loop n=1 callers
ARCH = os.environ.get("FTS_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# 16-bit signed windows for the G1 fixed-base tables (dev/jobs.h FTS_G1TAB_C)
DEFS = ["-DFTS_G1TAB_C=16", "-DFTS_G2TAB_C=13"]
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wno-unknown-pragmas", "--offload-arch=" + ARCH] + DEFS

SOURCES = (sorted(glob.glob(os.path.join(CSRC, "k_*.hip")))
           + [os.path.join(CSRC, "runtime.hip"), os.path.join(CSRC, "engine.hip"), os.path.join(CSRC, "msm_rt.hip"),
              os.path.join(CSRC, "request_rt.hip"), os.path.join(CSRC, "idemix_rt.hip")]
           + sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp"))))


def headers():
    return (glob.glob(os.path.join(CSRC, "dev", "*.h")) + glob.glob(os.path.join(CSRC, "host", "*.h"))
            + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(HERE, "..", "include", "ftsamd.h")])


def newest(paths):
    return max(os.path.getmtime(p) for p in paths if os.path.exists(p))


def compile_one(src, force, hdr_time):
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_time):
        return obj, None
    cmd = [HIPCC] + FLAGS + ["-c", src, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC, "-O3", "-std=c++17", "-fPIC", "-Wno-unknown-pragmas"] + DEFS + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, "%s\n%s%s" % (" ".join(cmd), r.stdout, r.stderr)
    return obj, None


def build(jobs=8, force=False, verbose=True):
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    hdr_time = newest(headers())
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        results = list(ex.map(lambda s: compile_one(s, force, hdr_time), SOURCES))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    objs = [o for o, _ in results]
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < newest(objs):
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB] + objs + ["-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s\n%s%s" % (" ".join(cmd), r.stdout, r.stderr))
    for src, out in ((os.path.join(CSRC, "tools", "madpeak.hip"), MADPEAK),
                     (os.path.join(CSRC, "tools", "fpcheck.hip"), FPCHECK)):
        if force or not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(src), hdr_time):
            r = subprocess.run([HIPCC] + FLAGS + ["-shared", src, "-o", out], capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError("tool build failed:\n" + r.stderr)
    src = os.path.join(CSRC, "tools", "callers.cpp")
    if force or not os.path.exists(CALLERS) or os.path.getmtime(CALLERS) < max(os.path.getmtime(src),
                                                                               os.path.getmtime(LIB)):
        r = subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-pthread", src, "-o", CALLERS,
                            "-L" + os.path.dirname(LIB), "-lftsamd", "-Wl,-rpath,$ORIGIN"],
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("callers build failed:\n" + r.stderr)
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=8)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    try:
        build(a.j, a.force)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)

#!/usr/bin/env python3
"""Build libftsamd.so (HIP kernels for gfx950 + C++ host planner + C ABI).

One hipcc process per translation unit, run in parallel, incremental on
source/header mtimes.  Output: zkatdlog/_lib/libftsamd.so (in-tree, so it
travels to the GPU box with the repo snapshot).

    python fabric-token-sdk_amd/build.py [-j N] [--force]
    python fabric-token-sdk_amd/build.py --variant NAME --defs "-DFTS_SX_KARA=0"

--variant builds an A/B library with extra defines into zkatdlog/_lib/ab/
libftsamd_NAME.so (objects in build/obj_NAME); `bench.py --lib <path>`
(zkatdlog._abi.use_library) loads it instead of the default library for
same-box A/B runs.
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
# 16-bit signed windows for the G1 fixed-base tables (dev/jobs.h FTS_G1TAB_C);
# FTS_HOST64: the host side's Montgomery products (gnark SetBytes checks of the
# request path, PP decoding, the MSM result's affine conversion) in 4 x 64-bit
# limbs with 128-bit products -- bit-identical to the device's 8 x 32-bit ones
# (dev/fp.h); the device code is unaffected
DEFS = ["-DFTS_G1TAB_C=16", "-DFTS_G2TAB_C=13", "-DFTS_HOST64"]
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


def compile_one(src, force, hdr_time, obj_dir=OBJ, extra=()):
    obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_time):
        return obj, None
    cmd = [HIPCC] + FLAGS + list(extra) + ["-c", src, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC, "-O3", "-std=c++17", "-fPIC", "-Wno-unknown-pragmas"] + DEFS + list(extra) + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, "%s\n%s%s" % (" ".join(cmd), r.stdout, r.stderr)
    return obj, None


def build_variant(name, defs, jobs=8, force=False):
    """A/B library: the same sources with extra defines (see module doc)."""
    obj_dir = os.path.join(HERE, "build", "obj_" + name)
    lib = os.path.join(os.path.dirname(LIB), "ab", "libftsamd_%s.so" % name)
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    force = flags_changed(obj_dir, defs) or force
    hdr_time = newest(headers())
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        results = list(ex.map(lambda s: compile_one(s, force, hdr_time, obj_dir, defs), SOURCES))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    objs = [o for o, _ in results]
    if force or not os.path.exists(lib) or os.path.getmtime(lib) < newest(objs):
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib] + objs + ["-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s\n%s%s" % (" ".join(cmd), r.stdout, r.stderr))
    print("built", lib)
    return lib


def flags_changed(obj_dir, extra=()):
    """True (and the stamp rewritten) when the compile flags differ from the
    ones the objects in obj_dir were built with: a define change rebuilds."""
    stamp = os.path.join(obj_dir, ".flags")
    want = " ".join([HIPCC] + FLAGS + list(extra))
    have = open(stamp).read() if os.path.exists(stamp) else ""
    if have == want:
        return False
    with open(stamp, "w") as f:
        f.write(want)
    return True


def build(jobs=8, force=False, verbose=True):
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    force = flags_changed(OBJ) or force
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
    ap.add_argument("--variant", default=None)
    ap.add_argument("--defs", default="")
    a = ap.parse_args()
    try:
        if a.variant:
            build_variant(a.variant, a.defs.split(), a.j, a.force)
        else:
            build(a.j, a.force)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)

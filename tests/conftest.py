import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle", "py"))
sys.path.insert(0, os.path.join(ROOT, "fabric-token-sdk_amd"))
GOLDEN = os.path.join(ROOT, "tests", "golden", "zkatdlog_golden.json")
EMU_LIB = os.path.join(ROOT, "tests", "_build", "libftsemu.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def build_emu():
    """TEST-ONLY host build of the device job code + planner (tests/native)."""
    srcs = [os.path.join(ROOT, "tests", "native", "emu.cpp"), os.path.join(ROOT, "tests", "native", "emu_exec.cpp"),
            os.path.join(ROOT, "tests", "native", "sx_emu.cpp"), os.path.join(ROOT, "tests", "native", "msm_emu.cpp"),
            os.path.join(ROOT, "fabric-token-sdk_amd", "csrc", "host", "planner.cpp"), os.path.join(ROOT, "fabric-token-sdk_amd", "csrc", "host", "planner_prove.cpp"),
            os.path.join(ROOT, "fabric-token-sdk_amd", "csrc", "host", "gojson.cpp"),
            os.path.join(ROOT, "fabric-token-sdk_amd", "csrc", "host", "request.cpp"),
            os.path.join(ROOT, "tests", "native", "idemix_emu.cpp"),
            os.path.join(ROOT, "fabric-token-sdk_amd", "csrc", "host", "idemix.cpp")]
    deps = srcs + [os.path.join(d, f) for d in (os.path.join(ROOT, "fabric-token-sdk_amd", "csrc", "dev"),
                                              os.path.join(ROOT, "fabric-token-sdk_amd", "csrc", "host"))
                   for f in os.listdir(d) if f.endswith(".h")]
    if os.path.exists(EMU_LIB) and os.path.getmtime(EMU_LIB) >= max(os.path.getmtime(p) for p in deps):
        return EMU_LIB
    os.makedirs(os.path.dirname(EMU_LIB), exist_ok=True)
    cmd = ["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-Wno-unknown-pragmas", "-pthread"] + srcs + ["-o", EMU_LIB]
    subprocess.run(cmd, check=True)
    return EMU_LIB


@pytest.fixture(scope="session")
def emu():
    import ctypes

    from zkatdlog import _abi as A
    lib = ctypes.CDLL(build_emu())
    lib.emu_ctx_create.restype = ctypes.c_void_p
    lib.emu_ctx_create.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
    lib.emu_ctx_destroy.argtypes = [ctypes.c_void_p]
    lib.emu_verify_transfers.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(A.Transfer),
                                         ctypes.POINTER(ctypes.c_int32)]
    lib.emu_verify_issues.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(A.Issue),
                                      ctypes.POINTER(ctypes.c_int32)]
    return lib


def case_tuple(c):
    import base64
    if c["kind"] == "transfer":
        return (bytes.fromhex(c["inputs"]), bytes.fromhex(c["outputs"]), base64.b64decode(c["proof"]))
    return (bytes.fromhex(c["outputs"]), base64.b64decode(c["proof"]), c["anonymous"])

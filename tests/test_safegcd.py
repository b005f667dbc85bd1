"""dev/safegcd.h (the divsteps field inversion behind fp_inv_var) on the host:
both limb layouts against Python's modular inverse on random values and the
edges (1, 2, p - 1, (p - 1) / 2, powers of two).  The device check against the
binary Euclid is tests/test_gpu.py::test_safegcd_inverse_device_check."""
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 0x30644e72e131a029b85045b68181585d97816a916871ca8d3c208c16d87cfd47


@pytest.fixture(scope="module")
def sg_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("sg") / "sg_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "fabric-token-sdk_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "sg_check.cpp"), "-o", out], check=True)
    return out


@pytest.mark.parametrize("limbs", ["30", "62"])
def test_safegcd_matches_python(sg_bin, limbs):
    rng = random.Random(int(limbs))
    xs = [rng.randrange(1, P) for _ in range(5000)]
    xs += [1, 2, 3, P - 1, P - 2, (P - 1) // 2, (1 << 253) % P, 1 << 200, (1 << 30) - 1, (1 << 62) - 1]
    out = subprocess.run([sg_bin, limbs], input="".join("%064x\n" % x for x in xs).encode(),
                         capture_output=True, check=True).stdout.decode().split()
    assert len(out) == len(xs)
    bad = [x for x, o in zip(xs, out) if int(o, 16) != pow(x, -1, P)]
    assert not bad, [hex(x) for x in bad[:3]]

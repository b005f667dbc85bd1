"""The planner's strict base64 decoder (AVX2 32-character blocks, scalar
tail) agrees with the Go-semantics decoder on 200k random encodings, valid and
corrupted (tests/native/b64_check.cpp)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_strict_base64_matches_go_semantics(tmp_path):
    exe = str(tmp_path / "b64_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wno-unknown-pragmas",
                    os.path.join(ROOT, "tests", "native", "b64_check.cpp"),
                    os.path.join(ROOT, "fabric-token-sdk_amd", "csrc", "host", "gojson.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout

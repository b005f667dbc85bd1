"""Deterministic proof mutations for the fuzz fixture (tests/golden/fuzz_cases.json):
make_fuzz.py records (base case, mode, pos, xor) and the oracle's verdict; the
tests rebuild the same bytes with mutate() and compare the library's verdicts.

Modes on a TransferAction proof (Go json.Marshal of {WellFormedness, RangeCorrectness}
with both inner documents base64-encoded):
  outer     xor one byte of the outer JSON bytes
  wf_raw    xor one byte of the decoded WellFormedness JSON, re-encode
  rc_raw    the same for RangeCorrectness
  wf_elem   flip one bit inside one base64 string of the WellFormedness JSON
            (decoded, flipped, re-encoded: still well-formed base64)
  rc_elem   the same for RangeCorrectness
"""
import base64
import json

MODES = ["outer", "wf_raw", "rc_raw", "wf_elem", "rc_elem"]
_KEY = {"wf": "WellFormedness", "rc": "RangeCorrectness"}


def _b64_leaves(node, path, out):
    if isinstance(node, dict):
        for k, v in node.items():
            _b64_leaves(v, path + [k], out)
    elif isinstance(node, list):
        for i, v in enumerate(node):
            _b64_leaves(v, path + [i], out)
    elif isinstance(node, str) and len(node) >= 4 and len(node) % 4 == 0:
        try:
            base64.b64decode(node, validate=True)
            out.append(path)
        except ValueError:
            pass


def _get(node, path):
    for p in path:
        node = node[p]
    return node


def _set(node, path, v):
    for p in path[:-1]:
        node = node[p]
    node[path[-1]] = v


def mutate(proof, mode, pos, xor):
    """proof: outer proof bytes; pos >= 0, xor in 1..255 -> mutated proof bytes"""
    if mode == "outer":
        b = bytearray(proof)
        b[pos % len(b)] ^= xor
        return bytes(b)
    part, kind = mode.split("_")
    outer = json.loads(proof)
    key = _KEY[part]
    inner = base64.b64decode(outer[key])
    if kind == "raw":
        b = bytearray(inner)
        b[pos % len(b)] ^= xor
        inner = bytes(b)
    else:
        doc = json.loads(inner)
        leaves = []
        _b64_leaves(doc, [], leaves)
        path = leaves[pos % len(leaves)]
        raw = bytearray(base64.b64decode(_get(doc, path)))
        raw[(pos // len(leaves)) % len(raw)] ^= 1 << (xor % 8)
        _set(doc, path, base64.b64encode(bytes(raw)).decode())
        inner = json.dumps(doc, separators=(",", ":")).encode()
    outer[key] = base64.b64encode(inner).decode()
    return json.dumps(outer, separators=(",", ":")).encode()

"""Synthetic zkatdlog workloads for the bench and the GPU tests.

Distinct transfer proofs are made by the GPU batch prover (ftz_prove_transfers)
from a few witness bases -- the 2-in/2-out PP-A transfers of
tests/golden/bench_transfers.json, whose commitments the oracle computed -- with
a fresh 32-byte seed per proof, so every proof's randomness, commitments to
randomness, challenges and bytes differ (values uniform
in [1, (b^e-1)/2], outputs re-split).  Tampered proofs are taken from the golden
corpus (tests/golden/zkatdlog_golden.json) with their expected codes.

A TransferSet keeps the proof bytes in flat buffers and the job as a packed
numpy ftz_transfer array (zero-copy: rows point into the buffers), so a
1M-transfer job is a numpy selection of rows, not 1M Python objects.
"""
import base64
import ctypes
import hashlib
import json
import os

import numpy as np

from . import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def witness_bases(path=None):
    """The bench witness bases (dicts for _abi.pack_transfer_witnesses_tiled)."""
    bs = json.load(open(path or os.path.join(GOLDEN, "bench_transfers.json")))["transfers"]
    return [{"inputs": bytes.fromhex(t["inputs"]), "outputs": bytes.fromhex(t["outputs"]),
             "in_values": t["in_values"], "in_bfs": [int(x) for x in t["in_bfs"]],
             "out_values": t["out_values"], "out_bfs": [int(x) for x in t["out_bfs"]], "type": t["type"]}
            for t in bs]


def random_witness_bases(ctx, n, seed=1, ttype="ABC"):
    """n 2-in/2-out transfer witnesses for ctx's public parameters (any base
    and exponent, e.g. PP-B's 64-bit range): input values uniform in
    [1, max/2], outputs a random re-split of their sum, blinding factors
    uniform mod r, commitments computed on the device (ftz_commit_tokens =
    computeTokens, token/token.go:64-76).  Dicts as witness_bases()."""
    import random
    R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
    rng = random.Random(seed)
    vmax = ctx.base ** ctx.exponent - 1
    bases = []
    for _ in range(n):
        vin = [rng.randint(1, vmax // 2) for _ in range(2)]
        o1 = rng.randint(0, sum(vin))
        vout = [o1, sum(vin) - o1]
        bin_, bout = [rng.randrange(1, R) for _ in range(2)], [rng.randrange(1, R) for _ in range(2)]
        coms = ctx.commit_tokens([(ttype, v, b) for v, b in zip(vin + vout, bin_ + bout)])
        bases.append({"inputs": coms[0] + coms[1], "outputs": coms[2] + coms[3], "in_values": vin, "in_bfs": bin_,
                      "out_values": vout, "out_bfs": bout, "type": ttype})
    return bases


def seeds(n, tag=b"bench"):
    """n distinct 32-byte prover seeds"""
    out = bytearray(32 * n)
    for i in range(n):
        out[32 * i:32 * i + 32] = hashlib.sha256(tag + b"/%d" % i).digest()
    return bytes(out)


class TransferSet:
    """n transfers whose bytes live in buffers kept alive by this object;
    rows = packed ftz_transfer numpy array pointing into them; expect = the
    expected verdict code of each row."""

    def __init__(self, rows, expect, keep):
        self.rows = rows
        self.n = len(rows)
        self.expect = np.asarray(expect, dtype=np.int32)
        self._keep = keep

    @staticmethod
    def from_flat(inputs, in_off, outputs, out_off, proofs, proof_off, expect):
        ptr, n, keep = _abi.pack_transfers_flat(inputs, in_off, outputs, out_off, proofs, proof_off)
        return TransferSet(keep[0][:n], expect, keep)

    @staticmethod
    def from_items(items, expect):
        """items: (inputs, outputs, proof) byte triples"""
        def flat(parts):
            off = np.zeros(len(parts) + 1, dtype=np.int64)
            off[1:] = np.cumsum([len(p) for p in parts])
            return np.frombuffer(b"".join(parts) or b"\0", dtype=np.uint8), off
        ib, io = flat([t[0] for t in items])
        ob, oo = flat([t[1] for t in items])
        pb, po = flat([t[2] for t in items])
        return TransferSet.from_flat(ib, io, ob, oo, pb, po, expect)

    def proof(self, i):
        r = self.rows[i]
        return ctypes.string_at(int(r["proof"]), int(r["proof_len"]))

    def item(self, i):
        r = self.rows[i]
        return (ctypes.string_at(int(r["inputs"]), 64 * int(r["n_in"])),
                ctypes.string_at(int(r["outputs"]), 64 * int(r["n_out"])), self.proof(i))


class Job:
    """A verification job: a row selection over one or more TransferSets
    (which must stay alive as long as the job)."""

    def __init__(self, rows, expect, sets):
        self.rows = np.ascontiguousarray(rows)
        self.expect = np.asarray(expect, dtype=np.int32)
        self.n = len(self.rows)
        self._sets = sets

    def ptr(self, start=0):
        return ctypes.cast(self.rows.ctypes.data + start * self.rows.itemsize, ctypes.POINTER(_abi.Transfer))


def prove_distinct(ctx, n, tag=b"bench", bases=None):
    """n distinct valid 2-in/2-out transfer proofs made on the GPU (witness
    bases tiled, a fresh seed per proof).  Returns a TransferSet."""
    bases = bases or witness_bases()
    sel = np.arange(n) % len(bases)
    wptr, wn, wkeep = _abi.pack_transfer_witnesses_tiled(bases, sel, seeds(n, tag))
    # proof size grows with the range proof's digits (2 outputs x exponent membership proofs)
    blob, offs, codes = ctx.prove_packed("transfer", wptr, wn, bytes_per_proof=4096 + 4096 * ctx.exponent)
    if not (codes == 0).all():
        raise RuntimeError("prover rejected a bench witness")
    ins = np.frombuffer(b"".join(b["inputs"] for b in bases), dtype=np.uint8)
    outs = np.frombuffer(b"".join(b["outputs"] for b in bases), dtype=np.uint8)
    ia, ik = _abi.buffer_address(ins)
    oa, ok = _abi.buffer_address(outs)
    pa, pk = _abi.buffer_address(blob)
    rows = np.zeros(n, dtype=_abi.transfer_dtype())
    rows["inputs"] = ia + 128 * sel
    rows["n_in"] = 2
    rows["outputs"] = oa + 128 * sel
    rows["n_out"] = 2
    rows["proof"] = pa + offs[:-1]
    rows["proof_len"] = offs[1:] - offs[:-1]
    return TransferSet(rows, np.zeros(n, dtype=np.int32), [ik, ok, pk, blob])


def golden_tampered(pp_key="pp_a", shape=(2, 2)):
    """The golden corpus' rejected transfers of the given shape, with codes."""
    g = json.load(open(os.path.join(GOLDEN, "zkatdlog_golden.json")))[pp_key]
    items, codes = [], []
    for c in g["cases"]:
        if c["kind"] != "transfer" or c["expect"] == 0:
            continue
        if len(c["inputs"]) != 128 * shape[0] or len(c["outputs"]) != 128 * shape[1]:
            continue
        items.append((bytes.fromhex(c["inputs"]), bytes.fromhex(c["outputs"]), base64.b64decode(c["proof"])))
        codes.append(c["expect"])
    return TransferSet.from_items(items, codes)


def mixed_job(valid, bad, n, rate=1 / 64, seed=2024, offset=0):
    """A job of n rows: row i is valid[(offset + i) % valid.n] except a
    pseudo-random ~rate of rows, which are tampered corpus cases."""
    rng = np.random.default_rng(seed)
    idx = (offset + np.arange(n)) % valid.n
    rows = valid.rows[idx].copy()
    expect = valid.expect[idx].copy()
    if bad is not None and bad.n and rate > 0:
        pick = rng.random(n) < rate
        which = rng.integers(0, bad.n, size=n)
        rows[pick] = bad.rows[which[pick]]
        expect[pick] = bad.expect[which[pick]]
    return Job(rows, expect, [valid, bad])


# ---------------------------------------------------------------- raw token requests
# asn1.Marshal(driver.TokenRequest) (token/driver/request.go:24-38) of transfer
# actions json.Marshal(transfer.TransferAction) (crypto/transfer/sender.go:105-116:
# Inputs, InputCommitments, OutputTokens, Proof, Metadata) whose G1 fields are
# mathlib's curveElement JSON {"curve":1,"element":base64(RawBytes)}; ledger
# values json.Marshal(token.Token{Owner, Data}) (crypto/token/token.go:20-25).
BENCH_OWNER = base64.b64encode(b"owner-identity").decode()


def _der_len(n):
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def _der(tag, body):
    return bytes([tag]) + _der_len(len(body)) + body


def _elem(raw):
    return '{"curve":1,"element":"%s"}' % base64.b64encode(raw).decode()


def token_json(raw):
    return ('{"Owner":"%s","Data":%s}' % (BENCH_OWNER, _elem(raw))).encode()


def transfer_action_json(keys, ins, outs, proof):
    """json(TransferAction) with 64-byte RawBytes input / output commitments"""
    return ('{"Inputs":[%s],"InputCommitments":[%s],"OutputTokens":[%s],"Proof":"%s","Metadata":null}' % (
        ",".join('"%s"' % k for k in keys),
        ",".join(_elem(ins[64 * i:64 * i + 64]) for i in range(len(ins) // 64)),
        ",".join('{"Owner":"%s","Data":%s}' % (BENCH_OWNER, _elem(outs[64 * i:64 * i + 64]))
                 for i in range(len(outs) // 64)),
        base64.b64encode(proof).decode())).encode()


def token_request(transfers, issues=(), sigs=(), auditor_sigs=()):
    """asn1.Marshal(TokenRequest{Issues, Transfers, Signatures, AuditorSignatures})"""
    def seq_of(items):
        return _der(0x30, b"".join(_der(0x04, x) for x in items))
    return _der(0x30, seq_of(issues) + seq_of(transfers) + seq_of(sigs) + seq_of(auditor_sigs))


class RequestSet:
    """n raw token requests of `per` transfer actions each (GPU-made proofs of a
    TransferSet, tiled), flat in one buffer, with the ledger holding their
    inputs.  Every `missing_every`-th request's last action spends a key that is
    not on the ledger (FTZ_ERR_INPUT at that action); all other requests verify.
    rows = a packed ftz_bytes numpy array pointing into the buffer."""

    def __init__(self, valid, n, per=2, missing_every=97, tag="blk"):
        parts, ledger, off = [], {}, [0]
        self.expect = np.zeros(n, dtype=np.int32)
        self.failed = np.full(n, -1, dtype=np.int32)
        sig = [b"\x30" * 72] * per  # signatures travel in the request; verified in Go
        cache = {}  # distinct proof -> (its action JSON after the Inputs list, ledger token JSONs)

        def tail(j):
            if j not in cache:
                ins, outs, proof = valid.item(j)
                act = transfer_action_json([], ins, outs, proof)
                cache[j] = (act[len(b'{"Inputs":[]'):], [token_json(ins[64 * i:64 * i + 64])
                                                         for i in range(len(ins) // 64)])
            return cache[j]
        for r in range(n):
            acts = []
            for a in range(per):
                rest, toks = tail((r * per + a) % valid.n)
                keys = ["%s%07d:%d:%d" % (tag, r, a, i) for i in range(len(toks))]
                missing = missing_every and r % missing_every == missing_every - 1 and a == per - 1
                for i, k in enumerate(keys):
                    if not (missing and i == 0):
                        ledger[k] = toks[i]
                acts.append(b'{"Inputs":[' + ",".join('"%s"' % k for k in keys).encode() + b"]" + rest)
                if missing:
                    self.expect[r] = _abi.FTZ_ERR_INPUT
                    self.failed[r] = a
            raw = token_request(acts, sigs=sig)
            parts.append(raw)
            off.append(off[-1] + len(raw))
        self.buf = np.frombuffer(b"".join(parts), dtype=np.uint8)
        self.off = np.asarray(off, dtype=np.int64)
        self.n, self.per, self.ledger = n, per, ledger
        addr, self._keep = _abi.buffer_address(self.buf)
        self.rows = np.zeros(n, dtype=[("p", np.uint64), ("len", np.uint64)])
        self.rows["p"] = addr + self.off[:-1]
        self.rows["len"] = self.off[1:] - self.off[:-1]

    def ptr(self):
        return ctypes.cast(self.rows.ctypes.data, ctypes.POINTER(_abi.Bytes))

    def nbytes(self):
        return int(self.off[-1])

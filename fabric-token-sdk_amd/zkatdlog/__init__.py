"""zkatdlog -- MI355X batch verifier for the Fabric Token SDK zkatdlog (nogh) driver.

Host-side mirror of the reference's verifier interfaces (Go, paths relative to
/root/reference/token/core/zkatdlog/crypto/):

    transfer.NewVerifier(inputs, outputs, pp).Verify(proof)   transfer/transfer.go:66,124
    issue.NewVerifier(tokens, anonymous, pp).Verify(proof)    issue/issue.go:194,202
    validator TransferZKProofValidate(ctx)                    validator/validator_transfer.go:84-98

backed by libftsamd.so (include/ftsamd.h): every proof is parsed on the host
and verified by HIP kernels on the GPU.  There is no CPU fallback: without
the library or without an MI355X the constructors raise.

Batch form (the point of the port):

    ctx = Context(pp_bytes, device=0)
    codes = ctx.verify_transfers([(inputs64, outputs64, proof), ...])   # 0 = accept
"""
import ctypes

from . import _abi
from ._abi import (FTZ_ERR_MALFORMED, FTZ_ERR_MEMBERSHIP, FTZ_ERR_OPENING, FTZ_ERR_PANIC,  # noqa: F401
                   FTZ_ERR_PARSE, FTZ_ERR_RANGE, FTZ_ERR_WF, FTZ_OK, KERNEL_NAMES, MESSAGES)

__all__ = ["Context", "Batch", "Msm", "Prover", "ZKError", "Idemix", "OwnerVerifier", "TransferVerifier", "IssueVerifier", "transfer_zkproof_validate",
           "FTZ_OK", "MESSAGES"]


class ZKError(Exception):
    """A rejected proof; ``code`` is the FTZ_ERR_* class, the message carries
    the reference's error text for that class."""

    def __init__(self, code):
        super().__init__(MESSAGES.get(code, "verification failed (%d)" % code))
        self.code = code


class DeviceError(RuntimeError):
    pass


def _check(rc, lib):
    if rc != 0:
        raise DeviceError("ftsamd error %d: %s" % (rc, lib.ftz_last_error().decode(errors="replace")))


class Context:
    """Public parameters resident on one GPU (crypto.PublicParams + the
    fixed-base tables / Miller lines the kernels use).  The reference builds
    its validator once per process (token/services/network/fabric/tcc/tcc.go:170-182);
    so does this."""

    def __init__(self, pp_bytes, device=0, threads=None, fexp="exact", batch=None, slots=None, window_us=None,
                 **options):
        """fexp: "exact" (FTZ_FEXP_EXACT, gnark-crypto v0.6.0) or "fuentes";
        batch / slots / window_us / threads and any other ftz_options field by name
        (hold_inflight, small_pass, msm_window_bits, msm_slot_cap, msm_seg_slots,
        msm_glv, msm_precompute): job-engine and MSM options."""
        self._lib = _abi.load()
        self.device = int(device)
        h = ctypes.c_void_p()
        pp_bytes = bytes(pp_bytes)
        o = _abi.Options()
        self._lib.ftz_options_default(ctypes.byref(o))
        o.fexp = _abi.FEXP[fexp]
        names = {k for k, _ in _abi.Options._fields_[1:]} - {"fexp"}
        unknown = set(options) - names
        if unknown:
            raise TypeError("unknown ftz_options field(s): %s" % ", ".join(sorted(unknown)))
        options.update(batch=batch, slots=slots, window_us=window_us, threads=threads)
        for k, v in options.items():
            if v is not None:
                setattr(o, k, int(v))
        _check(self._lib.ftz_ctx_create_ex(pp_bytes, len(pp_bytes), int(device), ctypes.byref(o), ctypes.byref(h)),
               self._lib)
        self._h = h
        _check(self._lib.ftz_ctx_options(h, ctypes.byref(o)), self._lib)
        self.options = {k: getattr(o, k) for k, _ in _abi.Options._fields_[1:]}
        b, e = ctypes.c_uint32(), ctypes.c_uint32()
        _check(self._lib.ftz_ctx_info(h, ctypes.byref(b), ctypes.byref(e)), self._lib)
        self.base, self.exponent = b.value, e.value

    def close(self):
        if getattr(self, "_h", None):
            self._lib.ftz_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def verify_transfers(self, transfers):
        """transfers: iterable of (inputs, outputs, proof) with inputs/outputs the
        concatenated 64-byte G1 RawBytes commitments.  Returns a list of codes."""
        arr, keep = _abi.pack_transfers(transfers)
        n = len(keep) // 3
        codes = (ctypes.c_int32 * max(1, n))()
        _check(self._lib.ftz_verify_transfers(self._h, n, arr, codes), self._lib)
        return list(codes)[:n]

    def verify_transfers_flat(self, inputs, in_off, outputs, out_off, proofs, proof_off):
        """Zero-copy verification of n transfers held in flat buffers (see
        _abi.pack_transfers_flat); returns a numpy int32 array of codes."""
        import numpy as np
        ptr, n, keep = _abi.pack_transfers_flat(inputs, in_off, outputs, out_off, proofs, proof_off)
        codes = np.zeros(max(1, n), dtype=np.int32)
        _check(self._lib.ftz_verify_transfers(self._h, n, ptr,
                                              codes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))), self._lib)
        del keep
        return codes[:n]

    def verify_issues_flat(self, outputs, out_off, proofs, proof_off, anonymous):
        import numpy as np
        ptr, n, keep = _abi.pack_issues_flat(outputs, out_off, proofs, proof_off, anonymous)
        codes = np.zeros(max(1, n), dtype=np.int32)
        _check(self._lib.ftz_verify_issues(self._h, n, ptr,
                                           codes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))), self._lib)
        del keep
        return codes[:n]

    def verify_transfers_packed(self, ptr, n):
        """Verify an already packed ftz_transfer array (e.g. a numpy selection
        of _abi.pack_transfers_flat rows); returns numpy int32 codes."""
        import numpy as np
        codes = np.zeros(max(1, n), dtype=np.int32)
        _check(self._lib.ftz_verify_transfers(self._h, n, ptr,
                                              codes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))), self._lib)
        return codes[:n]

    def prove_packed(self, kind, ptr, n, bytes_per_proof=12288):
        """One-shot ftz_prove_transfers / ftz_prove_issues on a packed witness
        array (_abi.pack_*_witnesses_tiled).  Returns (proof blob as a numpy
        uint8 array, offsets int64[n + 1], codes int32[n])."""
        import numpy as np
        fn = self._lib.ftz_prove_transfers if kind == "transfer" else self._lib.ftz_prove_issues
        cap = max(1, n * bytes_per_proof)
        buf = np.empty(cap, dtype=np.uint8)
        offs = np.zeros(n + 1, dtype=np.uint64)
        codes = np.zeros(max(1, n), dtype=np.int32)
        _check(fn(self._h, n, ptr, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), cap,
                  offs.ctypes.data_as(ctypes.POINTER(ctypes.c_size_t)),
                  codes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))), self._lib)
        return buf[:int(offs[n])], offs.astype(np.int64), codes[:n]

    def engine_stats(self, reset=False):
        """job-engine counters (ftz_ctx_engine_stats)"""
        st = _abi.EngineStats()
        _check(self._lib.ftz_ctx_engine_stats(self._h, ctypes.byref(st), 1 if reset else 0), self._lib)
        return {k: getattr(st, k) for k, _ in _abi.EngineStats._fields_}

    def prover_stats(self, reset=False):
        """host-side time of ftz_prove_* (ftz_ctx_prover_stats): wait / copy / plan / submit"""
        st = _abi.ProverHostStats()
        _check(self._lib.ftz_ctx_prover_stats(self._h, ctypes.byref(st), 1 if reset else 0), self._lib)
        return {k: getattr(st, k) for k, _ in _abi.ProverHostStats._fields_}

    def set_serial(self, serial):
        """profiling: every kernel of a batch on one stream (ftz_ctx_set_serial)"""
        _check(self._lib.ftz_ctx_set_serial(self._h, 1 if serial else 0), self._lib)

    LAYOUTS = {"one_lane": 1, "sextet": 6}
    STAGES = {"g2lines": 0, "prover_g2lines": 1}

    def set_debug(self, challenges=False):
        """ftz_ctx_set_debug: keep every recomputed challenge of batches loaded
        afterwards (Batch.challenges); set before planning on the context"""
        _check(self._lib.ftz_ctx_set_debug(self._h, _abi.FTZ_DEBUG_CHALLENGES if challenges else 0), self._lib)

    def set_layout(self, stage, layout):
        """profiling: kernel layout of a pipeline stage (ftz_ctx_set_layout); stage 'g2lines'
        (verifier, default 'one_lane') or 'prover_g2lines' (default 'one_lane'), layout 'one_lane'
        or 'sextet' -- same results, different speed"""
        _check(self._lib.ftz_ctx_set_layout(self._h, self.STAGES[stage], self.LAYOUTS[layout]), self._lib)

    def verify_issues(self, issues):
        """issues: iterable of (outputs, proof, anonymous)."""
        arr, keep = _abi.pack_issues(issues)
        n = len(keep) // 2
        codes = (ctypes.c_int32 * max(1, n))()
        _check(self._lib.ftz_verify_issues(self._h, n, arr, codes), self._lib)
        return list(codes)[:n]

    def prove_transfers(self, witnesses):
        """Proof bytes for each witness (see Prover); raises ZKError-free
        DeviceError on bad arguments (e.g. a value outside the range)."""
        p = Prover(self, list(witnesses), "transfer")
        try:
            p.run()
            return p.proofs()
        finally:
            p.close()

    def prove_issues(self, witnesses):
        p = Prover(self, list(witnesses), "issue")
        try:
            p.run()
            return p.proofs()
        finally:
            p.close()

    def commit_tokens(self, openings):
        """token commitments H(type)*Ped0 + v*Ped1 + bf*Ped2 (computeTokens,
        token/token.go:64-76) for (type, value, bf) openings: 64-byte RawBytes each."""
        openings = list(openings)
        arr, keep = _abi.pack_openings(openings)
        n = len(openings)
        out = (ctypes.c_uint8 * max(1, 64 * n))()
        _check(self._lib.ftz_commit_tokens(self._h, n, arr, out), self._lib)
        raw = bytes(out)
        return [raw[64 * i:64 * i + 64] for i in range(n)]

    def audit_openings(self, commitments, openings):
        """auditor opening check (audit/auditor.go:208-234): codes, 0 = match,
        FTZ_ERR_OPENING = mismatch, FTZ_ERR_PARSE = invalid commitment bytes."""
        openings = list(openings)
        arr, keep = _abi.pack_openings(openings)
        n = len(openings)
        coms = b"".join(bytes(c) for c in commitments)
        if len(coms) != 64 * n:
            raise ValueError("one 64-byte commitment per opening")
        codes = (ctypes.c_int32 * max(1, n))()
        _check(self._lib.ftz_audit_openings(self._h, n, coms, arr, codes), self._lib)
        return list(codes)[:n]

    def msm_g1(self, points, scalars):
        """sum_i k_i P_i (gnark G1Jac.MultiExp semantics): points n x 64-byte
        RawBytes, scalars n x 32 bytes big-endian.  Returns 64-byte RawBytes."""
        m = Msm(self, points, scalars)
        try:
            return m.run()
        finally:
            m.close()

    def verify_token_requests(self, requests, ledger, batched=False):
        """Raw token requests (asn1 TokenRequest bytes) validated as
        Validator.VerifyTokenRequestFromRaw does minus the Go-side signature /
        HTLC / metadata checks; ledger: dict key -> token.Token JSON bytes (or a
        callable), or a NativeLedger.  batched: the one-callback-per-chunk
        lookup (ftz_verify_token_requests_batched).  Returns (codes,
        failed_action) lists."""
        arr, keep = _abi.pack_bytes(requests)
        n = len(keep)
        codes = (ctypes.c_int32 * max(1, n))()
        failed = (ctypes.c_int32 * max(1, n))()
        self.verify_token_requests_packed(arr, n, ledger, codes, failed, batched=batched)
        return list(codes)[:n], list(failed)[:n]

    def request_stats(self, reset=False):
        """calling-thread ms per request-pipeline stage (ftz_ctx_request_stats)"""
        ms = (ctypes.c_double * 6)()
        _check(self._lib.ftz_ctx_request_stats(self._h, ms, 1 if reset else 0), self._lib)
        return dict(zip(("decode", "check", "lookup", "tokens", "build", "drain"), (round(x, 2) for x in ms)))

    def verify_token_requests_packed(self, arr, n, ledger, codes, failed, batched=False):
        """as verify_token_requests over a packed ftz_bytes array and caller-owned
        int32 code arrays (bench: the packing stays out of the timed call)"""
        if isinstance(ledger, NativeLedger):
            fn, user = ledger.fn(batched), ledger.handle
            keep_cb = None
        else:
            keep_cb = (_abi.get_states_callback if batched else _abi.get_state_callback)(ledger)
            fn, user = ctypes.cast(keep_cb, ctypes.c_void_p), None
        call = self._lib.ftz_verify_token_requests_batched if batched else self._lib.ftz_verify_token_requests
        _check(call(self._h, n, arr, fn, user, codes, failed), self._lib)
        del keep_cb

    def g1_sum(self, points):
        """Sum of RawBytes G1 points (n x 64 bytes, the identity = 64 zero
        bytes) on the device: the final add of a point-split MSM."""
        points = bytes(points)
        if len(points) % 64:
            raise ValueError("points must be n x 64 bytes")
        out = (ctypes.c_uint8 * 64)()
        _check(self._lib.ftz_g1_sum(self._h, len(points) // 64, points, out), self._lib)
        return bytes(out)

    def load_transfers(self, transfers):
        arr, keep = _abi.pack_transfers(transfers)
        n = len(keep) // 3
        h = ctypes.c_void_p()
        _check(self._lib.ftz_batch_load_transfers(self._h, n, arr, ctypes.byref(h)), self._lib)
        return Batch(self, h, n)

    def load_packed(self, ptr, n):
        """Staged batch (ftz_batch_load_transfers) of an already packed
        ftz_transfer array."""
        h = ctypes.c_void_p()
        _check(self._lib.ftz_batch_load_transfers(self._h, n, ptr, ctypes.byref(h)), self._lib)
        return Batch(self, h, n)

    def load_issues(self, issues):
        arr, keep = _abi.pack_issues(issues)
        n = len(keep) // 2
        h = ctypes.c_void_p()
        _check(self._lib.ftz_batch_load_issues(self._h, n, arr, ctypes.byref(h)), self._lib)
        return Batch(self, h, n)


def decode_token_request(raw):
    """driver.TokenRequest.FromBytes (Go encoding/asn1; host-side, no GPU):
    [issues, transfers, signatures, auditor_signatures] or ValueError."""
    lib = _abi.load()
    raw = bytes(raw)
    counts = (ctypes.c_size_t * 4)()
    cap = max(1, len(raw) // 2)
    elems = (_abi.Bytes * cap)()
    if lib.ftz_token_request_decode(raw, len(raw), counts, elems, cap) != 0:
        raise ValueError(lib.ftz_last_error().decode(errors="replace"))
    out, k = [], 0
    for f in range(4):
        items = []
        for _ in range(counts[f]):
            e = elems[k]
            k += 1
            items.append(ctypes.string_at(e.p, e.len) if e.len else b"")
        out.append(items)
    return out


def setup_public_params(base, exponent, seed, idemix_pk=b"idemix-issuer-pk", idemix_curve=0):
    """crypto.Setup(base, exponent, nymPK, idemixCurveID) (setup.go:214-236) +
    Serialize, with seed-derived randomness (ftz_pp_setup): the serialized PP bytes."""
    lib = _abi.load()
    n = ctypes.c_size_t()
    seed = bytes(seed)
    pk = None if idemix_pk is None else bytes(idemix_pk)
    args = (int(base), int(exponent), pk, 0 if pk is None else len(pk), int(idemix_curve), seed, len(seed))
    lib.ftz_pp_setup(*args, None, 0, ctypes.byref(n))
    buf = ctypes.create_string_buffer(n.value)
    _check(lib.ftz_pp_setup(*args, buf, n.value, ctypes.byref(n)), lib)
    return buf.raw[:n.value]


def validate_public_params(pp_bytes):
    """crypto.PublicParams.Validate (setup.go:238-273): "" or the error text
    (host-side check; no GPU needed)."""
    lib = _abi.load()
    pp_bytes = bytes(pp_bytes)
    rc = lib.ftz_pp_validate(pp_bytes, len(pp_bytes))
    return "" if rc == 0 else lib.ftz_last_error().decode(errors="replace")


class Msm:
    """A device-resident G1 multi-scalar multiplication (BASELINE configs[2]):
    run() returns sum_i k_i P_i as 64-byte gnark RawBytes."""

    def __init__(self, ctx, points=None, scalars=b"", n=None, gen_offset=None):
        self._ctx, self._lib, self._h = ctx, ctx._lib, None
        scalars = bytes(scalars)
        h = ctypes.c_void_p()
        if gen_offset is not None:
            self.n = len(scalars) // 32
            _check(self._lib.ftz_msm_load_gen(ctx._h, self.n, int(gen_offset), scalars, ctypes.byref(h)), self._lib)
        else:
            points = bytes(points)
            if len(points) % 64 or len(points) // 64 != len(scalars) // 32 or len(scalars) % 32:
                raise ValueError("points must be n x 64 bytes and scalars n x 32 bytes")
            self.n = len(points) // 64
            _check(self._lib.ftz_msm_load(ctx._h, self.n, points, scalars, ctypes.byref(h)), self._lib)
        self._h = h

    def set_scalars(self, scalars):
        """new scalars (n x 32 bytes) for the resident points"""
        scalars = bytes(scalars)
        if len(scalars) != 32 * self.n:
            raise ValueError("scalars must be n x 32 bytes")
        _check(self._lib.ftz_msm_set_scalars(self._h, scalars), self._lib)

    def run(self):
        out = (ctypes.c_uint8 * 64)()
        _check(self._lib.ftz_msm_run(self._h, out), self._lib)
        return bytes(out)

    def run_scalars(self, scalars):
        """set the scalars and run in one call (ftz_msm_run_scalars): scalars is
        n x 32 bytes (bytes, or a HostBuffer for page-locked memory)"""
        if isinstance(scalars, HostBuffer):
            if scalars.size < 32 * self.n:
                raise ValueError("scalars must be n x 32 bytes")
            ptr, keep = scalars.ptr, None
        else:
            keep = bytes(scalars)
            if len(keep) != 32 * self.n:
                raise ValueError("scalars must be n x 32 bytes")
            ptr = ctypes.cast(ctypes.c_char_p(keep), ctypes.c_void_p)
        out = (ctypes.c_uint8 * 64)()
        _check(self._lib.ftz_msm_run_scalars(self._h, ptr, out), self._lib)
        return bytes(out)

    def info(self):
        ms, c = ctypes.c_float(), ctypes.c_uint32()
        _check(self._lib.ftz_msm_info(self._h, ctypes.byref(ms), ctypes.byref(c)), self._lib)
        return {"last_ms": ms.value, "window_bits": c.value}

    def close(self):
        if getattr(self, "_h", None):
            self._lib.ftz_msm_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


class HostBuffer:
    """Page-locked host memory (ftz_host_alloc): inputs staged here copy to the
    device at the full link rate."""

    def __init__(self, ctx, size):
        self._lib, self.size, self.ptr = ctx._lib, int(size), ctypes.c_void_p()
        _check(self._lib.ftz_host_alloc(self.size, ctypes.byref(self.ptr)), self._lib)

    def write(self, data, offset=0):
        data = bytes(data)
        if offset + len(data) > self.size:
            raise ValueError("write past the end of the buffer")
        ctypes.memmove(self.ptr.value + offset, data, len(data))

    def close(self):
        if getattr(self, "ptr", None) is not None and self.ptr.value:
            self._lib.ftz_host_free(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Prover:
    """Device-resident batch prover (transfer.NewProver(...).Prove(),
    transfer/transfer.go:89-121; issue.NewProver(...).Prove(), issue/issue.go:162-184).
    witnesses: dicts as in _abi.pack_transfer_witnesses / pack_issue_witnesses."""

    def __init__(self, ctx, witnesses, kind="transfer"):
        self._ctx, self._lib, self._h = ctx, ctx._lib, None
        pack = _abi.pack_transfer_witnesses if kind == "transfer" else _abi.pack_issue_witnesses
        load = self._lib.ftz_prover_load_transfers if kind == "transfer" else self._lib.ftz_prover_load_issues
        arr, keep = pack(witnesses)
        self.n = len(list(witnesses)) if not isinstance(witnesses, list) else len(witnesses)
        h = ctypes.c_void_p()
        _check(load(ctx._h, self.n, arr, ctypes.byref(h)), self._lib)
        self._h = h

    def run(self):
        _check(self._lib.ftz_prover_run(self._h), self._lib)

    def submit(self):
        _check(self._lib.ftz_prover_submit(self._h), self._lib)

    def wait(self):
        _check(self._lib.ftz_prover_wait(self._h), self._lib)

    def proofs(self):
        """(list of proof bytes, list of codes)"""
        size = self._lib.ftz_prover_bytes(self._h)
        buf = (ctypes.c_uint8 * max(1, size))()
        offs = (ctypes.c_size_t * (self.n + 1))()
        codes = (ctypes.c_int32 * max(1, self.n))()
        _check(self._lib.ftz_prover_proofs(self._h, buf, size, offs, codes), self._lib)
        raw = bytes(buf)[:size]
        return [raw[offs[i]:offs[i + 1]] for i in range(self.n)], list(codes)[:self.n]

    def stats(self):
        s = _abi.Stats()
        _check(self._lib.ftz_prover_stats(self._h, ctypes.byref(s)), self._lib)
        return {name: (s.ms[k], s.jobs[k]) for k, name in enumerate(_abi.PROVER_STAGE_NAMES)}

    def close(self):
        if getattr(self, "_h", None):
            self._lib.ftz_prover_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


class Batch:
    """A planned, device-resident batch: run() re-executes the GPU pipeline."""

    def __init__(self, ctx, h, n):
        self._ctx, self._lib, self._h, self.n = ctx, ctx._lib, h, n

    def run(self):
        _check(self._lib.ftz_batch_run(self._h), self._lib)

    def submit(self):
        """Enqueue the pipeline on the batch's own streams and return (ftz_batch_submit)."""
        _check(self._lib.ftz_batch_submit(self._h), self._lib)

    def wait(self):
        """Block until the last submission finished (ftz_batch_wait)."""
        _check(self._lib.ftz_batch_wait(self._h), self._lib)

    def challenges(self, i, cap=256):
        """[(class code, 32-byte HashToZr)] recomputed for proof i (a batch
        loaded after Context.set_debug(challenges=True); ftz_batch_challenges)"""
        kinds = (ctypes.c_int32 * cap)()
        vals = ctypes.create_string_buffer(32 * cap)
        cnt = ctypes.c_size_t()
        _check(self._lib.ftz_batch_challenges(self._h, i, kinds, vals, cap, ctypes.byref(cnt)), self._lib)
        if cnt.value > cap:
            return self.challenges(i, cnt.value)
        return [(kinds[k], vals.raw[32 * k:32 * k + 32]) for k in range(cnt.value)]

    def codes(self):
        c = (ctypes.c_int32 * max(1, self.n))()
        _check(self._lib.ftz_batch_codes(self._h, c), self._lib)
        return list(c)[:self.n]

    def bitmap(self):
        b = (ctypes.c_uint8 * max(1, (self.n + 7) // 8))()
        _check(self._lib.ftz_batch_bitmap(self._h, b), self._lib)
        return bytes(b)[:(self.n + 7) // 8]

    def stats(self):
        s = _abi.Stats()
        _check(self._lib.ftz_batch_stats(self._h, ctypes.byref(s)), self._lib)
        return {name: (s.ms[k], s.jobs[k]) for k, name in enumerate(KERNEL_NAMES)}

    def close(self):
        if self._h:
            self._lib.ftz_batch_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


def _commitments(xs):
    """A list of 64-byte G1 RawBytes, or their concatenation."""
    if isinstance(xs, (bytes, bytearray, memoryview)):
        b = bytes(xs)
    else:
        b = b"".join(bytes(x) for x in xs)
    if len(b) % 64:
        raise ValueError("commitments must be 64-byte G1 RawBytes")
    return b


class TransferVerifier:
    """transfer.NewVerifier(inputs, outputs, pp) (transfer/transfer.go:66-77)."""

    def __init__(self, inputs, outputs, ctx):
        self.inputs = _commitments(inputs)
        self.outputs = _commitments(outputs)
        self.ctx = ctx

    def verify(self, proof):
        """transfer.Verifier.Verify (transfer/transfer.go:124-154): raises ZKError."""
        code = self.ctx.verify_transfers([(self.inputs, self.outputs, bytes(proof))])[0]
        if code != FTZ_OK:
            raise ZKError(code)


class IssueVerifier:
    """issue.NewVerifier(tokens, anonymous, pp) (issue/issue.go:194-199)."""

    def __init__(self, tokens, anonymous, ctx):
        self.tokens = _commitments(tokens)
        self.anonymous = bool(anonymous)
        self.ctx = ctx

    def verify(self, proof):
        code = self.ctx.verify_issues([(self.tokens, bytes(proof), self.anonymous)])[0]
        if code != FTZ_OK:
            raise ZKError(code)


def transfer_zkproof_validate(ctx, input_commitments, output_commitments, proof):
    """validator.TransferZKProofValidate (validator/validator_transfer.go:84-98):
    inputs are the commitments of the ledger tokens, not the action's own
    InputCommitments."""
    TransferVerifier(input_commitments, output_commitments, ctx).verify(proof)


class NativeLedger:
    """A ledger snapshot served by native callbacks (tools/callers.cpp
    ftz_ledger_*): key -> json(token.Token), looked up without Python in the
    call -- what a committer's state database hands the library."""

    def __init__(self, items):
        import os
        lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libftscallers.so"))
        lib.ftz_ledger_create.restype = ctypes.c_void_p
        lib.ftz_ledger_create.argtypes = [ctypes.c_size_t, ctypes.POINTER(_abi.Bytes), ctypes.POINTER(_abi.Bytes)]
        lib.ftz_ledger_destroy.argtypes = [ctypes.c_void_p]
        lib.ftz_ledger_counts.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                          ctypes.POINTER(ctypes.c_uint64)]
        items = list(items.items()) if isinstance(items, dict) else list(items)
        ks, kk = _abi.pack_bytes([k.encode() if isinstance(k, str) else k for k, _ in items])
        vs, vk = _abi.pack_bytes([v for _, v in items])
        self._lib = lib
        self.handle = lib.ftz_ledger_create(len(items), ks, vs)

    def fn(self, batched):
        return ctypes.cast(self._lib.ftz_ledger_get_states if batched else self._lib.ftz_ledger_get_state,
                           ctypes.c_void_p)

    def counts(self):
        """(callback calls, keys looked up) so far"""
        c, k = ctypes.c_uint64(), ctypes.c_uint64()
        self._lib.ftz_ledger_counts(self.handle, ctypes.byref(c), ctypes.byref(k))
        return c.value, k.value

    def close(self):
        if self.handle:
            self._lib.ftz_ledger_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Idemix:
    """Idemix owner-signature verification: the deserializer
    built from PublicParams.IdemixIssuerPK / IdemixCurveID
    (zkatdlog/nogh/deserializer.go:45-61, identity/msp/idemix/deserializer.go:33-75)
    with its Verify path on the GPU.  curve_id = FTZ_CURVE_BN254 (the curve
    cmd/pp/dlog/gen.go:117 and the NWO topologies deploy, gurvy translator) or
    FTZ_CURVE_FP256BN_AMCL (amcl translator, the reference's unit-test keys)."""

    def __init__(self, ctx, ipk, curve_id=_abi.FTZ_CURVE_FP256BN_AMCL):
        self.ctx = ctx
        self._lib = ctx._lib
        h = ctypes.c_void_p()
        _check(self._lib.ftz_idemix_create(ctx._h, bytes(ipk), len(ipk), curve_id, ctypes.byref(h)), self._lib)
        self._h = h

    def verify_owner_signatures(self, items):
        """items: (owner, msg, sig) -> FTZ codes (0 = the signature verifies)"""
        arr, keep = _abi.pack_owner_sigs(items)
        codes = (ctypes.c_int32 * max(len(items), 1))()
        _check(self._lib.ftz_verify_owner_signatures(self._h, len(items), arr, codes), self._lib)
        return list(codes[:len(items)])

    def set_strict_nym(self, on=True):
        """opt-in: off-curve nyms are FTZ_ERR_OWNER instead of amcl's point at
        infinity (ftz_idemix_set_strict_nym; a deliberate deviation, parity unpinned)"""
        _check(self._lib.ftz_idemix_set_strict_nym(self._h, 1 if on else 0), self._lib)

    def verify_owner_signatures_packed(self, arr, n):
        """pre-packed ftz_owner_sig array (bench: the binding's packing stays out of the timed call)"""
        codes = (ctypes.c_int32 * max(n, 1))()
        _check(self._lib.ftz_verify_owner_signatures(self._h, n, arr, codes), self._lib)
        return list(codes[:n])

    def audit_owners(self, items):
        """auditor owner inspection (InspectTokenOwner, crypto/audit/auditor.go:252-274):
        items (token Owner bytes, OwnerInfo = json(AuditInfo)) -> FTZ codes (0 = the owner
        matches its audit info; FTZ_ERR_AUDIT = Match failed)"""
        items = list(items)
        arr, keep = _abi.pack_owner_audits(items)
        codes = (ctypes.c_int32 * max(len(items), 1))()
        _check(self._lib.ftz_audit_owners(self._h, len(items), arr, codes), self._lib)
        return list(codes[:len(items)])

    def owner_verifier(self, owner):
        """GetOwnerVerifier(tok.Owner) (validator_transfer.go:66)"""
        return OwnerVerifier(self, owner)

    def close(self):
        if self._h:
            self._lib.ftz_idemix_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class OwnerVerifier:
    """driver.Verifier of an owner identity (identity/msp/idemix/deserializer.go:153-163)."""

    def __init__(self, ix, owner):
        self.ix = ix
        self.owner = bytes(owner)

    def verify(self, message, sigma):
        """Verifier.Verify(message, sigma): raises ZKError on a reject."""
        code = self.ix.verify_owner_signatures([(self.owner, bytes(message), bytes(sigma))])[0]
        if code != FTZ_OK:
            raise ZKError(code)


class SignatureError(Exception):
    """An owner-signature check failed: the text is the reference's
    (validator_transfer.go:50-76) error chain, outermost first."""


PSEUDONYM_INVALID = "pseudonym signature invalid: zero-knowledge proof is invalid"  # IBM/idemix NymSignature.Ver


def _unique_id(owner):
    # view.Identity.UniqueID (fabric-smart-client, not vendored [EXT]): the hex
    # SHA-256 of the identity bytes
    import hashlib
    return hashlib.sha256(bytes(owner)).hexdigest()


def transfer_signature_validate(keys, load, owner_verifier, has_been_signed_by, verify_batch, unique_id=_unique_id):
    """validator.TransferSignatureValidate (crypto/validator/validator_transfer.go:42-82)
    with the owners' signatures verified in ONE batch (the Go shim's
    go/gpu/owner.go transferSignatures, same order and texts):

    * load(key) -> token owner bytes (raises with the reference's ledger texts);
    * owner_verifier(owner) -> a verifier (the Go deserializer; raises on a bad owner);
    * has_been_signed_by(owner, verifier) -> sigma (the provider's cursor; calls
      verifier.verify(msg, sigma), raises "invalid state, insufficient number of signatures");
    * verify_batch([(owner, msg, sigma)]) -> FTZ codes (Idemix.verify_owner_signatures).

    The reference verifies input i's signature before it loads input i+1, so
    when a step of input j fails, the signatures of inputs 0..j-1 are checked
    first and the first bad one wins.  Returns [(owner, sigma)] or raises
    SignatureError with the reference's text."""

    class _Capture:
        msg = sigma = None

        def verify(self, message, sigma):
            self.msg, self.sigma = bytes(message), bytes(sigma)

    done = []  # (key, owner, go verifier, msg, sigma)

    def check():
        if not done:
            return None
        codes = verify_batch([(o, m, s) for _, o, _, m, s in done])
        for i, (c, (key, owner, v, m, s)) in enumerate(zip(codes, done)):
            err = None
            if c in (_abi.FTZ_ERR_UNSUPPORTED, _abi.FTZ_ERR_OWNER):
                try:  # owners the library does not verify: the Go verifier decides
                    v.verify(m, s)
                except Exception as e:  # noqa: BLE001 -- the verifier's own error text
                    err = str(e)
            elif c != FTZ_OK:
                err = PSEUDONYM_INVALID
            if err is not None:
                return "failed signature verification [%d][%s][%s]: %s" % (i, key, unique_id(owner), err)
        return None

    def fail(text):
        raise SignatureError(check() or text)

    for i, key in enumerate(keys):
        try:
            owner = bytes(load(key))
        except Exception as e:  # noqa: BLE001
            fail(str(e))
        try:
            v = owner_verifier(owner)
        except Exception as e:  # noqa: BLE001
            fail("failed deserializing owner [%d][%s][%s]: %s" % (i, key, unique_id(owner), e))
        cap = _Capture()
        try:
            has_been_signed_by(owner, cap)
        except Exception as e:  # noqa: BLE001
            fail("failed signature verification [%d][%s][%s]: %s" % (i, key, unique_id(owner), e))
        done.append((key, owner, v, cap.msg, cap.sigma))
    text = check()
    if text:
        raise SignatureError(text)
    return [(o, s) for _, o, _, _, s in done]

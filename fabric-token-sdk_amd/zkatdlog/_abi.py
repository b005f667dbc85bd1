"""ctypes mirror of include/ftsamd.h (structs, codes) and the library loader."""
import ctypes
import os

FTZ_OK = 0
FTZ_ERR_PARSE = 1
FTZ_ERR_MALFORMED = 2
FTZ_ERR_WF = 3
FTZ_ERR_RANGE = 4
FTZ_ERR_MEMBERSHIP = 5
FTZ_ERR_PANIC = 6
FTZ_ERR_OPENING = 7
FTZ_DEBUG_CHALLENGES = 1  # ftz_ctx_set_debug

FTZ_SUCCESS = 0
FTZ_E_INVALID = -1
FTZ_E_PP = -2
FTZ_E_DEVICE = -3
FTZ_E_NOMEM = -4

FTZ_NKERNELS = 12
KERNEL_NAMES = ["decode", "zr", "hash_pre", "scalar", "g1p", "g2", "miller", "fexp", "g1", "hash", "verdict", "total"]
# ftz_prover_stats uses the same slots with the prover's stages
PROVER_STAGE_NAMES = ["decode", "zr", "rand+hash_pre", "scalar", "g1p", "g2", "miller", "fexp", "g1", "hash+responses",
                      "emit+b64", "total"]

# error strings of the reference for each class (tests match substrings)
MESSAGES = {
    FTZ_ERR_PARSE: "invalid transfer proof: cannot parse proof",
    FTZ_ERR_MALFORMED: "range proof not well formed",
    FTZ_ERR_WF: "invalid zero-knowledge transfer",
    FTZ_ERR_RANGE: "invalid range proof",
    FTZ_ERR_MEMBERSHIP: "invalid membership proof",
    FTZ_ERR_PANIC: "proof would make the reference verifier panic",
    FTZ_ERR_OPENING: "does not match the provided opening",
    8: "input to spend does not exists",
    9: "failed deserializing owner",
    10: "pseudonym signature invalid: zero-knowledge proof is invalid",
    11: "owner type verified in Go (htlc script)",
}
FTZ_ERR_OWNER = 9
FTZ_ERR_SIGNATURE = 10
FTZ_ERR_UNSUPPORTED = 11
FTZ_CURVE_FP256BN_AMCL = 0
FTZ_CURVE_BN254 = 1


class OwnerSig(ctypes.Structure):
    _fields_ = [("owner", ctypes.c_void_p), ("owner_len", ctypes.c_size_t), ("msg", ctypes.c_void_p),
                ("msg_len", ctypes.c_size_t), ("sig", ctypes.c_void_p), ("sig_len", ctypes.c_size_t)]


class OwnerAudit(ctypes.Structure):
    _fields_ = [("owner", ctypes.c_void_p), ("owner_len", ctypes.c_size_t), ("audit_info", ctypes.c_void_p),
                ("audit_info_len", ctypes.c_size_t)]


FTZ_ERR_AUDIT = 12


def pack_owner_audits(items):
    """items: (owner, audit_info) byte strings -> (ftz_owner_audit array, keepalive)"""
    items = list(items)
    arr = (OwnerAudit * max(len(items), 1))()
    keep = []
    for i, (o, a) in enumerate(items):
        o, a = bytes(o), bytes(a)
        keep += [o, a]
        arr[i] = OwnerAudit(ctypes.cast(ctypes.c_char_p(o), ctypes.c_void_p) if o else None, len(o),
                            ctypes.cast(ctypes.c_char_p(a), ctypes.c_void_p) if a else None, len(a))
    return arr, keep


def pack_owner_sigs(items):
    """items: (owner, msg, sig) byte strings; identical msg objects share one buffer."""
    arr = (OwnerSig * max(len(items), 1))()
    keep = []
    bufs = {}
    for i, (o, m, s_) in enumerate(items):
        def buf(b):
            k = id(b)
            if k not in bufs:
                bufs[k] = ctypes.create_string_buffer(bytes(b), max(len(b), 1))
                keep.append((b, bufs[k]))
            return ctypes.cast(bufs[k], ctypes.c_void_p)
        arr[i] = OwnerSig(buf(o), len(o), buf(m), len(m), buf(s_), len(s_))
    return arr, keep


FTZ_FEXP_EXACT = 0
FTZ_FEXP_FUENTES = 1
FEXP = {"exact": FTZ_FEXP_EXACT, "fuentes": FTZ_FEXP_FUENTES}


class Options(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("batch", ctypes.c_uint32), ("slots", ctypes.c_uint32),
                ("window_us", ctypes.c_uint32), ("threads", ctypes.c_uint32), ("fexp", ctypes.c_uint32),
                ("hold_inflight", ctypes.c_uint32), ("small_pass", ctypes.c_uint32),
                ("msm_window_bits", ctypes.c_uint32), ("msm_slot_cap", ctypes.c_uint32),
                ("msm_seg_slots", ctypes.c_uint32), ("msm_glv", ctypes.c_uint32),
                ("msm_precompute", ctypes.c_uint32), ("prover_tables", ctypes.c_uint32),
                ("msm_radix_bits", ctypes.c_uint32), ("first_pass", ctypes.c_uint32),
                ("tail_split", ctypes.c_uint32), ("msm_graph", ctypes.c_uint32),
                ("request_threads", ctypes.c_uint32)]


HOLD_NEVER = 0xFFFFFFFF


class TokenOpening(ctypes.Structure):
    _fields_ = [("type", ctypes.c_void_p), ("type_len", ctypes.c_size_t), ("value", ctypes.c_void_p),
                ("bf", ctypes.c_void_p)]


class Bytes(ctypes.Structure):
    _fields_ = [("p", ctypes.c_void_p), ("len", ctypes.c_size_t)]


# int (*)(void* user, const char* key, size_t key_len, const uint8_t** val, size_t* val_len)
GET_STATE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t))
GET_STATES_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p)
FTZ_ERR_INPUT = 8


def pack_bytes(items):
    """list of bytes -> (ftz_bytes array, keepalive)."""
    items = [bytes(x) for x in items]
    arr = (Bytes * max(1, len(items)))()
    keep = []
    for k, x in enumerate(items):
        b = ctypes.create_string_buffer(x, max(1, len(x)))
        keep.append(b)
        arr[k] = Bytes(ctypes.addressof(b), len(x))
    return arr, keep


def get_state_callback(ledger):
    """A GET_STATE_FN over a dict key(str) -> bytes (or a callable key -> bytes
    or None); the returned object must stay referenced during the call."""
    lookup = ledger.get if isinstance(ledger, dict) else ledger
    hold = {}

    def cb(user, key, key_len, val, val_len):
        k = ctypes.string_at(key, key_len).decode("utf-8", errors="surrogateescape")
        v = lookup(k)
        if v is None:
            return 1
        v = bytes(v)
        ent = hold.get(k)
        if ent is None or ent[0] != v:  # a callable ledger may answer differently later
            ent = hold[k] = (v, ctypes.create_string_buffer(v, max(1, len(v))))
        val[0] = ctypes.addressof(ent[1])
        val_len[0] = len(ent[0])
        return 0
    return GET_STATE_FN(cb)


def get_states_callback(ledger):
    """A GET_STATES_FN (batched lookup) over a dict key(str) -> bytes; the
    returned object must stay referenced during the call."""
    lookup = ledger.get if isinstance(ledger, dict) else ledger
    hold = []

    def cb(user, n, keys, vals):
        ks = ctypes.cast(keys, ctypes.POINTER(Bytes))
        vs = ctypes.cast(vals, ctypes.POINTER(Bytes))
        hold.clear()
        for i in range(n):
            k = ctypes.string_at(ks[i].p, ks[i].len).decode("utf-8", errors="surrogateescape")
            v = lookup(k)
            if v is None or len(v) == 0:
                vs[i] = Bytes(None, 0)
                continue
            b = ctypes.create_string_buffer(bytes(v), len(v))
            hold.append(b)
            vs[i] = Bytes(ctypes.cast(b, ctypes.c_void_p), len(v))
        return 0
    return GET_STATES_FN(cb)


def pack_openings(openings):
    """openings: iterable of (type str/bytes, value int, bf int)."""
    openings = list(openings)
    keep = []
    arr = (TokenOpening * max(1, len(openings)))()
    for i, (t, v, b) in enumerate(openings):
        t = t.encode() if isinstance(t, str) else bytes(t)
        arr[i] = TokenOpening(_buf(t, keep), len(t), _buf(_zr32([v]), keep), _buf(_zr32([b]), keep))
    return arr, keep


class ProverHostStats(ctypes.Structure):
    _fields_ = [("passes", ctypes.c_uint64), ("proofs", ctypes.c_uint64), ("wait_ms", ctypes.c_double),
                ("copy_ms", ctypes.c_double), ("plan_ms", ctypes.c_double), ("submit_ms", ctypes.c_double),
                ("wall_ms", ctypes.c_double)]


class EngineStats(ctypes.Structure):
    _fields_ = [("batches", ctypes.c_uint64), ("proofs", ctypes.c_uint64), ("plan_ms", ctypes.c_double),
                ("submit_ms", ctypes.c_double), ("device_ms", ctypes.c_double), ("wall_ms", ctypes.c_double),
                ("max_in_flight", ctypes.c_uint32)]


class Transfer(ctypes.Structure):
    _fields_ = [("inputs", ctypes.c_void_p), ("n_in", ctypes.c_uint32),
                ("outputs", ctypes.c_void_p), ("n_out", ctypes.c_uint32),
                ("proof", ctypes.c_void_p), ("proof_len", ctypes.c_size_t)]


class Issue(ctypes.Structure):
    _fields_ = [("outputs", ctypes.c_void_p), ("n_out", ctypes.c_uint32),
                ("proof", ctypes.c_void_p), ("proof_len", ctypes.c_size_t),
                ("anonymous", ctypes.c_uint8)]


class TransferWitness(ctypes.Structure):
    _fields_ = [("inputs", ctypes.c_void_p), ("n_in", ctypes.c_uint32),
                ("outputs", ctypes.c_void_p), ("n_out", ctypes.c_uint32),
                ("in_values", ctypes.c_void_p), ("in_bfs", ctypes.c_void_p),
                ("out_values", ctypes.c_void_p), ("out_bfs", ctypes.c_void_p),
                ("type", ctypes.c_void_p), ("type_len", ctypes.c_size_t), ("seed", ctypes.c_void_p)]


class IssueWitness(ctypes.Structure):
    _fields_ = [("outputs", ctypes.c_void_p), ("n_out", ctypes.c_uint32),
                ("values", ctypes.c_void_p), ("bfs", ctypes.c_void_p),
                ("type", ctypes.c_void_p), ("type_len", ctypes.c_size_t),
                ("anonymous", ctypes.c_uint8), ("seed", ctypes.c_void_p)]


def _buf(b, keep):
    if not b:
        return None
    c = ctypes.create_string_buffer(bytes(b), len(b))
    keep.append(c)
    return ctypes.addressof(c)


def _zr32(vals):
    return b"".join(int(v).to_bytes(32, "big") for v in vals)


def pack_transfer_witnesses(ws):
    """ws: iterable of dicts with inputs/outputs (concatenated 64-byte RawBytes),
    in_values/in_bfs/out_values/out_bfs (ints), type (str) and seed (32 bytes).
    Returns (ctypes array, keep-alive list)."""
    ws = list(ws)
    keep = []
    arr = (TransferWitness * max(1, len(ws)))()
    for i, w in enumerate(ws):
        t = w["type"].encode() if isinstance(w["type"], str) else bytes(w["type"])
        arr[i] = TransferWitness(_buf(w["inputs"], keep), len(w["inputs"]) // 64,
                                 _buf(w["outputs"], keep), len(w["outputs"]) // 64,
                                 _buf(_zr32(w["in_values"]), keep), _buf(_zr32(w["in_bfs"]), keep),
                                 _buf(_zr32(w["out_values"]), keep), _buf(_zr32(w["out_bfs"]), keep),
                                 _buf(t, keep), len(t), _buf(w["seed"], keep))
    return arr, keep


def pack_issue_witnesses(ws):
    ws = list(ws)
    keep = []
    arr = (IssueWitness * max(1, len(ws)))()
    for i, w in enumerate(ws):
        t = w["type"].encode() if isinstance(w["type"], str) else bytes(w["type"])
        arr[i] = IssueWitness(_buf(w["outputs"], keep), len(w["outputs"]) // 64,
                              _buf(_zr32(w["values"]), keep), _buf(_zr32(w["bfs"]), keep),
                              _buf(t, keep), len(t), 1 if w.get("anonymous") else 0, _buf(w["seed"], keep))
    return arr, keep


class Stats(ctypes.Structure):
    _fields_ = [("ms", ctypes.c_float * FTZ_NKERNELS), ("jobs", ctypes.c_uint64 * FTZ_NKERNELS)]


LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libftsamd.so")

# every symbol include/ftsamd.h declares (checked by tests/test_abi.py)
SYMBOLS = ["ftz_options_default", "ftz_ctx_create", "ftz_ctx_create_ex", "ftz_ctx_destroy", "ftz_last_error",
           "ftz_ctx_set_threads", "ftz_ctx_set_serial", "ftz_ctx_debug_poison", "ftz_ctx_set_debug", "ftz_ctx_set_layout", "ftz_ctx_info", "ftz_ctx_options", "ftz_ctx_engine_stats", "ftz_pp_validate", "ftz_pp_setup",
           "ftz_commit_tokens", "ftz_audit_openings",
           "ftz_verify_transfers", "ftz_verify_issues", "ftz_batch_load_transfers", "ftz_batch_load_issues",
           "ftz_batch_run", "ftz_batch_submit", "ftz_batch_wait", "ftz_batch_codes", "ftz_batch_bitmap", "ftz_batch_stats", "ftz_batch_size",
           "ftz_batch_destroy", "ftz_batch_challenges", "ftz_msm_g1", "ftz_msm_load", "ftz_msm_load_gen", "ftz_msm_run", "ftz_msm_set_scalars", "ftz_msm_run_scalars", "ftz_host_alloc", "ftz_host_free", "ftz_msm_info", "ftz_msm_destroy", "ftz_g1_sum",
           "ftz_token_request_decode", "ftz_verify_token_requests", "ftz_verify_token_requests_batched", "ftz_ctx_request_stats",
           "ftz_idemix_create", "ftz_verify_owner_signatures", "ftz_idemix_set_strict_nym", "ftz_idemix_destroy", "ftz_audit_owners",
           "ftz_prove_transfers", "ftz_prove_issues", "ftz_ctx_prover_stats", "ftz_prover_load_transfers", "ftz_prover_load_issues",
           "ftz_prover_run", "ftz_prover_submit", "ftz_prover_wait", "ftz_prover_bytes", "ftz_prover_proofs", "ftz_prover_stats", "ftz_prover_destroy"]

_lib = None


def use_library(path):
    """Bench / A/B entry points only (bench.py --lib): load the variant build at
    `path` (build.py --variant) instead of the bundled library.  No environment
    variable does this, so a deployment always runs the bundled build; must be
    called before the first load()."""
    global LIB_PATH
    path = os.path.abspath(path)
    if _lib is not None and path != LIB_PATH:
        raise RuntimeError("libftsamd already loaded from %s" % LIB_PATH)
    LIB_PATH = path


def loaded_path():
    """The path of the library this process loaded (None before load())."""
    return LIB_PATH if _lib is not None else None


def load():
    """Load libftsamd.so; raises loudly when it is missing (no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libftsamd.so not built (%s); run fabric-token-sdk_amd/build.py "
                           "-- there is no CPU fallback for the zkatdlog GPU verifier" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    vp, sz, u32, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int32
    lib.ftz_options_default.argtypes = [ctypes.POINTER(Options)]
    lib.ftz_options_default.restype = None
    lib.ftz_ctx_create.argtypes = [ctypes.c_char_p, sz, ctypes.c_int, ctypes.POINTER(vp)]
    lib.ftz_ctx_create_ex.argtypes = [ctypes.c_char_p, sz, ctypes.c_int, ctypes.POINTER(Options), ctypes.POINTER(vp)]
    lib.ftz_ctx_set_serial.argtypes = [vp, ctypes.c_int]
    lib.ftz_ctx_debug_poison.argtypes = [vp, ctypes.c_void_p]
    lib.ftz_ctx_set_debug.argtypes = [vp, ctypes.c_int]
    lib.ftz_ctx_set_layout.argtypes = [vp, ctypes.c_int, ctypes.c_int]
    lib.ftz_ctx_options.argtypes = [vp, ctypes.POINTER(Options)]
    lib.ftz_pp_validate.argtypes = [ctypes.c_char_p, sz]
    lib.ftz_pp_setup.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_char_p, sz, ctypes.c_int, ctypes.c_char_p,
                                 sz, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    lib.ftz_commit_tokens.argtypes = [vp, sz, ctypes.POINTER(TokenOpening), ctypes.POINTER(ctypes.c_uint8)]
    lib.ftz_audit_openings.argtypes = [vp, sz, ctypes.c_char_p, ctypes.POINTER(TokenOpening),
                                       ctypes.POINTER(ctypes.c_int32)]
    lib.ftz_ctx_engine_stats.argtypes = [vp, ctypes.POINTER(EngineStats), ctypes.c_int]
    lib.ftz_ctx_prover_stats.argtypes = [vp, ctypes.POINTER(ProverHostStats), ctypes.c_int]
    lib.ftz_ctx_destroy.argtypes = [vp]
    lib.ftz_ctx_destroy.restype = None
    lib.ftz_last_error.restype = ctypes.c_char_p
    lib.ftz_ctx_set_threads.argtypes = [vp, ctypes.c_int]
    lib.ftz_ctx_info.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(u32)]
    lib.ftz_verify_transfers.argtypes = [vp, sz, ctypes.POINTER(Transfer), ctypes.POINTER(i32)]
    lib.ftz_verify_issues.argtypes = [vp, sz, ctypes.POINTER(Issue), ctypes.POINTER(i32)]
    lib.ftz_batch_load_transfers.argtypes = [vp, sz, ctypes.POINTER(Transfer), ctypes.POINTER(vp)]
    lib.ftz_batch_load_issues.argtypes = [vp, sz, ctypes.POINTER(Issue), ctypes.POINTER(vp)]
    lib.ftz_batch_run.argtypes = [vp]
    lib.ftz_batch_submit.argtypes = [vp]
    lib.ftz_batch_wait.argtypes = [vp]
    lib.ftz_batch_codes.argtypes = [vp, ctypes.POINTER(i32)]
    lib.ftz_batch_bitmap.argtypes = [vp, ctypes.POINTER(ctypes.c_uint8)]
    lib.ftz_batch_stats.argtypes = [vp, ctypes.POINTER(Stats)]
    lib.ftz_batch_size.argtypes = [vp]
    lib.ftz_batch_size.restype = sz
    lib.ftz_batch_destroy.argtypes = [vp]
    lib.ftz_batch_destroy.restype = None
    lib.ftz_batch_challenges.argtypes = [vp, sz, ctypes.POINTER(i32), ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    u8p = ctypes.POINTER(ctypes.c_uint8)
    lib.ftz_msm_g1.argtypes = [vp, sz, ctypes.c_char_p, ctypes.c_char_p, u8p]
    lib.ftz_msm_load.argtypes = [vp, sz, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(vp)]
    lib.ftz_msm_load_gen.argtypes = [vp, sz, u32, ctypes.c_char_p, ctypes.POINTER(vp)]
    lib.ftz_msm_run.argtypes = [vp, u8p]
    lib.ftz_msm_set_scalars.argtypes = [vp, ctypes.c_char_p]
    lib.ftz_msm_run_scalars.argtypes = [vp, ctypes.c_void_p, u8p]
    lib.ftz_host_alloc.argtypes = [sz, ctypes.POINTER(vp)]
    lib.ftz_host_free.argtypes = [vp]
    lib.ftz_host_free.restype = None
    lib.ftz_msm_info.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(u32)]
    lib.ftz_msm_destroy.argtypes = [vp]
    lib.ftz_msm_destroy.restype = None
    lib.ftz_g1_sum.argtypes = [vp, sz, ctypes.c_char_p, u8p]
    lib.ftz_idemix_create.argtypes = [vp, ctypes.c_char_p, sz, ctypes.c_int, ctypes.POINTER(vp)]
    lib.ftz_verify_owner_signatures.argtypes = [vp, sz, ctypes.POINTER(OwnerSig), ctypes.POINTER(ctypes.c_int32)]
    lib.ftz_audit_owners.argtypes = [vp, sz, ctypes.POINTER(OwnerAudit), ctypes.POINTER(ctypes.c_int32)]
    lib.ftz_idemix_set_strict_nym.argtypes = [vp, ctypes.c_int]
    lib.ftz_idemix_destroy.argtypes = [vp]
    lib.ftz_idemix_destroy.restype = None
    lib.ftz_token_request_decode.argtypes = [ctypes.c_char_p, sz, ctypes.POINTER(sz), ctypes.POINTER(Bytes), sz]
    # the callback as a plain function pointer: a ctypes GET_STATE(S)_FN or a native one
    lib.ftz_verify_token_requests.argtypes = [vp, sz, ctypes.POINTER(Bytes), vp, vp,
                                              ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]
    lib.ftz_verify_token_requests_batched.argtypes = [vp, sz, ctypes.POINTER(Bytes), vp, vp,
                                                      ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]
    lib.ftz_ctx_request_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    szp = ctypes.POINTER(ctypes.c_size_t)
    i32p = ctypes.POINTER(ctypes.c_int32)
    lib.ftz_prove_transfers.argtypes = [vp, sz, ctypes.POINTER(TransferWitness), u8p, sz, szp, i32p]
    lib.ftz_prove_issues.argtypes = [vp, sz, ctypes.POINTER(IssueWitness), u8p, sz, szp, i32p]
    lib.ftz_prover_load_transfers.argtypes = [vp, sz, ctypes.POINTER(TransferWitness), ctypes.POINTER(vp)]
    lib.ftz_prover_load_issues.argtypes = [vp, sz, ctypes.POINTER(IssueWitness), ctypes.POINTER(vp)]
    lib.ftz_prover_run.argtypes = [vp]
    lib.ftz_prover_submit.argtypes = [vp]
    lib.ftz_prover_wait.argtypes = [vp]
    lib.ftz_prover_bytes.argtypes = [vp]
    lib.ftz_prover_bytes.restype = sz
    lib.ftz_prover_proofs.argtypes = [vp, u8p, sz, szp, i32p]
    lib.ftz_prover_stats.argtypes = [vp, ctypes.POINTER(Stats)]
    lib.ftz_prover_destroy.argtypes = [vp]
    lib.ftz_prover_destroy.restype = None
    _lib = lib
    return lib


def pack_transfers(items):
    """items: iterable of (inputs: bytes (n_in*64), outputs: bytes (n_out*64), proof: bytes).
    Returns (ctypes array, keepalive list)."""
    items = list(items)
    arr = (Transfer * max(1, len(items)))()
    keep = []
    for k, (ins, outs, proof) in enumerate(items):
        bi, bo, bp = (ctypes.create_string_buffer(bytes(x), max(1, len(x))) for x in (ins, outs, proof))
        keep += [bi, bo, bp]
        arr[k] = Transfer(ctypes.addressof(bi), len(ins) // 64, ctypes.addressof(bo), len(outs) // 64,
                          ctypes.addressof(bp), len(proof))
    return arr, keep


def _np_struct(dtype_fields, ctype):
    import numpy as np
    dt = np.dtype(dtype_fields, align=True)
    assert dt.itemsize == ctypes.sizeof(ctype), (dt.itemsize, ctypes.sizeof(ctype))
    return dt


def _addr(buf):
    """(address, keep) of a bytes-like / numpy uint8 buffer, without copying numpy arrays."""
    import numpy as np
    if isinstance(buf, np.ndarray):
        a = np.ascontiguousarray(buf, dtype=np.uint8)
        return a.ctypes.data, a
    b = bytes(buf)
    c = ctypes.create_string_buffer(b, max(1, len(b)))
    return ctypes.addressof(c), c


def transfer_dtype():
    """numpy dtype with the layout of ftz_transfer"""
    return _np_struct([("inputs", "<u8"), ("n_in", "<u4"), ("outputs", "<u8"), ("n_out", "<u4"), ("proof", "<u8"),
                       ("proof_len", "<u8")], Transfer)


def buffer_address(buf):
    """(address, keepalive) of a bytes-like or numpy buffer"""
    return _addr(buf)


def pack_transfers_flat(inputs, in_off, outputs, out_off, proofs, proof_off):
    """Zero-copy ftz_transfer array over flat buffers (a block as it arrives):
    transfer i has inputs[in_off[i]:in_off[i+1]] (64-byte RawBytes each),
    outputs[out_off[i]:out_off[i+1]] and proof proofs[proof_off[i]:proof_off[i+1]];
    offsets are byte offsets, n+1 of each.  Returns (pointer, n, keepalive)."""
    import numpy as np
    in_off, out_off, proof_off = (np.asarray(o, dtype=np.int64) for o in (in_off, out_off, proof_off))
    n = len(proof_off) - 1
    dt = transfer_dtype()
    ai, ki = _addr(inputs)
    ao, ko = _addr(outputs)
    ap, kp = _addr(proofs)
    arr = np.zeros(max(1, n), dtype=dt)
    arr["inputs"][:n] = ai + in_off[:-1]
    arr["n_in"][:n] = (in_off[1:] - in_off[:-1]) // 64
    arr["outputs"][:n] = ao + out_off[:-1]
    arr["n_out"][:n] = (out_off[1:] - out_off[:-1]) // 64
    arr["proof"][:n] = ap + proof_off[:-1]
    arr["proof_len"][:n] = proof_off[1:] - proof_off[:-1]
    return ctypes.cast(arr.ctypes.data, ctypes.POINTER(Transfer)), n, (arr, ki, ko, kp)


def pack_issues_flat(outputs, out_off, proofs, proof_off, anonymous):
    """As pack_transfers_flat for issues; anonymous: n flags."""
    import numpy as np
    out_off, proof_off = (np.asarray(o, dtype=np.int64) for o in (out_off, proof_off))
    n = len(proof_off) - 1
    dt = _np_struct([("outputs", "<u8"), ("n_out", "<u4"), ("proof", "<u8"), ("proof_len", "<u8"),
                     ("anonymous", "u1")], Issue)
    ao, ko = _addr(outputs)
    ap, kp = _addr(proofs)
    arr = np.zeros(max(1, n), dtype=dt)
    arr["outputs"][:n] = ao + out_off[:-1]
    arr["n_out"][:n] = (out_off[1:] - out_off[:-1]) // 64
    arr["proof"][:n] = ap + proof_off[:-1]
    arr["proof_len"][:n] = proof_off[1:] - proof_off[:-1]
    arr["anonymous"][:n] = np.asarray(anonymous, dtype=np.uint8)[:n]
    return ctypes.cast(arr.ctypes.data, ctypes.POINTER(Issue)), n, (arr, ko, kp)


def pack_transfer_witnesses_tiled(bases, sel, seeds):
    """ftz_transfer_witness array for n proofs whose witnesses repeat a few
    distinct bases (dicts as in pack_transfer_witnesses, without "seed"):
    proof i uses bases[sel[i]] and the 32-byte seed seeds[32 i: 32 i + 32].
    Returns (pointer, n, keepalive) -- the struct array is built with numpy,
    so a 1M-proof job packs in well under a second."""
    import numpy as np
    sel = np.asarray(sel, dtype=np.int64)
    n = len(sel)
    keep = []
    cols = {k: [] for k in ("inputs", "n_in", "outputs", "n_out", "in_values", "in_bfs", "out_values", "out_bfs",
                            "type", "type_len")}
    for w in bases:
        t = w["type"].encode() if isinstance(w["type"], str) else bytes(w["type"])
        cols["inputs"].append(_buf(w["inputs"], keep) or 0)
        cols["n_in"].append(len(w["inputs"]) // 64)
        cols["outputs"].append(_buf(w["outputs"], keep) or 0)
        cols["n_out"].append(len(w["outputs"]) // 64)
        for k, src in (("in_values", "in_values"), ("in_bfs", "in_bfs"), ("out_values", "out_values"),
                       ("out_bfs", "out_bfs")):
            cols[k].append(_buf(_zr32(w[src]), keep) or 0)
        cols["type"].append(_buf(t, keep) or 0)
        cols["type_len"].append(len(t))
    dt = _np_struct([("inputs", "<u8"), ("n_in", "<u4"), ("outputs", "<u8"), ("n_out", "<u4"), ("in_values", "<u8"),
                     ("in_bfs", "<u8"), ("out_values", "<u8"), ("out_bfs", "<u8"), ("type", "<u8"),
                     ("type_len", "<u8"), ("seed", "<u8")], TransferWitness)
    arr = np.zeros(max(1, n), dtype=dt)
    for k, v in cols.items():
        arr[k][:n] = np.asarray(v, dtype=np.uint64)[sel]
    sa, sk = _addr(seeds)
    arr["seed"][:n] = sa + 32 * np.arange(n, dtype=np.uint64)
    return ctypes.cast(arr.ctypes.data, ctypes.POINTER(TransferWitness)), n, (arr, keep, sk)


def pack_issue_witnesses_tiled(bases, sel, seeds):
    """As pack_transfer_witnesses_tiled for issue witnesses."""
    import numpy as np
    sel = np.asarray(sel, dtype=np.int64)
    n = len(sel)
    keep = []
    cols = {k: [] for k in ("outputs", "n_out", "values", "bfs", "type", "type_len", "anonymous")}
    for w in bases:
        t = w["type"].encode() if isinstance(w["type"], str) else bytes(w["type"])
        cols["outputs"].append(_buf(w["outputs"], keep) or 0)
        cols["n_out"].append(len(w["outputs"]) // 64)
        cols["values"].append(_buf(_zr32(w["values"]), keep) or 0)
        cols["bfs"].append(_buf(_zr32(w["bfs"]), keep) or 0)
        cols["type"].append(_buf(t, keep) or 0)
        cols["type_len"].append(len(t))
        cols["anonymous"].append(1 if w.get("anonymous") else 0)
    dt = _np_struct([("outputs", "<u8"), ("n_out", "<u4"), ("values", "<u8"), ("bfs", "<u8"), ("type", "<u8"),
                     ("type_len", "<u8"), ("anonymous", "u1"), ("seed", "<u8")], IssueWitness)
    arr = np.zeros(max(1, n), dtype=dt)
    for k, v in cols.items():
        arr[k][:n] = np.asarray(v, dtype=np.uint64 if k != "anonymous" else np.uint8)[sel]
    sa, sk = _addr(seeds)
    arr["seed"][:n] = sa + 32 * np.arange(n, dtype=np.uint64)
    return ctypes.cast(arr.ctypes.data, ctypes.POINTER(IssueWitness)), n, (arr, keep, sk)


def pack_issues(items):
    """items: iterable of (outputs: bytes, proof: bytes, anonymous: bool)."""
    items = list(items)
    arr = (Issue * max(1, len(items)))()
    keep = []
    for k, (outs, proof, anon) in enumerate(items):
        bo, bp = (ctypes.create_string_buffer(bytes(x), max(1, len(x))) for x in (outs, proof))
        keep += [bo, bp]
        arr[k] = Issue(ctypes.addressof(bo), len(outs) // 64, ctypes.addressof(bp), len(proof), 1 if anon else 0)
    return arr, keep

"""Host-side mirror of the reference `crypto` crate (crypto/src/lib.rs) over
the MI355X engine's C ABI (include/coa_verify.h).

Same names, same argument meaning, same error behaviour as the Rust API the
reference's callers use:

    Digest([u8;32])                         crypto/src/lib.rs:20-57
    PublicKey([u8;32]) + base64 helpers      crypto/src/lib.rs:64-119
    Signature{part1, part2}                  crypto/src/lib.rs:177-182
    Signature.verify(digest, public_key)     crypto/src/lib.rs:200-204
    Signature.verify_batch(digest, votes)    crypto/src/lib.rs:206-219
    CryptoError (opaque ed25519::Error)      crypto/src/lib.rs:18

`verify`/`verify_batch` raise CryptoError exactly where the Rust functions
return Err.  All verification runs in the HIP kernels of
lib/libcoa_verify.so; if that library is missing or no GPU is present the
calls raise EngineError -- there is no CPU fallback.

Bulk (engine-level) entry points, used by the primary/worker callers'
batching paths and by the benchmark, take numpy arrays (host) or torch
tensors (device) -- see verify_strict_many, verify_batch_groups, sha512_many.

A process that also uses torch's GPU API must import torch before the first
call here: the library links libamdhip64 by soname and then shares torch's
HIP runtime; loaded first, it brings ROCm's own runtime and torch's bundled
copy finds no GPU (tools/probe_torch_after_init.py).
"""
import base64
import ctypes
import os

import numpy as np

from . import verified  # noqa: E402  (the verdict cache, rust/crypto/src/verified.rs)

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# COA_VERIFY_LIB overrides the library (A/B runs of two builds in one session)
LIB_PATH = os.environ.get("COA_VERIFY_LIB") or os.path.join(_PKG, "lib", "libcoa_verify.so")

COA_OK, COA_REJECT = 0, 1
_ERRORS = {-1: "COA_EINVAL", -2: "COA_ENODEVICE", -3: "COA_EHIP", -4: "COA_ENOMEM"}


class CryptoError(Exception):
    """crypto::CryptoError = ed25519::Error: opaque verification failure."""


class EngineError(RuntimeError):
    """The GPU engine could not run the call (no device, HIP error, bad args)."""


_lib = None


class QueueMetrics(ctypes.Structure):
    """coa_queue_metrics_t (include/coa_verify.h)."""
    _fields_ = [(n, ctypes.c_uint64) for n in ("requests", "windows", "signatures", "batches", "certificates",
                                               "digests", "max_window", "max_in_flight", "max_pending")] + \
               [(n, ctypes.c_double) for n in ("wait_us_mean", "wait_us_p50", "wait_us_p99", "wait_us_max")] + \
               [(n, ctypes.c_uint64) for n in ("retried_windows", "recovered_windows", "failed_windows")] + \
               [("window_us_max", ctypes.c_double), ("window_max_items", ctypes.c_uint64),
                ("window_max_kinds", ctypes.c_uint32), ("stream_kind", ctypes.c_int32),
                ("slot_wait_us_max", ctypes.c_double), ("staging_grows", ctypes.c_uint64),
                ("slots_verify", ctypes.c_uint32), ("slots_digest", ctypes.c_uint32),
                ("deferred_requests", ctypes.c_uint64), ("resolver_passes", ctypes.c_uint64),
                ("resolve_us_max", ctypes.c_double), ("stage_us", ctypes.c_double * 12),
                ("window_max_at_ms", ctypes.c_double), ("window_max_device_us", ctypes.c_double)]

    # COA_QSTAGE_* indices of stage_us
    STAGES = ("intake", "gather", "slot_wait", "pack", "enqueue", "device_wait", "scatter", "callbacks", "resolve")


def metrics_dict(m):
    """A QueueMetrics as a dict; stage_us becomes {stage name: microseconds}."""
    d = {name: getattr(m, name) for name, _ in QueueMetrics._fields_ if name != "stage_us"}
    d["stage_us"] = {k: m.stage_us[i] for i, k in enumerate(QueueMetrics.STAGES)}
    return d


# void (*coa_verdict_cb)(void* user, int status, const uint8_t* verdicts, size_t n)
VERDICT_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t)


def _u8p(a):
    """Address of a numpy buffer for a `void*`-typed argument (ctypes'
    data_as costs ~5 us a call; the address alone ~1 us), None for NULL."""
    return a.ctypes.data if a is not None else None


def lib():
    """Load the engine library (fail loudly if it is absent)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EngineError(f"{LIB_PATH} not built (run __graft_entry__.build()); no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    # byte and u64 buffers are passed as void*: numpy addresses (_u8p) and
    # bytes objects (no copy) both convert without a pointer object
    P8 = ctypes.c_void_p
    P64 = ctypes.c_void_p
    sz, vp = ctypes.c_size_t, ctypes.c_void_p
    sig = {
        "coa_init": ([ctypes.c_int], ctypes.c_int),
        "coa_init_devices": ([ctypes.POINTER(ctypes.c_int), ctypes.c_int], ctypes.c_int),
        "coa_shutdown": ([], ctypes.c_int),
        "coa_device_count": ([], ctypes.c_int),
        "coa_device_ids": ([ctypes.POINTER(ctypes.c_int), ctypes.c_int], ctypes.c_int),
        "coa_self_test": ([ctypes.c_int, P64], ctypes.c_int),
        "coa_fe_rows_check_device": ([ctypes.c_int, vp, sz, vp, vp], ctypes.c_int),
        "coa_last_error": ([], ctypes.c_char_p),
        "coa_engine_recoveries": ([P64, P64], ctypes.c_int),
        "coa_version": ([], ctypes.c_char_p),
        "coa_ed25519_verify_strict": ([P8, P8, P8], ctypes.c_int),
        "coa_ed25519_verify_strict_many": ([P8, sz, P8, P8, sz, P8], ctypes.c_int),
        "coa_verify_workspace_bytes": ([sz], sz),
        "coa_ed25519_verify_strict_many_device": ([ctypes.c_int, vp, sz, vp, vp, sz, vp, vp, vp], ctypes.c_int),
        "coa_ed25519_challenge_many_device": ([ctypes.c_int, vp, sz, vp, vp, sz, vp, vp], ctypes.c_int),
        "coa_ed25519_verify_prehashed_many_device": ([ctypes.c_int, vp, vp, vp, sz, vp, vp, vp], ctypes.c_int),
        "coa_ed25519_verify_batch": ([P8, P8, P8, sz, ctypes.c_uint64], ctypes.c_int),
        "coa_ed25519_verify_batch_groups": ([P8, P8, P8, P64, sz, P8, ctypes.c_uint64], ctypes.c_int),
        "coa_ed25519_verify_batch_groups_z": ([P8, P8, P8, P64, sz, P8, P8], ctypes.c_int),
        "coa_verify_batch_workspace_bytes": ([sz], sz),
        "coa_ed25519_verify_batch_device": ([ctypes.c_int, vp, vp, vp, sz, vp, ctypes.c_uint64, vp, vp, sz, vp],
                                            ctypes.c_int),
        "coa_sha512_many": ([P8, P64, sz, P8], ctypes.c_int),
        "coa_sha512_trunc32_many": ([P8, P64, sz, P8], ctypes.c_int),
        "coa_sha512_many_device": ([ctypes.c_int, vp, vp, sz, vp, vp], ctypes.c_int),
        "coa_ed25519_public_keys": ([P8, sz, P8], ctypes.c_int),
        "coa_ed25519_sign_many": ([P8, P8, sz, sz, P8, P8], ctypes.c_int),
        "coa_ed25519_sign_many_device": ([ctypes.c_int, vp, vp, sz, sz, vp, vp, vp], ctypes.c_int),
        "coa_committee_register": ([P8, sz], ctypes.c_int),
        "coa_committee_key_flags": ([ctypes.POINTER(ctypes.c_uint32), sz], ctypes.c_int),
        "coa_certificate_verify_many": ([P8, P64, P8, P8, P8, P64, P8, P8, P64, sz, ctypes.c_uint64, P8],
                                        ctypes.c_int),
        "coa_certificate_verify": ([P8, sz, P8, P8, P8, ctypes.c_uint64, P8, P8, sz, ctypes.c_uint64], ctypes.c_int),
        "coa_certificate_workspace_bytes": ([sz, sz], sz),
        "coa_certificate_verify_many_device": ([ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp, sz, sz, vp, vp, vp],
                                               ctypes.c_int),
        "coa_wire_scan": ([P8, P64, sz, ctypes.POINTER(ctypes.c_int32), P64, P64], ctypes.c_int),
        "coa_wire_decode_certificates": ([P8, P64, sz, P8, P64, P8, P8, P8, P64, P8, P8, P64,
                                          ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
        "coa_wire_decode_votes": ([P8, P64, sz, P8, P64, P8, P8, P8], ctypes.c_int),
        "coa_wire_decode_headers": ([P8, P64, sz, P8, P64, P8, P8, P8, P64, ctypes.POINTER(ctypes.c_uint32)],
                                    ctypes.c_int),
        # the engine's own CPU path (explicit only; never a silent fallback)
        "coa_cpu_ed25519_verify_strict": ([P8, sz, P8, P8], ctypes.c_int),
        "coa_cpu_ed25519_verify_strict_many": ([P8, sz, P8, P8, sz, P8, ctypes.c_int], ctypes.c_int),
        "coa_cpu_ed25519_verify_batch": ([P8, P8, P8, sz, ctypes.c_uint64], ctypes.c_int),
        "coa_cpu_ed25519_verify_batch_groups_z": ([P8, P8, P8, P64, sz, P8, P8, ctypes.c_int], ctypes.c_int),
        "coa_cpu_sha512_many": ([P8, P64, sz, P8, ctypes.c_int], ctypes.c_int),
        "coa_cpu_certificate_verify_many": ([P8, P64, P8, P8, P8, P64, P8, P8, P64, sz, ctypes.c_uint64, P8,
                                             ctypes.c_int], ctypes.c_int),
        "coa_cpu_certificate_verify_many_z": ([P8, P64, P8, P8, P8, P64, P8, P8, P64, sz, P8, P8, ctypes.c_int],
                                              ctypes.c_int),
        "coa_queue_create": ([sz, ctypes.c_uint32], vp),
        "coa_queue_submit_verify": ([vp, P8, P8, P8, VERDICT_CB, vp], ctypes.c_int),
        "coa_queue_submit_verify_many": ([vp, P8, P8, P8, sz, VERDICT_CB, vp], ctypes.c_int),
        "coa_queue_submit_batch": ([vp, P8, P8, P8, sz, VERDICT_CB, vp], ctypes.c_int),
        "coa_queue_submit_certificate": ([vp, P8, sz, P8, P8, P8, ctypes.c_uint64, P8, P8, sz, VERDICT_CB, vp],
                                         ctypes.c_int),
        "coa_queue_submit_certificate_borrowed": ([vp, P8, sz, P8, P8, P8, ctypes.c_uint64, P8, P8, sz, VERDICT_CB,
                                                   vp], ctypes.c_int),
        "coa_queue_submit_digest": ([vp, P8, sz, VERDICT_CB, vp], ctypes.c_int),
        "coa_queue_digest_count": ([vp, P64], ctypes.c_int),
        "coa_queue_flush": ([vp], ctypes.c_int),
        "coa_queue_set_idle_launch": ([vp, ctypes.c_uint32], ctypes.c_int),
        "coa_queue_stats": ([vp, P64, P64, P64], ctypes.c_int),
        "coa_queue_metrics": ([vp, ctypes.POINTER(QueueMetrics)], ctypes.c_int),
        "coa_queue_metrics_reset": ([vp], ctypes.c_int),
        "coa_queue_destroy": ([vp], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name, None)
        if f is None and os.environ.get("COA_VERIFY_LIB") and name.startswith("coa_cpu_"):
            continue  # an older A/B build (COA_VERIFY_LIB) without the CPU path
        if f is None:
            raise EngineError(f"{LIB_PATH} does not export {name}")
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def cpu_verify_strict_many(msgs, pks, sigs, nthreads=0):
    """The engine's own CPU path (csrc/coa_cpu.cpp) for n triples: verdict
    bytes 0 Ok / 1 Err.  Explicit only -- what a caller runs when its GPU
    calls failed (rust/crypto/src/degrade.rs); no GPU entry point calls it."""
    msgs, pks, sigs = (np.ascontiguousarray(a, dtype=np.uint8) for a in (msgs, pks, sigs))
    n = pks.shape[0]
    out = np.ones(n, np.uint8)
    _check(lib().coa_cpu_ed25519_verify_strict_many(_u8p(msgs), msgs.shape[1] if n else 0, _u8p(pks), _u8p(sigs), n,
                                                    _u8p(out), nthreads))
    return out


def cpu_verify_batch_groups(msgs, pks, sigs, group_offsets, zs, nthreads=0):
    """CPU path of coa_ed25519_verify_batch_groups_z (explicit weights)."""
    msgs, pks, sigs, zs = (np.ascontiguousarray(a, dtype=np.uint8) for a in (msgs, pks, sigs, zs))
    off = np.ascontiguousarray(group_offsets, dtype=np.uint64)
    g = off.size - 1
    out = np.ones(g, np.uint8)
    _check(lib().coa_cpu_ed25519_verify_batch_groups_z(_u8p(msgs), _u8p(pks), _u8p(sigs), _u8p(off), g, _u8p(zs),
                                                       _u8p(out), nthreads))
    return out


def cpu_sha512_many(messages, nthreads=0):
    """CPU path of coa_sha512_many: 64-byte digests, one row per message."""
    data = np.frombuffer(b"".join(bytes(m) for m in messages) + b"\0", np.uint8)
    off = np.zeros(len(messages) + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in messages])
    out = np.zeros((len(messages), 64), np.uint8)
    _check(lib().coa_cpu_sha512_many(_u8p(data), _u8p(off), len(messages), _u8p(out), nthreads))
    return out


def cpu_certificate_verify_many(header_inputs, ids, origins, header_sigs, rounds, vote_pks, vote_sigs, vote_offsets,
                                zs=None, rng_seed=0, nthreads=0):
    """CPU path of coa_certificate_verify_many: COA_CERT_* bits per
    certificate (zs: the votes' 16-byte weights, else drawn from rng_seed)."""
    n = len(header_inputs)
    hdata = np.frombuffer(b"".join(bytes(h) for h in header_inputs) + b"\0", np.uint8)
    hoff = np.zeros(n + 1, np.uint64)
    hoff[1:] = np.cumsum([len(h) for h in header_inputs])
    ids, origins, header_sigs, vote_pks, vote_sigs = (np.ascontiguousarray(a, dtype=np.uint8) for a in
                                                      (ids, origins, header_sigs, vote_pks, vote_sigs))
    rounds = np.ascontiguousarray(rounds, dtype=np.uint64)
    voff = np.ascontiguousarray(vote_offsets, dtype=np.uint64)
    out = np.full(n, 0xff, np.uint8)
    L = lib()
    if zs is None:
        _check(L.coa_cpu_certificate_verify_many(_u8p(hdata), _u8p(hoff), _u8p(ids), _u8p(origins), _u8p(header_sigs),
                                                 _u8p(rounds), _u8p(vote_pks), _u8p(vote_sigs), _u8p(voff), n,
                                                 rng_seed, _u8p(out), nthreads))
    else:
        zs = np.ascontiguousarray(zs, dtype=np.uint8)
        _check(L.coa_cpu_certificate_verify_many_z(_u8p(hdata), _u8p(hoff), _u8p(ids), _u8p(origins),
                                                   _u8p(header_sigs), _u8p(rounds), _u8p(vote_pks), _u8p(vote_sigs),
                                                   _u8p(voff), n, _u8p(zs), _u8p(out), nthreads))
    return out


def _check(rc):
    if rc < 0:
        msg = lib().coa_last_error().decode(errors="replace")
        raise EngineError(f"{_ERRORS.get(rc, rc)}: {msg}")
    return rc


def _bytes_array(items, width):
    a = np.frombuffer(b"".join(bytes(x) for x in items), dtype=np.uint8) if items else np.zeros(0, np.uint8)
    if a.size != len(items) * width:
        raise ValueError(f"every item must be {width} bytes")
    return np.ascontiguousarray(a).copy()


# --------------------------------------------------------------- the types
class Digest:
    """crypto::Digest -- 32 bytes (crypto/src/lib.rs:20-57)."""

    __slots__ = ("data",)

    def __init__(self, data=bytes(32)):
        data = bytes(data)
        if len(data) != 32:
            raise ValueError("Digest is 32 bytes")
        self.data = data

    def to_vec(self):
        return list(self.data)

    def size(self):
        return 32

    def __bytes__(self):
        return self.data

    def __eq__(self, o):
        return isinstance(o, Digest) and o.data == self.data

    def __lt__(self, o):
        return self.data < o.data

    def __hash__(self):
        return hash(self.data)

    def __repr__(self):  # Debug = base64
        return base64.b64encode(self.data).decode()

    def __str__(self):  # Display = first 16 base64 chars
        return base64.b64encode(self.data).decode()[:16]


class PublicKey:
    """crypto::PublicKey -- 32-byte compressed point (crypto/src/lib.rs:64-119)."""

    __slots__ = ("data",)

    def __init__(self, data=bytes(32)):
        data = bytes(data)
        if len(data) != 32:
            raise ValueError("PublicKey is 32 bytes")
        self.data = data

    def encode_base64(self):
        return base64.b64encode(self.data).decode()

    @staticmethod
    def decode_base64(s):
        raw = base64.b64decode(s)
        if len(raw) < 32:
            raise ValueError("InvalidLength")
        return PublicKey(raw[:32])

    def __bytes__(self):
        return self.data

    def __eq__(self, o):
        return isinstance(o, PublicKey) and o.data == self.data

    def __lt__(self, o):
        return self.data < o.data

    def __hash__(self):
        return hash(self.data)

    def __repr__(self):
        return self.encode_base64()

    def __str__(self):
        return self.encode_base64()[:16]


class Signature:
    """crypto::Signature {part1: R, part2: s} (crypto/src/lib.rs:177-219)."""

    __slots__ = ("part1", "part2")

    def __init__(self, part1=bytes(32), part2=bytes(32)):  # Default = 64 zero bytes
        self.part1, self.part2 = bytes(part1), bytes(part2)
        if len(self.part1) != 32 or len(self.part2) != 32:
            raise ValueError("Signature parts are 32 bytes")

    @classmethod
    def from_bytes(cls, b):
        b = bytes(b)
        if len(b) != 64:
            raise ValueError("Signature is 64 bytes")
        return cls(b[:32], b[32:])

    def flatten(self):
        return self.part1 + self.part2

    def verify(self, digest, public_key):
        """Ok (returns None) or raises CryptoError -- Signature::verify.  A
        triple the pre-verification stage already verified (Ok or Err) is
        answered from `verified`, as rust/crypto/src/gpu.rs does; any other
        goes to the engine (one single-signature launch)."""
        d, pk = bytes(digest), bytes(public_key)
        if len(d) != 32 or len(pk) != 32:
            raise ValueError("digest and public key are 32 bytes")
        sig = self.flatten()
        ok = verified.take_signature(d, pk, sig)
        if ok is None:
            ok = engine_verify_strict(d, pk, sig) == COA_OK
        if not ok:
            raise CryptoError("signature verification failed")

    @staticmethod
    def verify_batch(digest, votes, rng_seed=0):
        """Ok or raises CryptoError -- Signature::verify_batch over
        (PublicKey, Signature) votes that all sign `digest`."""
        votes = list(votes)
        d = np.frombuffer(bytes(digest), np.uint8).copy()
        pks = _bytes_array([bytes(pk) for pk, _ in votes], 32)
        sgs = _bytes_array([s.flatten() for _, s in votes], 64)
        rc = _check(lib().coa_ed25519_verify_batch(_u8p(d), _u8p(pks), _u8p(sgs), len(votes), rng_seed))
        if rc != COA_OK:
            raise CryptoError("batch verification failed")

    def __repr__(self):
        return f"Signature({self.flatten().hex()})"


# ----------------------------------------------------------- engine level
def engine_verify_strict(digest, public_key, signature):
    """One Signature::verify through the engine (coa_ed25519_verify_strict):
    COA_OK or COA_REJECT."""
    return _check(lib().coa_ed25519_verify_strict(bytes(digest), bytes(public_key), bytes(signature)))


def init(n_gpus=0):
    return _check(lib().coa_init(n_gpus))


def init_devices(ids):
    """Open exactly these HIP devices (bench.py: each rank its own GPU).  A
    device listed k times gets k contexts, i.e. k index-range shards."""
    arr = (ctypes.c_int * len(ids))(*ids)
    return _check(lib().coa_init_devices(arr, len(ids)))


def device_count():
    return _check(lib().coa_device_count())


def device_ids():
    """HIP device id of every opened context, in shard order."""
    n = _check(lib().coa_device_ids(None, 0))
    arr = (ctypes.c_int * max(n, 1))()
    _check(lib().coa_device_ids(arr, n))
    return list(arr[:n])


def shutdown():
    """Release every context (the next call re-initialises lazily)."""
    return _check(lib().coa_shutdown())


def engine_recoveries():
    """coa_engine_recoveries: contexts rebuilt and shards re-run after device
    failures of host-pointer calls since the library loaded."""
    a, b = ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib().coa_engine_recoveries(ctypes.byref(a), ctypes.byref(b)))
    return {"contexts_rebuilt": a.value, "shards_rerun": b.value}


def self_test(device=0):
    """Number of inconsistent entries in the device's wide B comb (0 = every
    entry is m * 2^(20 j) * B; also 0 when the table is disabled)."""
    bad = ctypes.c_uint64(0)
    _check(lib().coa_self_test(device, ctypes.byref(bad)))
    return bad.value


def verify_strict_many(msgs, pks, sigs):
    """msgs: uint8 [n, msg_len]; pks [n, 32]; sigs [n, 64] -> uint8 verdicts
    (0 = Ok, 1 = Err) from the HIP verify_strict kernel."""
    msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
    pks = np.ascontiguousarray(pks, dtype=np.uint8)
    sigs = np.ascontiguousarray(sigs, dtype=np.uint8)
    n = pks.shape[0]
    assert pks.shape == (n, 32) and sigs.shape == (n, 64) and msgs.shape[0] == n
    msg_len = msgs.shape[1] if msgs.ndim == 2 else 0
    out = np.ones(n, np.uint8)
    _check(lib().coa_ed25519_verify_strict_many(_u8p(msgs), msg_len, _u8p(pks), _u8p(sigs), n, _u8p(out)))
    return out


def verify_batch_groups(msgs, pks, sigs, group_offsets, zs=None, rng_seed=0):
    """One verdict per group (certificate).  zs: optional uint8 [n_votes, 16]
    explicit weights (parity tests); otherwise derived from rng_seed."""
    msgs = np.ascontiguousarray(msgs, dtype=np.uint8).reshape(-1, 32)
    pks = np.ascontiguousarray(pks, dtype=np.uint8).reshape(-1, 32)
    sigs = np.ascontiguousarray(sigs, dtype=np.uint8).reshape(-1, 64)
    offs = np.ascontiguousarray(group_offsets, dtype=np.uint64)
    ng = msgs.shape[0]
    assert offs.shape == (ng + 1,) and int(offs[-1]) == pks.shape[0] == sigs.shape[0]
    out = np.ones(ng, np.uint8)
    P64 = ctypes.POINTER(ctypes.c_uint64)
    op = offs.ctypes.data_as(P64)
    if zs is not None:
        zs = np.ascontiguousarray(zs, dtype=np.uint8).reshape(-1, 16)
        assert zs.shape[0] == pks.shape[0]
        _check(lib().coa_ed25519_verify_batch_groups_z(_u8p(msgs), _u8p(pks), _u8p(sigs), op, ng, _u8p(zs), _u8p(out)))
    else:
        _check(lib().coa_ed25519_verify_batch_groups(_u8p(msgs), _u8p(pks), _u8p(sigs), op, ng, _u8p(out), rng_seed))
    return out


def sha512_many(messages):
    """list of bytes -> uint8 [n, 64] SHA-512 digests (HIP kernel)."""
    n = len(messages)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum([len(m) for m in messages]) if n else []
    data = np.frombuffer(b"".join(bytes(m) for m in messages) + b"\0", np.uint8).copy()
    out = np.zeros((n, 64), np.uint8)
    _check(lib().coa_sha512_many(_u8p(data), offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n, _u8p(out)))
    return out


def digest_many(messages):
    """crypto::Digest of each message: Sha512(bytes)[..32]."""
    return [Digest(bytes(r[:32])) for r in sha512_many(messages)]


def sign_many(seeds, msgs):
    """RFC 8032 keypairs + signatures on the device: seeds uint8 [n, 32],
    msgs [n, msg_len] -> (pks [n, 32], sigs [n, 64])."""
    seeds = np.ascontiguousarray(seeds, dtype=np.uint8)
    msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
    n = seeds.shape[0]
    msg_len = msgs.shape[1] if msgs.ndim == 2 else 0
    pks = np.zeros((n, 32), np.uint8)
    sigs = np.zeros((n, 64), np.uint8)
    _check(lib().coa_ed25519_sign_many(_u8p(seeds), _u8p(msgs), msg_len, n, _u8p(pks), _u8p(sigs)))
    return pks, sigs


def public_keys(seeds):
    seeds = np.ascontiguousarray(seeds, dtype=np.uint8)
    n = seeds.shape[0]
    pks = np.zeros((n, 32), np.uint8)
    _check(lib().coa_ed25519_public_keys(_u8p(seeds), n, _u8p(pks)))
    return pks


# ----------------------------------------------------------- device level
def verify_workspace_bytes(n):
    return lib().coa_verify_workspace_bytes(n)


def verify_batch_workspace_bytes(n):
    return lib().coa_verify_batch_workspace_bytes(n)


def verify_batch_device(device, msg, pks, sigs, verdict, zs=None, rng_seed=0, workspace=None, stream=None):
    """Enqueue the Pippenger batch equation over ONE group of HBM-resident
    torch uint8 tensors (msg [32], pks [n, 32], sigs [n, 64], zs [n, 16] or
    None); verdict[0] = 0 Ok / 1 Err."""
    import torch

    if stream is None:
        stream = torch.cuda.current_stream(device)
    handle = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    n = pks.shape[0]
    assert tuple(sigs.shape) == (n, 64) and msg.numel() == 32
    zp = zs.data_ptr() if zs is not None else None
    if zs is not None:
        assert tuple(zs.shape) == (n, 16)
    ws = workspace.data_ptr() if workspace is not None else None
    wsb = workspace.numel() * workspace.element_size() if workspace is not None else 0
    _check(lib().coa_ed25519_verify_batch_device(device, msg.data_ptr(), pks.data_ptr(), sigs.data_ptr(), n, zp,
                                                 rng_seed, verdict.data_ptr(), ws, wsb, handle))


def verify_strict_many_device(device, msgs, pks, sigs, verdicts, workspace=None, stream=None):
    """Enqueue verification of HBM-resident torch uint8 tensors on `stream`
    (a torch.cuda.Stream or raw handle; None = current torch stream)."""
    import torch

    if stream is None:
        stream = torch.cuda.current_stream(device)
    handle = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    n = pks.shape[0]
    msg_len = msgs.shape[1] if msgs.dim() == 2 else 0
    ws = workspace.data_ptr() if workspace is not None else None
    _check(lib().coa_ed25519_verify_strict_many_device(device, msgs.data_ptr(), msg_len, pks.data_ptr(),
                                                       sigs.data_ptr(), n, verdicts.data_ptr(), ws, handle))


def _handle(device, stream):
    import torch

    if stream is None:
        stream = torch.cuda.current_stream(device)
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else stream


def fe_rows_check_device(device, values, out, stream=None):
    """Row-parallel field arithmetic self-test: values uint8 [n, 32] on the
    device, out int32 [n] on the device (0 = every row-parallel result equals
    the one-lane result for that input)."""
    n = values.shape[0]
    assert values.is_contiguous() and tuple(values.shape) == (n, 32) and out.numel() >= n
    _check(lib().coa_fe_rows_check_device(device, values.data_ptr(), n, out.data_ptr(), _handle(device, stream)))


def challenge_many_device(device, msgs, pks, sigs, k_out, stream=None):
    """k_out[i] = SHA-512(R_i || A_i || M_i) mod l (uint8 [n, 32] tensor)."""
    n = pks.shape[0]
    msg_len = msgs.shape[1] if msgs.dim() == 2 else 0
    _check(lib().coa_ed25519_challenge_many_device(device, msgs.data_ptr(), msg_len, pks.data_ptr(), sigs.data_ptr(),
                                                   n, k_out.data_ptr(), _handle(device, stream)))


def verify_prehashed_many_device(device, k, pks, sigs, verdicts, workspace=None, stream=None):
    n = pks.shape[0]
    ws = workspace.data_ptr() if workspace is not None else None
    _check(lib().coa_ed25519_verify_prehashed_many_device(device, k.data_ptr(), pks.data_ptr(), sigs.data_ptr(), n,
                                                          verdicts.data_ptr(), ws, _handle(device, stream)))


def sign_many_device(device, seeds, msgs, pks_out, sigs_out, stream=None):
    import torch

    if stream is None:
        stream = torch.cuda.current_stream(device)
    handle = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    n = seeds.shape[0]
    msg_len = msgs.shape[1] if msgs.dim() == 2 else 0
    _check(lib().coa_ed25519_sign_many_device(device, seeds.data_ptr(), msgs.data_ptr(), msg_len, n,
                                              pks_out.data_ptr(), sigs_out.data_ptr(), handle))


def sha512_many_device(device, data, offsets, out64, stream=None):
    import torch

    if stream is None:
        stream = torch.cuda.current_stream(device)
    handle = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    n = offsets.shape[0] - 1
    _check(lib().coa_sha512_many_device(device, data.data_ptr(), offsets.data_ptr(), n, out64.data_ptr(), handle))


# ------------------------------------------- committee cache / certificates
CERT_BAD_HEADER_ID, CERT_BAD_HEADER_SIG, CERT_BAD_VOTES = 1, 2, 4
CERT_NEEDS_EXACT, CERT_UNCACHED = 8, 16  # raw device status bits only
KEY_DECOMPRESSES, KEY_SMALL_ORDER, KEY_TORSION_FREE = 1, 2, 4


def committee_register(pks):
    """Register the committee's public keys (f2 key cache); returns the number
    of distinct keys.  Verdict-neutral."""
    pks = np.ascontiguousarray(np.asarray(pks, dtype=np.uint8).reshape(-1, 32))
    return _check(lib().coa_committee_register(_u8p(pks), pks.shape[0]))


def committee_key_flags():
    """Flags of the registered keys, in the engine's sorted key order."""
    n = _check(lib().coa_committee_key_flags(None, 0))
    out = np.zeros(max(n, 1), np.uint32)
    _check(lib().coa_committee_key_flags(out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n))
    return out[:n]


def _u64p(a):
    return a.ctypes.data


def certificate_verify_many(header_inputs, ids, origins, header_sigs, rounds, vote_pks, vote_sigs, vote_offsets,
                            rng_seed=0):
    """Crypto of Certificate::verify for n certificates (fused kernel for the
    registered committee, exact fallbacks otherwise).  Returns uint8 [n] of
    CERT_BAD_* bits (0 = every crypto check Ok)."""
    n = len(header_inputs)
    hdata = np.frombuffer(b"".join(header_inputs), np.uint8) if n else np.zeros(0, np.uint8)
    hoff = np.zeros(n + 1, np.uint64)
    hoff[1:] = np.cumsum([len(h) for h in header_inputs])
    ids = np.ascontiguousarray(ids, dtype=np.uint8)
    origins = np.ascontiguousarray(origins, dtype=np.uint8)
    hsigs = np.ascontiguousarray(header_sigs, dtype=np.uint8)
    rounds = np.ascontiguousarray(np.broadcast_to(np.asarray(rounds, np.uint64), (n,)))
    vpks = np.ascontiguousarray(vote_pks, dtype=np.uint8)
    vsigs = np.ascontiguousarray(vote_sigs, dtype=np.uint8)
    voff = np.ascontiguousarray(vote_offsets, dtype=np.uint64)
    out = np.zeros(max(n, 1), np.uint8)
    _check(lib().coa_certificate_verify_many(_u8p(hdata), _u64p(hoff), _u8p(ids), _u8p(origins), _u8p(hsigs),
                                             _u64p(rounds), _u8p(vpks), _u8p(vsigs), _u64p(voff), n, rng_seed,
                                             _u8p(out)))
    return out[:n]


def certificate_verify(header_input, id_, origin, header_sig, round_, vote_pks, vote_sigs, rng_seed=0):
    """One certificate through the latency path; returns the CERT_BAD_* bits."""
    h, i, o, s = bytes(header_input), bytes(id_), bytes(origin), bytes(header_sig)
    if len(i) != 32 or len(o) != 32 or len(s) != 64:
        raise ValueError("id/origin are 32 bytes, the header signature 64")
    vp = np.ascontiguousarray(vote_pks, dtype=np.uint8)
    vs = np.ascontiguousarray(vote_sigs, dtype=np.uint8)
    nv = vp.size // 32
    if vs.size != 64 * nv:
        raise ValueError("one 64-byte signature per 32-byte vote key")
    return _check(lib().coa_certificate_verify(h, len(h), i, o, s, round_, vp.ctypes.data if nv else None,
                                               vs.ctypes.data if nv else None, nv, rng_seed))


def certificate_workspace_bytes(n, n_votes):
    return lib().coa_certificate_workspace_bytes(n, n_votes)


def certificate_verify_many_device(device, hdata, hoff, ids, origins, hsigs, rounds, vpks, vsigs, voff, status,
                                   stream=None, workspace=None):
    """Device-resident certificates (torch tensors); raw status words (uint32
    tensor [n]) enqueued on `stream`.  workspace: None (engine-owned; the call
    waits for the stream) or a device tensor of certificate_workspace_bytes."""
    n = ids.shape[0]
    nv = vpks.shape[0]
    ws = workspace.data_ptr() if workspace is not None else None
    _check(lib().coa_certificate_verify_many_device(device, hdata.data_ptr(), hoff.data_ptr(), ids.data_ptr(),
                                                    origins.data_ptr(), hsigs.data_ptr(), rounds.data_ptr(),
                                                    vpks.data_ptr(), vsigs.data_ptr(), voff.data_ptr(), n, nv,
                                                    status.data_ptr(), ws, _handle(device, stream)))


# ------------------------------------------------------------- wire (f4)
MSG_HEADER, MSG_VOTE, MSG_CERTIFICATE, MSG_CERT_REQUEST = 0, 1, 2, 3
WIRE_ETRUNC, WIRE_EFORMAT, WIRE_EKEY = -10, -11, -12


def _frames(frames):
    data = np.frombuffer(b"".join(bytes(f) for f in frames), np.uint8) if frames else np.zeros(0, np.uint8)
    offs = np.zeros(len(frames) + 1, np.uint64)
    offs[1:] = np.cumsum([len(f) for f in frames])
    return (data if data.size else np.zeros(1, np.uint8)), offs


def wire_scan(frames):
    """bincode PrimaryMessage frames -> (kinds int32 [n], header digest input
    bytes [n], vote counts [n]); kinds are MSG_* or negative WIRE_E*."""
    n = len(frames)
    data, offs = _frames(frames)
    kinds = np.zeros(max(n, 1), np.int32)
    hb = np.zeros(max(n, 1), np.uint64)
    nv = np.zeros(max(n, 1), np.uint64)
    _check(lib().coa_wire_scan(_u8p(data), _u64p(offs), n, kinds.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                               _u64p(hb), _u64p(nv)))
    return kinds[:n], hb[:n], nv[:n]


def wire_decode_certificates(frames):
    """Certificate frames -> the arguments of certificate_verify_many:
    dict(header_inputs, ids, origins, header_sigs, rounds, vote_pks, vote_sigs, vote_offsets)."""
    n = len(frames)
    kinds, hb, nv = wire_scan(frames)
    if n and (kinds != MSG_CERTIFICATE).any():
        raise ValueError("not all frames are well-formed Certificate messages")
    data, offs = _frames(frames)
    hd = np.zeros(max(int(hb.sum()), 1), np.uint8)
    hoff = np.zeros(n + 1, np.uint64)
    ids, origins = np.zeros((n, 32), np.uint8), np.zeros((n, 32), np.uint8)
    hsigs, rounds = np.zeros((n, 64), np.uint8), np.zeros(n, np.uint64)
    tv = int(nv.sum())
    vp, vs = np.zeros((max(tv, 1), 32), np.uint8), np.zeros((max(tv, 1), 64), np.uint8)
    voff = np.zeros(n + 1, np.uint64)
    pc = np.zeros(max(n, 1), np.uint32)
    _check(lib().coa_wire_decode_certificates(_u8p(data), _u64p(offs), n, _u8p(hd), _u64p(hoff), _u8p(ids),
                                              _u8p(origins), _u8p(hsigs), _u64p(rounds), _u8p(vp), _u8p(vs),
                                              _u64p(voff), pc.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))))
    hdr = [bytes(hd[int(hoff[i]):int(hoff[i + 1])]) for i in range(n)]
    return {"header_inputs": hdr, "ids": ids, "origins": origins, "header_sigs": hsigs, "rounds": rounds,
            "vote_pks": vp[:tv], "vote_sigs": vs[:tv], "vote_offsets": voff, "payload_counts": pc[:n]}


def wire_decode_votes(frames):
    n = len(frames)
    data, offs = _frames(frames)
    ids, origins, authors = (np.zeros((n, 32), np.uint8) for _ in range(3))
    rounds, sigs = np.zeros(n, np.uint64), np.zeros((n, 64), np.uint8)
    _check(lib().coa_wire_decode_votes(_u8p(data), _u64p(offs), n, _u8p(ids), _u64p(rounds), _u8p(origins),
                                       _u8p(authors), _u8p(sigs)))
    return {"ids": ids, "rounds": rounds, "origins": origins, "authors": authors, "sigs": sigs}


def wire_decode_headers(frames):
    n = len(frames)
    _, hb, _ = wire_scan(frames)
    data, offs = _frames(frames)
    hd = np.zeros(max(int(hb.sum()), 1), np.uint8)
    hoff = np.zeros(n + 1, np.uint64)
    ids, authors = np.zeros((n, 32), np.uint8), np.zeros((n, 32), np.uint8)
    sigs, rounds = np.zeros((n, 64), np.uint8), np.zeros(n, np.uint64)
    pc = np.zeros(max(n, 1), np.uint32)
    _check(lib().coa_wire_decode_headers(_u8p(data), _u64p(offs), n, _u8p(hd), _u64p(hoff), _u8p(ids),
                                         _u8p(authors), _u8p(sigs), _u64p(rounds),
                                         pc.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))))
    return {"header_inputs": [bytes(hd[int(hoff[i]):int(hoff[i + 1])]) for i in range(n)], "ids": ids,
            "authors": authors, "sigs": sigs, "rounds": rounds, "payload_counts": pc[:n]}


# --------------------------------------------------------- aggregation queue
class AggregationQueue:
    """Python face of the native coalescing stage (coa_queue_*): submit
    header/vote signatures, certificate vote batches, whole certificates and
    worker batch digests from any thread, get a concurrent.futures.Future per
    request -- True (Ok) / False (Err) for signatures and vote batches, the
    CERT_BAD_* bits for certificates, the 32-byte Digest for digests; the
    engine error status raises EngineError in the future."""

    def __init__(self, max_batch=65536, max_delay_us=500):
        import concurrent.futures as cf
        import threading

        self._cf = cf
        self._lock = threading.Lock()
        self._pending = {}
        self._borrowed = {}  # key -> arrays a borrowed request's queue entry points into
        self._next = 1
        self._cb = VERDICT_CB(self._on_verdict)  # keep alive for the queue's lifetime
        self._q = lib().coa_queue_create(max_batch, max_delay_us)

    def _on_verdict(self, user, status, verdicts, n):
        with self._lock:
            fut, kind = self._pending.pop(user)
            self._borrowed.pop(user, None)  # a borrowed request's arrays: the queue is done with them
        if status < 0:
            fut.set_exception(EngineError(f"{_ERRORS.get(status, status)}"))
        elif kind == "digest":
            fut.set_result(Digest(bytes(verdicts[:32])))
        elif kind == "certificate":
            fut.set_result(int(verdicts[0]))
        else:
            fut.set_result(verdicts[0] == 0)

    def _register(self, kind="verdict"):
        fut = self._cf.Future()
        with self._lock:
            key = self._next
            self._next += 1
            self._pending[key] = (fut, kind)
        return key, fut

    def _submitted(self, key, rc):
        if rc < 0:
            with self._lock:
                self._pending.pop(key, None)
            _check(rc)

    def submit_certificate(self, header_input, id_, origin, header_sig, round_, votes, borrow=False):
        """Future of the certificate's CERT_BAD_* bits (0 = all crypto Ok).
        borrow=True submits through coa_queue_submit_certificate_borrowed: the
        arrays built here are kept alive until the callback (no intake copy)."""
        key, fut = self._register("certificate")
        votes = list(votes)
        h = np.frombuffer(bytes(header_input), np.uint8).copy() if len(header_input) else np.zeros(1, np.uint8)
        i = np.frombuffer(bytes(id_), np.uint8).copy()
        o = np.frombuffer(bytes(origin), np.uint8).copy()
        sg = np.frombuffer(header_sig.flatten() if isinstance(header_sig, Signature) else bytes(header_sig),
                           np.uint8).copy()
        pks = _bytes_array([bytes(pk) for pk, _ in votes], 32) if votes else np.zeros(32, np.uint8)
        sgs = _bytes_array([s.flatten() for _, s in votes], 64) if votes else np.zeros(64, np.uint8)
        if borrow:
            with self._lock:
                self._borrowed[key] = (h, i, o, sg, pks, sgs)
        submit = lib().coa_queue_submit_certificate_borrowed if borrow else lib().coa_queue_submit_certificate
        rc = submit(self._q, _u8p(h), len(header_input), _u8p(i), _u8p(o), _u8p(sg), round_, _u8p(pks), _u8p(sgs),
                    len(votes), self._cb, key)
        if rc < 0:
            with self._lock:
                self._borrowed.pop(key, None)
        self._submitted(key, rc)
        return fut

    def submit_digest(self, data):
        """Future of Digest(Sha512(data)[..32]) (worker/src/processor.rs:38)."""
        key, fut = self._register("digest")
        buf = np.frombuffer(bytes(data), np.uint8).copy() if len(data) else np.zeros(1, np.uint8)
        rc = lib().coa_queue_submit_digest(self._q, _u8p(buf), len(data), self._cb, key)
        self._submitted(key, rc)
        return fut

    def submit_verify(self, digest, public_key, signature):
        key, fut = self._register()
        d = np.frombuffer(bytes(digest), np.uint8).copy()
        pk = np.frombuffer(bytes(public_key), np.uint8).copy()
        sg = np.frombuffer(signature.flatten() if isinstance(signature, Signature) else bytes(signature),
                           np.uint8).copy()
        rc = lib().coa_queue_submit_verify(self._q, _u8p(d), _u8p(pk), _u8p(sg), self._cb, key)
        if rc < 0:
            with self._lock:
                self._pending.pop(key, None)
            _check(rc)
        return fut

    def submit_batch(self, digest, votes):
        key, fut = self._register()
        votes = list(votes)
        d = np.frombuffer(bytes(digest), np.uint8).copy()
        pks = _bytes_array([bytes(pk) for pk, _ in votes], 32) if votes else np.zeros(32, np.uint8)
        sgs = _bytes_array([s.flatten() for _, s in votes], 64) if votes else np.zeros(64, np.uint8)
        rc = lib().coa_queue_submit_batch(self._q, _u8p(d), _u8p(pks), _u8p(sgs), len(votes), self._cb, key)
        if rc < 0:
            with self._lock:
                self._pending.pop(key, None)
            _check(rc)
        return fut

    def flush(self):
        _check(lib().coa_queue_flush(self._q))

    def stats(self):
        a, b, c, d = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().coa_queue_stats(self._q, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        _check(lib().coa_queue_digest_count(self._q, ctypes.byref(d)))
        return {"launches": a.value, "signatures": b.value, "batches": c.value, "digests": d.value}

    def set_idle_launch(self, windows_in_flight=1):
        """coa_queue_set_idle_launch: also close a window at once while fewer
        than windows_in_flight windows are in flight (0 = deadline policy)."""
        _check(lib().coa_queue_set_idle_launch(self._q, windows_in_flight))

    def metrics(self):
        """coa_queue_metrics: request counts per kind, window sizes, windows in
        flight (double buffering), pending depth and submit -> callback wait
        times in microseconds."""
        m = QueueMetrics()
        _check(lib().coa_queue_metrics(self._q, ctypes.byref(m)))
        return metrics_dict(m)

    def metrics_reset(self):
        """coa_queue_metrics_reset: start a new measurement interval."""
        _check(lib().coa_queue_metrics_reset(self._q))

    def close(self):
        if self._q:
            lib().coa_queue_destroy(self._q)
            self._q = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

"""ctypes loader for the C oracle (oracle/coa_oracle.c) -- TEST INFRASTRUCTURE
and CPU BASELINE ONLY.  Builds oracle/_build/*.so with gcc on first use."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")
_libs = {}


def build():
    pairs = [("coa_oracle.c", "libcoa_oracle.so"), ("coa_oracle.c", "libcoa_oracle_count.so"),
             ("sodium_drive.c", "libcoa_sodium_drive.so")]
    if all(os.path.exists(os.path.join(BUILD, o))
           and os.path.getmtime(os.path.join(BUILD, o)) >= os.path.getmtime(os.path.join(HERE, s))
           for s, o in pairs):
        return
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib(count=False):
    key = "count" if count else "plain"
    if key not in _libs:
        build()
        L = ctypes.CDLL(os.path.join(BUILD, "libcoa_oracle_count.so" if count else "libcoa_oracle.so"))
        P8 = ctypes.c_void_p  # numpy addresses (_p) or bytes objects, no pointer objects
        sz = ctypes.c_size_t
        L.coa_oracle_verify_strict.argtypes = [P8, sz, P8, P8]
        L.coa_oracle_verify_strict.restype = ctypes.c_int
        L.coa_oracle_verify_batch.argtypes = [P8, sz, P8, P8, sz, P8]
        L.coa_oracle_verify_batch.restype = ctypes.c_int
        L.coa_oracle_verify_strict_many.argtypes = [P8, sz, P8, P8, sz, P8, ctypes.c_int]
        L.coa_oracle_verify_strict_many.restype = None
        L.coa_oracle_sha512.argtypes = [P8, sz, P8]
        L.coa_oracle_sha512.restype = None
        L.coa_oracle_sha512_many_mt.argtypes = [P8, ctypes.c_void_p, sz, P8, ctypes.c_int]
        L.coa_oracle_sha512_many_mt.restype = None
        L.coa_oracle_certificate_verify_many.argtypes = [P8, P8, P8, P8, P8, P8, P8, P8, P8, P8, sz, P8, ctypes.c_int]
        L.coa_oracle_certificate_verify_many.restype = None
        if count:
            L.coa_oracle_counts.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 2
            L.coa_oracle_reset_counts.argtypes = []
        _libs[key] = L
    return _libs[key]


SODIUM = "/opt/conda/lib/libsodium.so"


def sodium_verify_many(msgs, pks, sigs, nthreads=1, path=SODIUM):
    """libsodium crypto_sign_verify_detached over rows (second CPU reference,
    bench.py only).  Returns (out, version) or None when libsodium is absent."""
    if "sodium" not in _libs:
        build()
        L = ctypes.CDLL(os.path.join(BUILD, "libcoa_sodium_drive.so"))
        P8 = ctypes.c_void_p
        L.coa_sodium_verify_many.argtypes = [ctypes.c_char_p, P8, ctypes.c_size_t, P8, P8, ctypes.c_size_t, P8,
                                             ctypes.c_int, ctypes.POINTER(ctypes.c_char_p)]
        L.coa_sodium_verify_many.restype = ctypes.c_int
        _libs["sodium"] = L
    msgs, pks, sigs = (np.ascontiguousarray(a, dtype=np.uint8) for a in (msgs, pks, sigs))
    n = pks.shape[0]
    out = np.zeros(n, np.uint8)
    ver = ctypes.c_char_p()
    rc = _libs["sodium"].coa_sodium_verify_many(path.encode(), _p(msgs), msgs.shape[1], _p(pks), _p(sigs), n,
                                                _p(out), nthreads, ctypes.byref(ver))
    if rc != 0:
        return None
    return out, ver.value.decode()


def _p(a):
    return a.ctypes.data


def _arr(b):
    return np.frombuffer(bytes(b), np.uint8).copy() if len(b) else np.zeros(1, np.uint8)


def verify_strict(msg, pk, sig, L=None):
    L = L or lib()
    m = bytes(msg)
    return L.coa_oracle_verify_strict(m if m else b"\0", len(m), bytes(pk), bytes(sig)) == 0


def verify_batch(msg, pks, sigs, zs):
    n = len(pks)
    m = bytes(msg)
    P = b"".join(bytes(p) for p in pks) or b"\0"
    S = b"".join(bytes(s) for s in sigs) or b"\0"
    Z = b"".join(z.to_bytes(16, "little") for z in zs) or b"\0"
    return lib().coa_oracle_verify_batch(m if m else b"\0", len(m), P, S, n, Z) == 0


def verify_strict_many(msgs, pks, sigs, nthreads=1):
    msgs = np.ascontiguousarray(msgs, np.uint8)
    pks = np.ascontiguousarray(pks, np.uint8)
    sigs = np.ascontiguousarray(sigs, np.uint8)
    n = pks.shape[0]
    out = np.ones(n, np.uint8)
    lib().coa_oracle_verify_strict_many(_p(msgs), msgs.shape[1], _p(pks), _p(sigs), n, _p(out), nthreads)
    return out


def sha512(data):
    d = bytes(data)
    out = ctypes.create_string_buffer(64)
    lib().coa_oracle_sha512(d if d else b"\0", len(d), out)
    return out.raw


def field_op_counts(msg, pk, sig):
    """(fe_mul, fe_sq) count of one verify_strict in the dalek algorithm."""
    L = lib(count=True)
    L.coa_oracle_reset_counts()
    m, p, s = _arr(msg), _arr(pk), _arr(sig)
    L.coa_oracle_verify_strict(_p(m), len(msg), _p(p), _p(s))
    a, b = ctypes.c_uint64(), ctypes.c_uint64()
    L.coa_oracle_counts(ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def sha512_many(data, offsets, nthreads=1):
    """data: uint8 array, offsets: uint64 [n+1] -> uint8 [n, 64]."""
    data = np.ascontiguousarray(data, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = offsets.shape[0] - 1
    out = np.zeros((n, 64), np.uint8)
    lib().coa_oracle_sha512_many_mt(_p(data), offsets.ctypes.data, n, _p(out), nthreads)
    return out


def certificate_verify(header_input, header_id, author, header_sig, round_, vote_pks, vote_sigs, zs):
    """Certificate::verify crypto as the reference runs it on one core:
    Header::digest == id, Signature::verify(id, author), Certificate::digest,
    verify_batch(digest, votes) (primary/src/messages.rs:48-84,189-234)."""
    import struct as _st

    if sha512(header_input)[:32] != bytes(header_id):
        return False
    if not verify_strict(bytes(header_id), bytes(author), bytes(header_sig)):
        return False
    d = sha512(bytes(header_id) + _st.pack("<Q", round_) + bytes(author))[:32]
    return verify_batch(d, [bytes(p) for p in vote_pks], [bytes(s) for s in vote_sigs], zs)


def certificate_verify_many(header_inputs, ids, origins, header_sigs, rounds, vote_pks, vote_sigs, vote_offsets, zs,
                            nthreads=1):
    """Certificate::verify crypto for n certificates on nthreads C threads:
    uint8 [n] of bits 1 (header id), 2 (header signature), 4 (vote batch with
    the given weights zs, uint8 [n_votes, 16]), each check independent."""
    n = len(header_inputs)
    hdata = np.frombuffer(b"".join(bytes(h) for h in header_inputs) + b"\0", np.uint8).copy()
    hoff = np.zeros(n + 1, np.uint64)
    hoff[1:] = np.cumsum([len(h) for h in header_inputs])
    a = [np.ascontiguousarray(x, np.uint8) for x in (ids, origins, header_sigs)]
    r = np.ascontiguousarray(np.broadcast_to(np.asarray(rounds, np.uint64), (n,)))
    vp, vs, z = (np.ascontiguousarray(x, np.uint8) for x in (vote_pks, vote_sigs, zs))
    voff = np.ascontiguousarray(vote_offsets, np.uint64)
    out = np.zeros(max(n, 1), np.uint8)
    lib().coa_oracle_certificate_verify_many(_p(hdata), _p(hoff), _p(a[0]), _p(a[1]), _p(a[2]), _p(r), _p(vp), _p(vs),
                                             _p(voff), _p(z), n, _p(out), nthreads)
    return out[:n]

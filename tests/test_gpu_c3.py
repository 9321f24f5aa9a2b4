"""C3 at its stated size (BASELINE.json configs[2]): one round
of 10,000 certificates of a committee of 100 (67 votes each, 3,336-byte
headers), with injected failures of every crypto kind, through the engine's
Certificate::verify crypto (coa_certificate_verify_many: fused kernel over the
registered committee, exact fallbacks for keys outside it) and compared status
bit for status bit with the C restatement of dalek run the reference's way,
per certificate (oracle/coa_oracle.c coa_oracle_certificate_verify_many:
Header::digest == id, Signature::verify(id, author),
verify_batch(Certificate::digest, votes), each check evaluated on its own --
primary/src/messages.rs:48-84,189-234).  The round runs with the fused
kernel's jobs in key order (the default) and in certificate order."""
import os
import struct

import numpy as np
import pytest

import coa_oracle as co

pytestmark = pytest.mark.gpu

L_ORDER = 2 ** 252 + 27742317777372353535851937790883648493
SMALL_ORDER_R = bytes.fromhex("c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a")
OFF_CURVE = (2).to_bytes(32, "little")
KINDS = ("header_byte", "header_sig_flip", "header_sig_small_R", "vote_sig_flip", "vote_s_plus_l",
         "vote_small_R", "vote_foreign_key_valid", "vote_wrong_member_key", "vote_off_curve_key",
         "author_outside_committee_valid")


@pytest.fixture(scope="module")
def c3_round(engine):
    """The 10k-certificate round of a committee of 100 with 300 injected
    failures (KINDS, 30 of each), as arrays; the committee registered."""
    import certificates as C
    import workloads

    n = 10_000
    committee, b = C.synth_certificates(n, committee_size=100, n_payload=32, seed=3)
    assert committee.register() == 100
    hin = list(b.header_inputs)
    ids, authors, hsigs = b.ids.copy(), b.authors.copy(), b.header_sigs.copy()
    vpks, vsigs = b.vote_pks.copy(), b.vote_sigs.copy()
    rng = np.random.default_rng(0xC3)
    victims = rng.permutation(n)[:300]
    kind_of = {}
    for j, c in enumerate(victims):
        c = int(c)
        k = j % len(KINDS)
        kind_of[c] = k
        lo = int(b.offsets[c])
        v = lo + int(rng.integers(0, 67))
        if k == 0:
            h = bytearray(hin[c]); h[100 + j % 3000] ^= 0x10; hin[c] = bytes(h)
        elif k == 1:
            hsigs[c, 40] ^= 1
        elif k == 2:
            hsigs[c, :32] = np.frombuffer(SMALL_ORDER_R, np.uint8)
        elif k == 3:
            vsigs[v, 5] ^= 0x80
        elif k == 4:
            s = int.from_bytes(bytes(vsigs[v, 32:]), "little") + L_ORDER
            vsigs[v, 32:] = np.frombuffer(s.to_bytes(32, "little"), np.uint8)
        elif k == 5:
            vsigs[v, :32] = np.frombuffer(SMALL_ORDER_R, np.uint8)
        elif k == 6:  # a valid signature by a key outside the committee: Ok crypto (uncached kernels)
            p, s = engine.sign_many(workloads.key_seeds(1, start=10 ** 6 + c), b.cert_digests[c:c + 1])
            vpks[v], vsigs[v] = p[0], s[0]
        elif k == 7:  # another member's key under this vote's signature
            vpks[v] = vpks[lo + (v - lo + 1) % 67]
        elif k == 8:
            vpks[v] = np.frombuffer(OFF_CURVE, np.uint8)
        else:  # header re-authored by a key outside the committee, every signature valid
            seed = workloads.key_seeds(1, start=2 * 10 ** 6 + c)
            apk = engine.public_keys(seed)[0]
            h = bytes(apk) + hin[c][32:]
            hin[c] = h
            ids[c] = engine.sha512_many([h])[0, :32]
            authors[c] = apk
            _, hs = engine.sign_many(seed, ids[c:c + 1])
            hsigs[c] = hs[0]
            cd = engine.sha512_many([bytes(ids[c]) + struct.pack("<Q", b.round) + bytes(apk)])[0, :32]
            vseeds = workloads.key_seeds(100)[(c + np.arange(67)) % 100]
            p, s = engine.sign_many(vseeds, np.tile(cd, (67, 1)))
            vpks[lo:lo + 67], vsigs[lo:lo + 67] = p, s
    return dict(n=n, committee=committee, b=b, hin=hin, ids=ids, authors=authors, hsigs=hsigs, vpks=vpks,
                vsigs=vsigs, victims=victims, kind_of=kind_of)


# what each injected kind does to the COA_CERT_* bits (1 header id, 2 header
# signature, 4 votes); kinds 6 and 9 are valid crypto with keys outside the
# committee (the exact fallbacks decide them)
WANT = {0: 1, 1: 2, 2: 2, 3: 4, 4: 4, 5: 4, 6: 0, 7: 4, 8: 4, 9: 0}


@pytest.mark.timeout(600)
def test_c3_round_full_size_with_injected_failures(engine, monkeypatch, c3_round):
    r = c3_round
    n, b, hin, ids, authors, hsigs, vpks, vsigs = (r[k] for k in ("n", "b", "hin", "ids", "authors", "hsigs", "vpks",
                                                                  "vsigs"))
    victims, kind_of = r["victims"], r["kind_of"]
    assert r["committee"].register() == 100
    rounds = np.full(n, b.round, np.uint64)
    got = engine.certificate_verify_many(hin, ids, authors, hsigs, rounds, vpks, vsigs, b.offsets, rng_seed=17)
    # the same round with the fused kernel's jobs in key order
    # (k_job_count/k_job_place; COA_CERT_PIPE_KEYSORT=1 asks for it on the
    # host path's chunks): every status word is the same
    monkeypatch.setenv("COA_CERT_PIPE_KEYSORT", "1")
    keyed = engine.certificate_verify_many(hin, ids, authors, hsigs, rounds, vpks, vsigs, b.offsets, rng_seed=17)
    monkeypatch.delenv("COA_CERT_PIPE_KEYSORT")
    assert (keyed == got).all()
    # device-resident (coa_certificate_verify_many_device, the fused kernel's
    # raw status words, key order by default): the same words in certificate
    # order (COA_CERT_KEYSORT=0), and Ok exactly where the host path says Ok
    # and the fused kernel could decide (no key outside the committee)
    import torch

    dev = torch.device("cuda:0")
    hd = np.frombuffer(b"".join(hin) + bytes(16), np.uint8)
    hoff = np.zeros(n + 1, np.int64)
    hoff[1:] = np.cumsum([len(h) for h in hin])
    t = lambda a: torch.from_numpy(np.array(a)).to(dev)  # noqa: E731
    args = (t(hd), t(hoff), t(ids), t(authors), t(hsigs), t(rounds.view(np.int64)), t(vpks), t(vsigs),
            t(b.offsets.view(np.int64)))
    raws = []
    for order in ("1", "0"):
        monkeypatch.setenv("COA_CERT_KEYSORT", order)
        status = torch.empty(n, dtype=torch.int32, device=dev)
        engine.certificate_verify_many_device(0, *args, status)
        torch.cuda.synchronize()
        raws.append(status.cpu().numpy())
    monkeypatch.delenv("COA_CERT_KEYSORT")
    assert (raws[0] == raws[1]).all()
    decided = np.array([kind_of.get(c) not in (6, 9) for c in range(n)])
    assert ((raws[0] == 0)[decided] == (got == 0)[decided]).all()

    zs = np.random.default_rng(1).integers(0, 256, (int(b.offsets[-1]), 16), dtype=np.uint8)
    exp = co.certificate_verify_many(hin, ids, authors, hsigs, b.round, vpks, vsigs, b.offsets, zs,
                                     min(16, os.cpu_count() or 1))
    mism = np.nonzero(got != exp)[0]
    assert mism.size == 0, [(int(c), kind_of.get(int(c)), int(got[c]), int(exp[c])) for c in mism[:20]]
    # every injected kind had its intended effect, untouched certificates are Ok
    for c, k in kind_of.items():
        assert got[c] == WANT[k], (c, KINDS[k], int(got[c]))
    untouched = np.setdiff1d(np.arange(n), victims)
    assert (got[untouched] == 0).all()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("borrowed", [1, 0])
def test_c3_round_streamed_through_the_queue_with_injected_failures(engine, c3_round, borrowed):
    """The same adversarial round streamed as the Rust VerifyService submits
    it: one coa_queue_submit_certificate(_borrowed) per certificate from four
    C producer threads (tools/latc.c, lib/liblatc.so), max_batch 16,384 items
    (windows of ~240 certificates, so backlog windows form), every callback's
    COA_CERT_* bits checked against the expected bits of its certificate --
    the 300 injected failures included, the certificates with keys outside
    the committee decided by the queue's resolver thread."""
    import ctypes

    r = c3_round
    n, b = r["n"], r["b"]
    assert r["committee"].register() == 100
    expect = np.zeros(n, np.uint8)
    for c, k in r["kind_of"].items():
        expect[c] = WANT[k]
    path = os.path.join(os.path.dirname(engine.LIB_PATH), "liblatc.so")
    assert os.path.exists(path), path
    lib = ctypes.CDLL(path)
    vp, sz, ci, dp = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_double)
    lib.latc_stream_certificates.argtypes = [sz, ctypes.c_uint, ci, ci, ci, ctypes.c_double] + [vp] * 9 + [sz, vp, dp,
                                                                                                          vp]
    lib.latc_stream_certificates.restype = ci
    hin = r["hin"]
    hd = np.frombuffer(b"".join(hin) + bytes(16), np.uint8)
    hoff = np.zeros(n + 1, np.uint64)
    hoff[1:] = np.cumsum([len(h) for h in hin])
    arrs = [hd, hoff, np.ascontiguousarray(r["ids"]), np.ascontiguousarray(r["authors"]),
            np.ascontiguousarray(r["hsigs"]), np.full(n, b.round, np.uint64), np.ascontiguousarray(r["vpks"]),
            np.ascontiguousarray(r["vsigs"]), np.ascontiguousarray(b.offsets)]
    el = ctypes.c_double()
    met = engine.QueueMetrics()
    wrong = lib.latc_stream_certificates(16384, 200, 4, 1, borrowed, 0.0, *[a.ctypes.data for a in arrs], n,
                                         expect.ctypes.data, ctypes.byref(el), ctypes.addressof(met))
    m = engine.metrics_dict(met)
    assert wrong == 0, (wrong, m)
    assert m["certificates"] == n and m["failed_windows"] == 0, m
    assert m["deferred_requests"] >= 30, m  # kinds 6 and 9 went through the resolver

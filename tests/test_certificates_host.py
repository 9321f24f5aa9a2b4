"""CPU: the vote checks of Certificate::verify in the bulk helper
(certificates._quorum_errors, primary/src/messages.rs:196-211) read each
voter's stake and identity from the vote keys themselves -- UnknownAuthority
for a key outside the committee, AuthorityReuse for a repeated key,
CertificateRequiresQuorum below 2N/3 + 1 of stake (config/src/lib.rs:168-173)."""
import numpy as np

import certificates as C


def _batch(vote_pks, counts):
    n = len(counts)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(counts)
    z = np.zeros((n, 32), np.uint8)
    return C.CertificateBatch([b""] * n, z, z, np.zeros((n, 64), np.uint8), z, np.asarray(vote_pks, np.uint8),
                              np.zeros((len(vote_pks), 64), np.uint8), offs, None, None, 1)


def test_quorum_errors_read_vote_keys():
    keys = [bytes([i + 1]) * 32 for i in range(4)]
    # unequal stakes: quorum = 2 * 10 // 3 + 1 = 7
    committee = C.Committee({keys[0]: 4, keys[1]: 3, keys[2]: 2, keys[3]: 1})
    assert committee.quorum_threshold() == 7
    outsider = bytes([0xEE]) * 32
    certs = [
        [keys[0], keys[1]],               # 7: Ok
        [keys[0], keys[2]],               # 6: below quorum
        [keys[0], keys[1], outsider],     # UnknownAuthority (stake 0) even with quorum reached
        [keys[0], keys[0], keys[1]],      # AuthorityReuse
        [keys[3], keys[2], keys[1], keys[0]],  # all four, any order: Ok
        [],                               # no votes: below quorum
    ]
    vp = [np.frombuffer(k, np.uint8) for c in certs for k in c]
    b = _batch(np.array(vp).reshape(-1, 32), [len(c) for c in certs])
    assert list(C._quorum_errors(b, committee)) == [0, 1, 1, 1, 0, 1]


def test_quorum_errors_match_object_path():
    """Same answers as Certificate.quorum_check on the object form."""
    keys = [bytes([7 * i + 3]) * 32 for i in range(7)]
    committee = C.Committee({k: 1 for k in keys})
    rng = np.random.default_rng(4)
    certs = []
    for _ in range(40):
        m = int(rng.integers(3, 8))
        pick = [keys[int(i)] for i in rng.integers(0, 7, m)]
        if rng.random() < 0.2:
            pick[0] = bytes([0x99]) * 32
        certs.append(pick)
    vp = np.array([np.frombuffer(k, np.uint8) for c in certs for k in c]).reshape(-1, 32)
    got = C._quorum_errors(_batch(vp, [len(c) for c in certs]), committee)
    for c, g in zip(certs, got):
        cert = C.Certificate(C.Header(), [(C.PublicKey(k), C.Signature()) for k in c])
        try:
            cert.quorum_check(committee)
            want = 0
        except C.DagError:
            want = 1
        assert g == want

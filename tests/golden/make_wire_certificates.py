"""Generate tests/golden/wire_certificates.bin: bincode PrimaryMessage::Certificate
frames (as PrimaryReceiverHandler::dispatch receives them,
primary/src/primary.rs:223-244) with the COA_CERT_* status bits
Certificate::verify's crypto must give for each, for the C harness that decodes
them natively and queues them (tests/c_abi/wire_queue_harness.c).

Frames are encoded by the independent test encoder (tests/wire_codec.py) from
the reference's serde layout; keys are RFC 8032 keypairs from seeds
SHA512("wire-cert-key" || i)[..32], signatures by oracle/ed25519_ref.py.  The
expected bits come from the C restatement of dalek (oracle/coa_oracle.c
certificate_verify_many: Header::digest == id, verify_strict of the header
signature, verify_batch of the votes over Certificate::digest; no torsion
inputs here, so the batch verdict does not depend on the weights).

Format (little endian): "CQWC", u32 n_keys, n_keys x 32-byte committee key,
u32 n_frames, n_frames x {u32 len, frame, u8 expected bits}.
Usage: python tests/golden/make_wire_certificates.py
"""
import hashlib
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
sys.path.insert(0, os.path.join(HERE, ".."))
import coa_oracle as co  # noqa: E402
import ed25519_ref as o  # noqa: E402
import wire_codec as W  # noqa: E402

N_KEYS = 4          # committee (quorum 3)
N_OUTSIDE = 2       # keys outside the registered committee


def main():
    rng = random.Random(0x31CE)
    seeds = [hashlib.sha512(b"wire-cert-key" + bytes([i])).digest()[:32] for i in range(N_KEYS + N_OUTSIDE)]
    pks = [o.public_key(s) for s in seeds]
    frames, expect = [], []
    kinds = ["valid"] * 10 + ["bad_id", "bad_header_sig", "bad_vote", "bad_vote", "outside_voter", "outside_author",
                               "bad_id_and_vote", "s_high", "no_votes", "valid_4_votes"]
    for n, kind in enumerate(kinds):
        author = n % N_KEYS if kind != "outside_author" else N_KEYS
        rnd = 5 + n
        payload = [(bytes(rng.getrandbits(8) for _ in range(32)), rng.getrandbits(8) % 3) for _ in range(1 + n % 3)]
        parents = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(3)]
        hin = W.header_digest_input(pks[author], rnd, payload, parents)
        hid = hashlib.sha512(hin).digest()[:32]
        if kind in ("bad_id", "bad_id_and_vote"):
            hid = bytes([hid[0] ^ 1]) + hid[1:]
        hsig = o.sign(seeds[author], hid)
        if kind == "bad_header_sig":
            hsig = hsig[:10] + bytes([hsig[10] ^ 4]) + hsig[11:]
        cdig = hashlib.sha512(hid + struct.pack("<Q", rnd) + pks[author]).digest()[:32]
        voters = [(author + 1 + j) % N_KEYS for j in range(3)]
        if kind == "outside_voter":
            voters[2] = N_KEYS + 1
        if kind == "valid_4_votes":
            voters = list(range(N_KEYS))
        if kind == "no_votes":
            voters = []
        votes = [(pks[v], o.sign(seeds[v], cdig)) for v in voters]
        if kind in ("bad_vote", "bad_id_and_vote"):
            pk, sg = votes[n % len(votes)]
            votes[n % len(votes)] = (pk, sg[:40] + bytes([sg[40] ^ 0x10]) + sg[41:])
        if kind == "s_high":  # s + l: non-canonical, rejected by verify_batch's from_bytes
            pk, sg = votes[0]
            s = int.from_bytes(sg[32:], "little") + o.L
            votes[0] = (pk, sg[:32] + s.to_bytes(32, "little"))
        hdr = W.header(pks[author], rnd, payload, parents, hid, hsig)
        frames.append(W.primary_message(2, W.certificate(hdr, votes)))
        zs = [rng.getrandbits(128) for _ in votes]
        bits = 0
        if hashlib.sha512(hin).digest()[:32] != hid:
            bits |= 1
        if not co.verify_strict(hid, pks[author], hsig):
            bits |= 2
        d = hashlib.sha512(hid + struct.pack("<Q", rnd) + pks[author]).digest()[:32]
        if not co.verify_batch(d, [p for p, _ in votes], [s for _, s in votes], zs):
            bits |= 4
        expect.append(bits)
    out = bytearray(b"CQWC") + struct.pack("<I", N_KEYS) + b"".join(pks[:N_KEYS])
    out += struct.pack("<I", len(frames))
    for f, e in zip(frames, expect):
        out += struct.pack("<I", len(f)) + f + bytes([e])
    with open(os.path.join(HERE, "wire_certificates.bin"), "wb") as fh:
        fh.write(bytes(out))
    print(f"{len(frames)} certificate frames, expected bits {expect}")


if __name__ == "__main__":
    main()

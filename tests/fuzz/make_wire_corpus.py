"""Writes the seed corpus of the wire-decoder fuzzer (tests/fuzz/wire_fuzz.cpp):
well-formed bincode PrimaryMessage frames of every variant and a range of
sizes, encoded by the independent test encoder (tests/wire_codec.py) from the
reference's serde layout.  Deterministic (seeded); the .bin files are
committed.  usage: python tests/fuzz/make_wire_corpus.py"""
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import wire_codec as W  # noqa: E402


def main():
    rng = random.Random(0xF022)
    rb = lambda n: bytes(rng.getrandbits(8) for _ in range(n))  # noqa: E731
    out = os.path.join(HERE, "wire_corpus")
    os.makedirs(out, exist_ok=True)
    frames = []
    for n_pay, n_par, n_votes in ((0, 0, 0), (1, 1, 1), (3, 4, 3), (32, 67, 67), (2, 2, 0)):
        hdr = W.header(rb(32), rng.getrandbits(64), [(rb(32), rng.getrandbits(32)) for _ in range(n_pay)],
                       [rb(32) for _ in range(n_par)], rb(32), rb(64))
        frames.append(W.primary_message(0, hdr))
        frames.append(W.primary_message(2, W.certificate(hdr, [(rb(32), rb(64)) for _ in range(n_votes)])))
    for _ in range(3):
        frames.append(W.primary_message(1, W.vote(rb(32), rng.getrandbits(64), rb(32), rb(32), rb(64))))
    frames.append(W.primary_message(3, W.cert_request([rb(32) for _ in range(5)], rb(32))))
    # a key longer than 32 bytes (decode_base64 keeps the first 32) and a duplicate payload key
    d = rb(32)
    hdr = W.header(None, 7, [(d, 1), (d, 2)], [rb(32)], rb(32), rb(64), author_field=W.key(rb(48)))
    frames.append(W.primary_message(0, hdr))
    for i, f in enumerate(frames):
        with open(os.path.join(out, f"{i:02d}.bin"), "wb") as fh:
            fh.write(f)
    print(f"{len(frames)} frames, {sum(len(f) for f in frames)} bytes")


if __name__ == "__main__":
    main()

"""Test infrastructure: an independent bincode 1.3 (legacy fixint, LE)
ENCODER for the primary's messages, written from the serde derives of the
reference (primary/src/messages.rs:13-21,105-112,168-172,
primary/src/primary.rs:33-38, crypto/src/lib.rs:94-112,177-182) -- used to
feed the native decoder (coa_wire.cpp) frames it did not produce itself."""
import base64
import struct


def key(pk):  # PublicKey: serde string of base64 (crypto/src/lib.rs:94-101)
    s = base64.b64encode(bytes(pk))
    return struct.pack("<Q", len(s)) + s


def raw_key(s):  # a key string given as raw text (malformed-input tests)
    return struct.pack("<Q", len(s)) + s


def header(author, round_, payload, parents, id_, sig, author_field=None):
    """payload: list of (digest, worker id) in WIRE order (duplicates kept)."""
    out = (author_field if author_field is not None else key(author)) + struct.pack("<Q", round_)
    out += struct.pack("<Q", len(payload))
    for d, w in payload:
        out += bytes(d) + struct.pack("<I", w)
    out += struct.pack("<Q", len(parents))
    for p in parents:
        out += bytes(p)
    return out + bytes(id_) + bytes(sig)


def vote(id_, round_, origin, author, sig):
    return bytes(id_) + struct.pack("<Q", round_) + key(origin) + key(author) + bytes(sig)


def certificate(hdr_bytes, votes):
    out = hdr_bytes + struct.pack("<Q", len(votes))
    for pk, sg in votes:
        out += key(pk) + bytes(sg)
    return out


def primary_message(variant, body):  # enum PrimaryMessage: u32 variant index
    return struct.pack("<I", variant) + body


def cert_request(digests, requestor):
    return struct.pack("<Q", len(digests)) + b"".join(bytes(d) for d in digests) + key(requestor)


def header_digest_input(author, round_, payload, parents):
    """Header::digest's input (messages.rs:70-84): BTreeMap/BTreeSet order,
    last value of a repeated payload key."""
    pm = {}
    for d, w in payload:
        pm[bytes(d)] = w
    out = bytes(author) + struct.pack("<Q", round_)
    for d in sorted(pm):
        out += d + struct.pack("<I", pm[d])
    for p in sorted(set(bytes(p) for p in parents)):
        out += p
    return out

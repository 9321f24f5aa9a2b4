"""Probe: does the order of a C3 round's vote jobs matter to k_cert_verify?
The key combs (radix 2^20, 654 MB per key, 65 GB at committee 100) are read
at random magnitudes, and the kernel's vote jobs miss the per-CU
translation cache half the time (profiles/r05_cert_tlb_pmc.txt).  The
launcher sorts the jobs by key (k_job_keys/k_job_scan/k_job_place) so a
chunk's 64 lanes read one key's comb; COA_CERT_KEYSORT=0 keeps certificate
order (A/B).  Both on the bench's round (voters rotated by certificate) and
on one whose certificates list the same members in the same positions
(rotate=False).  Device-resident 10k-certificate rounds, median of the
timed calls, statuses checked.

usage: python tools/vote_order_probe.py [calls]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xrpl-coa-prototype_amd"))


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    import numpy as np
    import torch

    import certificates as C
    import coa_crypto

    coa_crypto.init(1)
    dev = torch.device("cuda:0")
    n = 10000
    for rotate in (True, False):
        committee, b = C.synth_certificates(n, committee_size=100, n_payload=32, seed=3, rotate=rotate)
        committee.register()
        hd = np.frombuffer(b"".join(b.header_inputs) + bytes(16), np.uint8)
        hoff = np.zeros(n + 1, np.uint64)
        hoff[1:] = np.cumsum([len(h) for h in b.header_inputs])
        t = lambda a: torch.from_numpy(np.array(a)).to(dev)  # noqa: E731
        args = [t(hd), t(hoff.view(np.int64)), t(b.ids), t(b.authors), t(b.header_sigs),
                t(np.full(n, b.round, np.int64)), t(b.vote_pks), t(b.vote_sigs), t(b.offsets.view(np.int64))]
        V = int(b.offsets[1])
        status = torch.empty(n, dtype=torch.int32, device=dev)
        ws = torch.empty(coa_crypto.certificate_workspace_bytes(n, n * V), dtype=torch.uint8, device=dev)
        for mode in ("0", "1", "0", "1"):
            os.environ["COA_CERT_KEYSORT"] = mode
            ts = []
            for i in range(calls + 3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                coa_crypto.certificate_verify_many_device(0, *args, status, workspace=ws)
                torch.cuda.synchronize()
                if i >= 3:
                    ts.append(time.perf_counter() - t0)
            ok = int((status != 0).sum().item()) == 0
            ms = sorted(ts)[len(ts) // 2] * 1e3
            print(json.dumps({"rotate": rotate, "keysort": mode, "ms_p50": round(ms, 3),
                              "certs_per_s": round(n / ms * 1e3, 1), "all_valid": ok}), flush=True)


if __name__ == "__main__":
    main()

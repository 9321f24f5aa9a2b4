"""The registration-under-load scenario of
tests/test_gpu_recovery.py::test_registration_never_holds_a_window_back,
repeated, printing each run's slowest window (launch call -> outputs), its
size and the registration times, with the queue settings of this process's
environment (A/B: alternate runs of this script with and without a switch).

  python tools/register_window_probe.py [reps]"""
import gc
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xrpl-coa-prototype_amd"))


def main():
    import torch  # noqa: F401  (one HIP runtime: torch's, as in the tests)

    import certificates as C
    import coa_crypto as engine

    engine.init(0)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    committee, batch = C.synth_certificates(64, committee_size=100, n_payload=4, seed=41)
    committee.register()
    votes = []
    for c in range(len(batch)):
        lo, hi = int(batch.offsets[c]), int(batch.offsets[c + 1])
        votes.append([(engine.PublicKey(bytes(batch.vote_pks[j])), engine.Signature.from_bytes(bytes(batch.vote_sigs[j])))
                      for j in range(lo, hi)])
    gc.collect()
    gc.freeze()
    gc.disable()
    for rep in range(reps):
        stop = threading.Event()
        reg_s = []

        def registrar():
            time.sleep(0.4)
            for _ in range(2):
                t0 = time.perf_counter()
                committee.register()
                reg_s.append(round(time.perf_counter() - t0, 3))
            stop.set()

        results = []
        with engine.AggregationQueue(max_batch=4096, max_delay_us=200) as q:
            q.set_idle_launch(1)
            reg = threading.Thread(target=registrar)
            reg.start()
            i = 0
            deadline = time.perf_counter() + 60
            while not stop.is_set() and time.perf_counter() < deadline:
                c = i % len(batch)
                results.append(q.submit_certificate(batch.header_inputs[c], bytes(batch.ids[c]), bytes(batch.authors[c]),
                                                    bytes(batch.header_sigs[c]), batch.round, votes[c]))
                i += 1
                time.sleep(0.0002)
            reg.join()
            q.flush()
            bad = sum(1 for f in results if f.result(timeout=120) != 0)
            m = q.metrics()
        print(json.dumps({"rep": rep, "env": {k: v for k, v in os.environ.items() if k.startswith("COA_QUEUE")},
                          "requests": len(results), "bad": bad, "window_ms_max": round(m["window_us_max"] * 1e-3, 2),
                          "window_max_items": m["window_max_items"], "window_max_at_ms": round(m["window_max_at_ms"], 1),
                          "windows": m["windows"], "wait_ms_p99": round(m["wait_us_p99"] * 1e-3, 3), "reg_s": reg_s}),
              flush=True)
    gc.enable()
    gc.unfreeze()


if __name__ == "__main__":
    main()

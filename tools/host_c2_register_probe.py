"""Host-pointer C2 (coa_ed25519_verify_strict_many, 65,536 triples per call)
from 1 / 2 / 4 C threads over as many contexts (tools/latc.c
latc_verify_many), with the inputs in ordinary pageable memory and then
page-locked in place (hipHostRegister).  Question: do the two threads'
calls serialise on the runtime's pageable host-to-device copies?

  python tools/host_c2_register_probe.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    import numpy as np
    import torch  # noqa: F401  (torch's HIP runtime: the engine links the same soname)

    import coa_crypto
    import workloads

    coa_crypto.init_devices([0])
    n = 65536
    pks, sigs = coa_crypto.sign_many(workloads.key_seeds(n), workloads.messages(n))
    msgs = np.ascontiguousarray(workloads.messages(n))
    pks, sigs = np.ascontiguousarray(pks), np.ascontiguousarray(sigs)
    lib = bench._latc()
    vp, sz, ci, dp = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_double)
    lib.latc_verify_many.argtypes = [vp, vp, vp, sz, ci, ci, dp]
    lib.latc_verify_many.restype = ci
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostRegister.argtypes = [vp, sz, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [vp]
    el = ctypes.c_double()

    def run(tag):
        out = {}
        for threads in (1, 2, 4):
            coa_crypto.shutdown()
            coa_crypto.init_devices([0] * threads)
            calls = 40 if threads == 1 else 24
            assert lib.latc_verify_many(msgs.ctypes.data, pks.ctypes.data, sigs.ctypes.data, n, 2, threads,
                                        ctypes.byref(el)) == 0
            rc = lib.latc_verify_many(msgs.ctypes.data, pks.ctypes.data, sigs.ctypes.data, n, calls, threads,
                                      ctypes.byref(el))
            assert rc == 0, rc
            out[threads] = round(n * calls * threads / el.value / 1e6, 1)
        print(json.dumps({"inputs": tag, "M_verify_per_s_by_threads": out}), flush=True)

    for rep in range(2):
        run("pageable")
        for a in (msgs, pks, sigs):
            assert hip.hipHostRegister(a.ctypes.data, a.nbytes, 0) == 0
        run("registered (hipHostRegister)")
        for a in (msgs, pks, sigs):
            hip.hipHostUnregister(a.ctypes.data)


if __name__ == "__main__":
    main()

"""Probe: torch's HIP runtime and the engine's in one process.  The engine
library links libamdhip64 by soname; when torch is imported first the
process has one HIP runtime (torch's), when the engine loads first torch's
bundled runtime is a second copy that sees no GPU.  Usage:
  python tools/probe_torch_after_init.py [torch-first]"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "xrpl-coa-prototype_amd")]
if len(sys.argv) > 1 and sys.argv[1] == "torch-first":
    import torch  # noqa: F401
import coa_crypto

coa_crypto.init(0)
print("engine devices", coa_crypto.device_count(), "self_test bad", coa_crypto.self_test(0), flush=True)
import torch

s = torch.cuda.Stream(torch.device("cuda", 0))
print("torch stream ok; hip runtime:", [l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l][:1],
      flush=True)

"""CPU: the host-side runtime under sanitizers.

* coa_wire.cpp -- the bincode decoder of untrusted network frames
  (PrimaryReceiverHandler::dispatch, primary/src/primary.rs:223-244) -- built
  with AddressSanitizer + UndefinedBehaviorSanitizer and driven by a mutation
  fuzzer (tests/fuzz/wire_fuzz.cpp) over the committed seed corpus
  (tests/fuzz/wire_corpus, made by tests/fuzz/make_wire_corpus.py):
  truncations, huge length prefixes, byte flips, splices, bad base64.
* coa_queue.cpp -- the multi-producer aggregation queue -- built with
  ThreadSanitizer (clang's runtime: GCC 11's libtsan does not intercept
  pthread_cond_clockwait and reports false double locks) and, separately,
  ASan + UBSan, with a deterministic stub in place of its HIP launch backend
  (same two-slot double buffering), with 16 producer threads submitting
  every request kind while they also flush and read the stats and metrics,
  and with injected launch failures (engine-failure recovery: re-run and
  exact, or reported to every callback when every attempt fails).
No device code is involved (GPU sanitizers are not available on the pool)."""
import os
import subprocess

import pytest

from conftest import ROOT

CSRC = os.path.join(ROOT, "xrpl-coa-prototype_amd", "csrc")
INC = os.path.join(ROOT, "include")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


def _build(out, srcs, flags, cxx="g++"):
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-I", INC, "-I", CSRC] + flags + srcs + ["-o", out,
                                                                                                   "-pthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


def _run(cmd, env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    return r.stdout


def test_wire_decoder_fuzz_asan_ubsan():
    exe = _build(os.path.join(ROOT, "tests", "fuzz", "_build", "wire_fuzz"),
                 [os.path.join(CSRC, "coa_wire.cpp"), os.path.join(ROOT, "tests", "fuzz", "wire_fuzz.cpp")],
                 ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"])
    corpus = os.path.join(ROOT, "tests", "fuzz", "wire_corpus")
    assert len(os.listdir(corpus)) >= 10
    for seed in (1, 2):
        out = _run([exe, corpus, "60000", str(seed)], {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1",
                                                      "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})
        assert "wire fuzz ok" in out
        # the mutations reach every decoder, accepted and rejected frames alike
        assert "certificate 0" not in out and "rejected 0" not in out


@pytest.mark.skipif(not os.path.exists(CLANG), reason="ROCm clang (TSan runtime) not present")
def test_queue_many_producers_tsan():
    exe = _build(os.path.join(ROOT, "tests", "sanitize", "_build", "queue_tsan"),
                 [os.path.join(CSRC, "coa_queue.cpp"), os.path.join(ROOT, "tests", "sanitize", "queue_tsan.cpp")],
                 ["-fsanitize=thread"], cxx=CLANG)
    out = _run([exe, "16", "500"], {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"})
    assert "8000/8000 answered, 0 wrong" in out
    # engine-failure recovery: every 7th launch fails; each is re-run and
    # every callback still gets its exact verdict (the binary checks that
    # retried == recovered == injected and no callback saw an engine error)
    out = _run([exe, "16", "500", "7"], {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"})
    assert "8000/8000 answered, 0 wrong" in out and "injected 0," not in out, out
    # idle launch: windows also launched by submitting threads that find the
    # engine idle (beside the collector), with and without injected failures
    for k in ("1", "2"):
        env = {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1", "COA_QUEUE_IDLE_LAUNCH": k}
        out = _run([exe, "16", "500"], env)
        assert "8000/8000 answered, 0 wrong" in out, out
        out = _run([exe, "16", "300", "7"], env)
        assert "4800/4800 answered, 0 wrong" in out and "injected 0," not in out, out


def test_queue_many_producers_asan_ubsan():
    exe = _build(os.path.join(ROOT, "tests", "sanitize", "_build", "queue_asan"),
                 [os.path.join(CSRC, "coa_queue.cpp"), os.path.join(ROOT, "tests", "sanitize", "queue_tsan.cpp")],
                 ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"])
    env = {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1", "UBSAN_OPTIONS": "halt_on_error=1"}
    out = _run([exe, "16", "500"], env)
    assert "8000/8000 answered, 0 wrong" in out
    # every 5th launch fails and so does every retry: those windows' callbacks
    # get the engine error (counted as failed windows), the rest are exact
    out = _run([exe, "8", "300", "5", "1"], env)
    assert "2400/2400 answered, 0 wrong" in out and "recovered 0" in out and "engine errors 0" not in out, out
    out = _run([exe, "16", "500"], dict(env, COA_QUEUE_IDLE_LAUNCH="1"))
    assert "8000/8000 answered, 0 wrong" in out, out


def _copy_pool_inc(dst_dir):
    """The CopyPool class text of coa_runtime.cpp (the runtime itself needs
    HIP; the class is plain C++)."""
    src = open(os.path.join(CSRC, "coa_runtime.cpp")).read()
    body = src[src.index("class CopyPool {"):src.index("struct Dev {")]
    os.makedirs(dst_dir, exist_ok=True)
    with open(os.path.join(dst_dir, "copy_pool_class.inc"), "w") as f:
        f.write(body)
    return dst_dir


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_copy_pool_concurrent_jobs(san):
    """Round 6: several copies in progress on the pool at once (two
    collectors' windows); a worker's job is taken in its wait predicate (a
    second lookup after the wait raced the other workers' claims and came
    back empty: a null job, SIGSEGV on a GPU box)."""
    inc = _copy_pool_inc(os.path.join(ROOT, "tests", "sanitize", "_build"))
    flags = ["-fsanitize=" + san, "-fno-sanitize-recover=all", "-I", inc]
    cxx = CLANG if san == "thread" and os.path.exists(CLANG) else "g++"
    exe = _build(os.path.join(inc, "copy_pool_" + san.split(",")[0]),
                 [os.path.join(ROOT, "tests", "sanitize", "copy_pool_stress.cpp")], flags, cxx=cxx)
    out = _run([exe], {"TSAN_OPTIONS": "halt_on_error=1", "ASAN_OPTIONS": "abort_on_error=1",
                       "UBSAN_OPTIONS": "halt_on_error=1"})
    assert "copy pool ok: 0 bad" in out


def _cpu_vectors(path):
    """tests/sanitize/cpu_path_driver.cpp's input: the golden verify vectors
    and batch groups in a flat binary form."""
    import json
    import struct

    gold = os.path.join(ROOT, "tests", "golden")
    vv = json.load(open(os.path.join(gold, "verify_vectors.json")))
    bv = json.load(open(os.path.join(gold, "batch_vectors.json")))
    out = [b"CPUV", struct.pack("<I", len(vv))]
    for v in vv:
        m = bytes.fromhex(v["msg"])
        out.append(struct.pack("<I", len(m)) + m + bytes.fromhex(v["pk"]) + bytes.fromhex(v["sig"]) +
                   bytes([1 if v["expect"] else 0]))
    out.append(struct.pack("<I", len(bv)))
    for g in bv:
        out.append(bytes.fromhex(g["msg"]) + struct.pack("<I", len(g["pks"])))
        for pk, sg, z in zip(g["pks"], g["sigs"], g["zs"]):
            out.append(bytes.fromhex(pk) + bytes.fromhex(sg) + int(z, 16).to_bytes(16, "little"))
        out.append(bytes([1 if g["expect"] else 0]))
    with open(path, "wb") as f:
        f.write(b"".join(out))
    return path


def test_cpu_path_asan_ubsan():
    """Round 6: the engine's own CPU path (coa_cpu.cpp) built with ASan +
    UBSan and run over the golden verify vectors (single and 4-thread many
    calls), the golden batch groups, SHA-512 and a certificate round."""
    d = os.path.join(ROOT, "tests", "sanitize", "_build")
    exe = _build(os.path.join(d, "cpu_path_asan"),
                 [os.path.join(CSRC, "coa_cpu.cpp"), os.path.join(ROOT, "tests", "sanitize", "cpu_path_driver.cpp")],
                 ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"])
    vec = _cpu_vectors(os.path.join(d, "cpu_vectors.bin"))
    out = _run([exe, vec], {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1",
                            "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})
    assert "cpu path ok" in out and " 0 bad" in out

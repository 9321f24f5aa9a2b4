"""CPU: the Rust drop-in (rust/, the cargo side of the boundary: build.rs,
crypto/src/coa_ffi.rs, crypto/src/gpu.rs, primary/src/gpu_certificate.rs)
cannot be compiled in this image (no cargo/rustc), so its consistency with
the C ABI is checked here: every function include/coa_verify.h declares is
declared in coa_ffi.rs with the same parameter kinds in the same order and
the same return kind, every extern block elsewhere in rust/ agrees with the
header, and no placeholder is left (todo!/unimplemented!/helpers that are
called but never defined)."""
import os
import re

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "coa_verify.h")
RUST = os.path.join(ROOT, "rust")


def _c_kind(t):
    t = t.strip()
    if "*" in t or "[" in t:
        return "ptr"
    t = re.sub(r"\bconst\b", "", t).split()
    base = t[0] if t else ""
    return {"int": "int", "size_t": "usize", "uint64_t": "u64", "uint32_t": "u32", "int32_t": "int",
            "coa_verdict_cb": "cb", "void": "void"}[base]


def c_prototypes():
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for ret, name, args in re.findall(r"(int|size_t|const char\*|coa_queue\*)\s+(coa_\w+)\s*\(([^)]*)\)\s*;", text):
        params = [] if args.strip() in ("", "void") else [_c_kind(a.rsplit(" ", 1)[0] if "[" not in a else a)
                                                          for a in args.split(",")]
        out[name] = (_c_kind(ret), params)
    return out


def _r_kind(t):
    t = t.strip()
    if t.startswith("*"):
        return "ptr"
    return {"c_int": "int", "i32": "int", "usize": "usize", "u64": "u64", "u32": "u32", "CoaVerdictCb": "cb"}[t]


def rust_externs(path):
    text = open(path).read()
    out = {}
    for block in re.findall(r'extern "C"\s*\{(.*?)\n\}', text, flags=re.S):
        for name, args, ret in re.findall(r"fn\s+(coa_\w+)\s*\((.*?)\)\s*(?:->\s*([^;]+))?;", block, flags=re.S):
            params = [_r_kind(a.split(":", 1)[1]) for a in args.split(",") if a.strip()]
            out[name] = ("void" if not ret else _r_kind(ret.strip()) if "*" not in ret else "ptr", params)
    return out


def test_coa_ffi_declares_the_whole_header_with_matching_prototypes():
    c = c_prototypes()
    r = rust_externs(os.path.join(RUST, "crypto", "src", "coa_ffi.rs"))
    assert len(c) >= 40
    missing = sorted(set(c) - set(r))
    assert not missing, missing
    for name, (ret, params) in c.items():
        assert r[name][1] == params, (name, params, r[name][1])
        assert r[name][0] == ret, (name, ret, r[name][0])
    assert not sorted(set(r) - set(c)), "coa_ffi.rs declares functions the header does not"


def test_other_rust_extern_blocks_match_header():
    c = c_prototypes()
    for dirpath, _, files in os.walk(RUST):
        for f in files:
            if f.endswith(".rs") and f != "coa_ffi.rs":
                for name, (ret, params) in rust_externs(os.path.join(dirpath, f)).items():
                    assert name in c, (f, name)
                    assert c[name] == (ret, params), (f, name)


def test_no_placeholders_and_helpers_defined():
    text = ""
    for dirpath, _, files in os.walk(RUST):
        for f in files:
            if f.endswith(".rs"):
                src = open(os.path.join(dirpath, f)).read()
                src = re.sub(r"//[^\n]*", "", src)            # comments
                src = re.sub(r"#!?\[[^\]]*\]", "", src)       # attributes
                src = re.sub(r'"(?:[^"\\]|\\.)*"', '""', src)  # string literals
                text += src
    assert "todo!" not in text and "unimplemented!" not in text
    # every free function called is defined in the shim, taken from the FFI,
    # or a std / reference crate API (method calls excluded)
    defined = set(re.findall(r"\bfn\s+(\w+)", text))
    called = set(re.findall(r"(?<![\w.:!])([a-z_][a-z0-9_]*)\s*\(", text))
    keywords = {"if", "for", "while", "match", "assert", "assert_eq", "panic", "vec", "fn", "return", "Some", "Ok",
                "Err", "ensure", "println", "loop", "in", "as", "unsafe", "move", "Box", "format", "mod", "let"}
    unknown = sorted(called - defined - keywords)
    assert not unknown, unknown
    assert "header_digest_input" in defined
    assert os.path.exists(os.path.join(RUST, "crypto", "build.rs"))

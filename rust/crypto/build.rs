//! cargo build script of the reference's `crypto` crate with the MI355X
//! engine: builds `libcoa_verify.so` for gfx950 (hipcc, through the engine's
//! own build script) and links the crate against it.
//!
//! Add to `crypto/Cargo.toml` under `[package]`:  `build = "build.rs"`.
//! `COA_ENGINE_DIR` points at this repository's `xrpl-coa-prototype_amd`
//! directory (default: `../xrpl-coa-prototype_amd` next to the workspace).
use std::env;
use std::path::PathBuf;
use std::process::Command;

fn main() {
    let engine = PathBuf::from(
        env::var("COA_ENGINE_DIR").unwrap_or_else(|_| "../xrpl-coa-prototype_amd".to_string()),
    );
    let include = engine.join("..").join("include");
    // hipcc --offload-arch=gfx950 -O3 ... -shared -> <engine>/lib/libcoa_verify.so
    let status = Command::new(env::var("PYTHON").unwrap_or_else(|_| "python3".to_string()))
        .arg(engine.join("build.py"))
        .status()
        .expect("failed to start the gfx950 engine build (python3 build.py, hipcc)");
    assert!(status.success(), "gfx950 engine build failed");
    let lib = engine.join("lib");
    println!("cargo:rustc-link-search=native={}", lib.display());
    println!("cargo:rustc-link-lib=dylib=coa_verify");
    // the engine links libamdhip64 by soname; ROCm's lib directory resolves it
    let rocm = env::var("ROCM_PATH").unwrap_or_else(|_| "/opt/rocm".to_string());
    println!("cargo:rustc-link-search=native={}/lib", rocm);
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", lib.display());
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}/lib", rocm);
    println!("cargo:rerun-if-changed={}", engine.join("csrc").display());
    println!("cargo:rerun-if-changed={}", include.join("coa_verify.h").display());
    println!("cargo:rerun-if-env-changed=COA_ENGINE_DIR");
}

//! Verdicts computed ahead of the synchronous call that asks for them.
//!
//! The pre-verification stage (rust/primary/src/pre_verify.rs) verifies the
//! messages the receiver hands to `Core` in large coalesced launches through
//! `VerifyService`, before `Core` sees them.  `Core` itself is unchanged: it
//! still calls `Header::verify`, `Vote::verify` and `Certificate::verify`
//! one message at a time (primary/src/core.rs:306-346), and those reach
//! `gpu::verify` / `gpu_certificate::verify`, which first look here.
//!
//! Exactness: an entry is keyed by EVERY byte the verdict depends on -- the
//! (digest, key, signature) triple of a `Signature::verify`, the full crypto
//! input of a `Certificate::verify` (header digest input, id, origin, header
//! signature, round, every vote) -- and compared for equality on lookup, so a
//! hit returns exactly the verdict the engine returns for those bytes.  Both
//! outcomes are kept: a verify_strict verdict is a pure function of the 128
//! bytes, so a remembered Err is exactly as faithful as a remembered Ok, and
//! `Core` never asks the engine a second time for a message the stage saw
//! (a flood of bad signatures costs one coalesced verification each, not one
//! more single-signature launch on `Core`'s task).  Certificate entries keep
//! their COA_CERT_* bits, which `gpu_certificate::checks_in_order` consumes
//! in the reference's order.
//! Entries are taken (removed) by the lookup that uses them, and the oldest
//! are dropped beyond a fixed capacity, so messages that never reach the
//! verify call (e.g. `DagError::TooOld`) cannot grow the cache.
//!
//! Toolchain: std only, no `OnceLock` (Rust 1.70) -- the caches are set up
//! through `std::sync::Once`, which the reference's pinned 1.51.0
//! (.github/workflows/rust.yml:20) has.
use crate::{Digest, PublicKey};
use std::borrow::Borrow;
use std::collections::hash_map::Entry;
use std::collections::{HashMap, VecDeque};
use std::hash::Hash;
use std::sync::{Mutex, Once};

const SIGNATURES: usize = 1 << 17;
const CERTIFICATES: usize = 1 << 14;

/// A map with FIFO eviction.  `order` may hold keys already taken; the
/// generation stamp tells a live entry from a stale order slot.
struct Fifo<K, V> {
    map: HashMap<K, (V, u64)>,
    order: VecDeque<(K, u64)>,
    cap: usize,
    next_gen: u64,
}

impl<K: Eq + Hash + Clone, V> Fifo<K, V> {
    fn new(cap: usize) -> Self {
        Self { map: HashMap::new(), order: VecDeque::new(), cap, next_gen: 0 }
    }

    fn insert(&mut self, key: K, value: V) {
        let gen = self.next_gen;
        self.next_gen += 1;
        match self.map.entry(key.clone()) {
            Entry::Occupied(mut e) => {
                e.insert((value, gen));
            }
            Entry::Vacant(e) => {
                e.insert((value, gen));
            }
        }
        self.order.push_back((key, gen));
        while self.order.len() > self.cap {
            if let Some((old, old_gen)) = self.order.pop_front() {
                if self.map.get(&old).map(|(_, g)| *g) == Some(old_gen) {
                    self.map.remove(&old);
                }
            }
        }
    }

    fn take<Q: ?Sized + Eq + Hash>(&mut self, key: &Q) -> Option<V>
    where
        K: Borrow<Q>,
    {
        self.map.remove(key).map(|(v, _)| v)
    }
}

type SignatureCache = Mutex<Fifo<[u8; 128], bool>>;
type CertificateCache = Mutex<Fifo<Vec<u8>, u8>>;

fn signatures() -> &'static SignatureCache {
    static INIT: Once = Once::new();
    static mut CACHE: *const SignatureCache = std::ptr::null();
    unsafe {
        INIT.call_once(|| CACHE = Box::into_raw(Box::new(Mutex::new(Fifo::new(SIGNATURES)))));
        &*CACHE
    }
}

fn certificates() -> &'static CertificateCache {
    static INIT: Once = Once::new();
    static mut CACHE: *const CertificateCache = std::ptr::null();
    unsafe {
        INIT.call_once(|| CACHE = Box::into_raw(Box::new(Mutex::new(Fifo::new(CERTIFICATES)))));
        &*CACHE
    }
}

fn triple(digest: &Digest, key: &PublicKey, signature: &[u8; 64]) -> [u8; 128] {
    let mut k = [0u8; 128];
    k[..32].copy_from_slice(&digest.0);
    k[32..64].copy_from_slice(&key.0);
    k[64..].copy_from_slice(signature);
    k
}

/// The engine's `Signature::verify(digest, key)` verdict of `signature`:
/// `ok` = Ok, else Err.
pub fn remember_signature(digest: &Digest, key: &PublicKey, signature: &[u8; 64], ok: bool) {
    signatures().lock().unwrap().insert(triple(digest, key, signature), ok);
}

/// The verdict remembered for exactly this triple, if any (the entry is
/// consumed): `Some(true)` = Ok, `Some(false)` = Err.
pub fn take_signature(digest: &Digest, key: &PublicKey, signature: &[u8; 64]) -> Option<bool> {
    signatures().lock().unwrap().take(&triple(digest, key, signature))
}

/// The COA_CERT_* bits of the certificate whose crypto input is `key`
/// (`service::CertificateCrypto::into_key`; no copy is made).
pub fn remember_certificate(key: Vec<u8>, bits: u8) {
    certificates().lock().unwrap().insert(key, bits);
}

/// The bits remembered for exactly this crypto input, if any (consumed).
pub fn take_certificate(key: &[u8]) -> Option<u8> {
    certificates().lock().unwrap().take(key)
}

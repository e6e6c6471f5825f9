//! overlord-hip: the MI355X backend of consensus_overlord's `Crypto` trait.
//!
//! `HipCrypto` is a drop-in for `ConsensusCrypto` (reference `src/consensus.rs:334-463`): the same
//! five trait methods with the same error precedence, over libovhip.so (include/ovhip.h). A node
//! selects it by config (`crypto_backend = "hip"` beside `src/config.rs:18-31`); nothing else in
//! the node changes. The arithmetic runs on the GPU (gfx950 HIP kernels); there is no CPU path.
//!
//! Like `ConsensusCrypto` (`#[derive(Clone)]`, consensus.rs:339) it is cheap to clone:
//! `Consensus::new` clones it into `Brain`, into the `Arc` overlord holds and into itself
//! (consensus.rs:61-76). The clones share one device context (`Arc<Ctx>`: the last clone to drop
//! destroys it, never twice) and one key list, as the reference's clones share
//! `Arc<RwLock<Vec<BlsPublicKey>>>`. `update_pubkeys` is `async` and takes the reference callers'
//! `Vec<BlsPublicKey>` (consensus.rs:131-136, :622-629) through ophelia's `PublicKey` trait.
//!
//! Error mapping (reference `src/error.rs:20-44`, `consensus.rs:391-462`): code 100 is
//! `Other("failed to convert hash value")`, 101 `Other("signatures length does not match voters
//! length")`, 102 `Other("lose public key")`, 1..=7 a blst error (`CryptoErr`), anything else a
//! device error. The variants and their Display follow the reference's `ConsensusError`
//! (derive_more `{_0:?}` / `"Crypto error {_0:?}"`); overlord only observes Ok / Err.
//!
//! Not compiled in this repository's image (no Rust toolchain): `tests/test_crate_ffi.py` checks
//! the FFI block against the header and the drop-in shape (Clone, `update_pubkeys`, the ingress
//! module's calls) textually.
pub mod ffi;
pub mod ingress;

use bytes::Bytes;
use overlord::Crypto as OverlordCrypto;
use std::error::Error;
use std::fmt;
use std::sync::atomic::{AtomicI32, Ordering};
use std::sync::Arc;
use tokio::sync::RwLock;

/// The reference's `ConsensusError` variants this backend can return (`src/error.rs:20-44`).
#[derive(Debug)]
pub enum HipCryptoError {
    /// `ConsensusError::Other(String)`: hash length, list length mismatch, key parse.
    Other(String),
    /// `ConsensusError::CryptoErr`: a blst error code (1 BAD_ENCODING ... 7 BAD_SCALAR).
    CryptoErr(i32),
    /// The device or the OS random source failed (codes 103, 200, 201).
    Device(i32),
}

impl fmt::Display for HipCryptoError {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        match self {
            HipCryptoError::Other(s) => write!(f, "{s:?}"),
            HipCryptoError::CryptoErr(c) => write!(f, "Crypto error {c:?}"),
            HipCryptoError::Device(c) => write!(f, "hip device error {c}"),
        }
    }
}

impl Error for HipCryptoError {}

/// As the reference's `impl From<ConsensusError> for Box<dyn Error + Send>` (error.rs:41-45).
impl From<HipCryptoError> for Box<dyn Error + Send> {
    fn from(error: HipCryptoError) -> Self {
        Box::new(error) as Box<dyn Error + Send>
    }
}

pub(crate) fn to_err(code: i32) -> Box<dyn Error + Send> {
    match code {
        ffi::OVH_ERR_HASH_LEN => HipCryptoError::Other("failed to convert hash value".into()),
        ffi::OVH_ERR_LEN_MISMATCH => {
            HipCryptoError::Other("signatures length does not match voters length".into())
        }
        ffi::OVH_ERR_PUBKEY => HipCryptoError::Other("lose public key".into()),
        1..=7 => HipCryptoError::CryptoErr(code),
        c => HipCryptoError::Device(c),
    }
    .into()
}

pub(crate) fn check(code: i32) -> Result<(), Box<dyn Error + Send>> {
    if code == ffi::OVH_OK {
        Ok(())
    } else {
        Err(to_err(code))
    }
}

/// `Vec<Bytes>` across the C ABI: one concatenated buffer plus the item lengths.
fn concat(v: &[Bytes]) -> (Vec<u8>, Vec<usize>) {
    (v.iter().flat_map(|b| b.iter().copied()).collect(), v.iter().map(|b| b.len()).collect())
}

/// The device context. Owned through `Arc` by every clone of `HipCrypto` (and by the blocking
/// tasks `update_pubkeys` and the ingress shim start); `ovh_destroy` runs once, when the last
/// owner drops it.
pub(crate) struct Ctx(pub(crate) *mut ffi::OvhCtx);
// libovhip serialises every entry point on the context's own mutex (include/ovhip.h: the trait
// object is Send + Sync and is called by overlord and the check_block handler concurrently).
unsafe impl Send for Ctx {}
unsafe impl Sync for Ctx {}

impl Drop for Ctx {
    fn drop(&mut self) {
        unsafe { ffi::ovh_destroy(self.0) }
    }
}

/// The GPU `Crypto` of a node: its private key (as `ConsensusCrypto::new` reads it), the name
/// (48-byte compressed public key) and the validator keys (`ConsensusCrypto::pubkeys`).
#[derive(Clone)]
pub struct HipCrypto {
    ctx: Arc<Ctx>,
    private_key: Arc<Vec<u8>>,
    pub name: Bytes,
    /// The validator keys as last given to `update_pubkeys` (the device table holds them
    /// decompressed and group-checked); shared by every clone, as the reference's field.
    pub pubkeys: Arc<RwLock<Vec<Bytes>>>,
    /// The code of the last failed device table upload (0: none); `update_pubkeys` returns
    /// nothing, as the reference's does.
    table_error: Arc<AtomicI32>,
}

impl HipCrypto {
    /// `ConsensusCrypto::new` (consensus.rs:347-359): hex key file -> key bytes -> name. `devices`
    /// empty: GPU 0; several: one context over those GPUs (batches shard across them).
    pub fn new(private_key_path: &str, devices: &[i32]) -> Result<Self, Box<dyn Error + Send>> {
        let text = std::fs::read_to_string(private_key_path)
            .map_err(|e| Box::new(HipCryptoError::Other(e.to_string())) as Box<dyn Error + Send>)?;
        let key = hex::decode(text.trim())
            .map_err(|e| Box::new(HipCryptoError::Other(e.to_string())) as Box<dyn Error + Send>)?;
        Self::from_key(key, devices)
    }

    pub fn from_key(private_key: Vec<u8>, devices: &[i32]) -> Result<Self, Box<dyn Error + Send>> {
        let ctx = unsafe {
            match devices.len() {
                0 => ffi::ovh_create(0, std::ptr::null(), 0, 0),
                1 => ffi::ovh_create(devices[0], std::ptr::null(), 0, 0),
                n => ffi::ovh_create_multi(devices.as_ptr(), n as i32, std::ptr::null(), 0, 0),
            }
        };
        if ctx.is_null() {
            return Err(to_err(ffi::OVH_ERR_DEVICE));
        }
        let ctx = Ctx(ctx);
        let mut name = [0u8; 48];
        check(unsafe {
            ffi::ovh_sk_to_pk(ctx.0, private_key.as_ptr(), private_key.len(), name.as_mut_ptr())
        })?;
        Ok(HipCrypto {
            ctx: Arc::new(ctx),
            private_key: Arc::new(private_key),
            name: Bytes::copy_from_slice(&name),
            pubkeys: Arc::new(RwLock::new(Vec::new())),
            table_error: Arc::new(AtomicI32::new(0)),
        })
    }

    pub(crate) fn raw(&self) -> *mut ffi::OvhCtx {
        self.ctx.0
    }

    /// `ConsensusCrypto::update_pubkeys` (consensus.rs:361-363), same shape: `async`, no result,
    /// takes the callers' `Vec<BlsPublicKey>` (consensus.rs:131-136, :622-629) -- any ophelia
    /// `PublicKey`. The keys go to the device table (decompressed and group-checked once, on a
    /// blocking task: never on the reactor). A key the device cannot parse stays in the table as
    /// unparsed, and a vote by it answers "lose public key" exactly as the key path does; a
    /// failed upload leaves the table empty (every vote then takes the key path, still exact)
    /// and is reported by `table_error`.
    pub async fn update_pubkeys<K: ophelia::PublicKey>(&self, new_pubkeys: Vec<K>) {
        let keys: Vec<Bytes> = new_pubkeys.iter().map(|k| k.to_bytes()).collect();
        let ctx = self.ctx.clone();
        let n = keys.len();
        let all48 = keys.iter().all(|k| k.len() == 48);
        let flat: Vec<u8> = keys.iter().flat_map(|k| k.iter().copied()).collect();
        let code = tokio::task::spawn_blocking(move || {
            if all48 {
                unsafe { ffi::ovh_set_validators(ctx.0, flat.as_ptr(), n) }
            } else {
                // not compressed G1 keys: an empty table (the key path serves every vote)
                let c = unsafe { ffi::ovh_set_validators(ctx.0, std::ptr::null(), 0) };
                if c == ffi::OVH_OK {
                    ffi::OVH_ERR_PUBKEY
                } else {
                    c
                }
            }
        })
        .await
        .unwrap_or(ffi::OVH_ERR_DEVICE);
        self.table_error.store(code, Ordering::Relaxed);
        *self.pubkeys.write().await = keys;
    }

    /// The code of the last failed `update_pubkeys` upload (0 when the table is current).
    pub fn table_error(&self) -> i32 {
        self.table_error.load(Ordering::Relaxed)
    }

    /// The vote-batching hook at `proc_network_msg` (consensus.rs:210-262, `ingress::VoteIngress`):
    /// batch-verify held votes; later `verify_signature` calls on them are answered from the
    /// verdict cache. Blocking: call from `spawn_blocking`, never on the reactor.
    pub fn prefetch(&self, sigs: &[[u8; 96]], hashes: &[[u8; 32]], voters: &[[u8; 48]]) -> Result<(), Box<dyn Error + Send>> {
        if sigs.len() != hashes.len() || sigs.len() != voters.len() {
            return Err(to_err(ffi::OVH_ERR_LEN_MISMATCH));
        }
        check(unsafe {
            ffi::ovh_prefetch(self.raw(), sigs.len(), sigs.as_ptr() as *const u8, hashes.as_ptr() as *const u8,
                              voters.as_ptr() as *const u8)
        })
    }

    /// hash(rlp(Vote)) of n votes on the device (`ovh_vote_digests`: rlp + SM3 per vote, the
    /// bytes overlord signs, consensus.rs:169-175). `block_hashes` holds one hash per vote of at
    /// most OVH_VOTE_HASH_MAX bytes. Blocking.
    pub fn vote_digests(&self, heights: &[u64], rounds: &[u64], vote_types: &[u8], block_hashes: &[Bytes]) -> Result<Vec<[u8; 32]>, Box<dyn Error + Send>> {
        let n = heights.len();
        if rounds.len() != n || vote_types.len() != n || block_hashes.len() != n {
            return Err(to_err(ffi::OVH_ERR_LEN_MISMATCH));
        }
        let mut hb = vec![0u8; n * ffi::OVH_VOTE_HASH_MAX];
        let mut hl = vec![0u8; n];
        for (i, h) in block_hashes.iter().enumerate() {
            if h.len() > ffi::OVH_VOTE_HASH_MAX {
                return Err(to_err(ffi::OVH_ERR_ARG));
            }
            hb[i * ffi::OVH_VOTE_HASH_MAX..i * ffi::OVH_VOTE_HASH_MAX + h.len()].copy_from_slice(h);
            hl[i] = h.len() as u8;
        }
        let mut out = vec![[0u8; 32]; n];
        check(unsafe {
            ffi::ovh_vote_digests(self.raw(), n, heights.as_ptr(), rounds.as_ptr(), vote_types.as_ptr(), hb.as_ptr(),
                                  hl.as_ptr(), out.as_mut_ptr() as *mut u8)
        })?;
        Ok(out)
    }

    /// n x `verify_signature` in one call: codes[i] is the per-call code of vote i (0 = Ok).
    pub fn verify_batch(&self, sigs: &[[u8; 96]], hashes: &[[u8; 32]], voters: &[[u8; 48]]) -> Result<Vec<i32>, Box<dyn Error + Send>> {
        if sigs.len() != hashes.len() || sigs.len() != voters.len() {
            return Err(to_err(ffi::OVH_ERR_LEN_MISMATCH));
        }
        let mut codes = vec![0i32; sigs.len()];
        check(unsafe {
            ffi::ovh_verify_batch(self.raw(), sigs.len(), sigs.as_ptr() as *const u8, hashes.as_ptr() as *const u8,
                                  voters.as_ptr() as *const u8, codes.as_mut_ptr())
        })?;
        Ok(codes)
    }
}

impl OverlordCrypto for HipCrypto {
    /// consensus.rs:386-388 -> util.rs:81-87 (SM3).
    fn hash(&self, msg: Bytes) -> Bytes {
        let mut out = [0u8; 32];
        unsafe { ffi::ovh_sm3(msg.as_ptr(), msg.len(), out.as_mut_ptr()) };
        Bytes::copy_from_slice(&out)
    }

    /// consensus.rs:390-395: hash length (100), then sigma = sk H(hash), compressed.
    fn sign(&self, hash: Bytes) -> Result<Bytes, Box<dyn Error + Send>> {
        let mut out = [0u8; 96];
        check(unsafe {
            ffi::ovh_sign(self.raw(), self.private_key.as_ptr(), self.private_key.len(), hash.as_ptr(), hash.len(),
                          out.as_mut_ptr())
        })?;
        Ok(Bytes::copy_from_slice(&out))
    }

    /// consensus.rs:397-416: hash length (100), pk parse (102), sig parse (1..3), verify (3, 5, 6).
    fn verify_signature(&self, signature: Bytes, hash: Bytes, voter: Bytes) -> Result<(), Box<dyn Error + Send>> {
        check(unsafe {
            ffi::ovh_verify(self.raw(), signature.as_ptr(), signature.len(), hash.as_ptr(), hash.len(),
                            voter.as_ptr(), voter.len())
        })
    }

    /// consensus.rs:418-444: length check (101), per pair sig parse then pk parse (102), empty
    /// (4), sum in G2, compressed.
    fn aggregate_signatures(&self, signatures: Vec<Bytes>, voters: Vec<Bytes>) -> Result<Bytes, Box<dyn Error + Send>> {
        let (s, sl) = concat(&signatures);
        let (v, vl) = concat(&voters);
        let mut out = [0u8; 96];
        check(unsafe {
            ffi::ovh_aggregate_sigs(self.raw(), s.as_ptr(), sl.as_ptr(), sl.len(), v.as_ptr(), vl.as_ptr(), vl.len(),
                                    out.as_mut_ptr())
        })?;
        Ok(Bytes::copy_from_slice(&out))
    }

    /// consensus.rs:446-462 + 365-382: pk parse (102), aggregate (4), sig parse, hash length
    /// (100), verify.
    fn verify_aggregated_signature(&self, aggregated_signature: Bytes, hash: Bytes, voters: Vec<Bytes>) -> Result<(), Box<dyn Error + Send>> {
        let (v, vl) = concat(&voters);
        check(unsafe {
            ffi::ovh_verify_aggregated(self.raw(), aggregated_signature.as_ptr(), aggregated_signature.len(),
                                       hash.as_ptr(), hash.len(), v.as_ptr(), vl.as_ptr(), vl.len())
        })
    }
}

/// Backend selection beside `ConsensusConfig` (reference `src/config.rs:18-31`): the node reads
/// `crypto_backend` ("blst", the default, or "hip") and `crypto_devices` from its
/// `[consensus_overlord]` section and builds `ConsensusCrypto` or `HipCrypto` accordingly; the
/// `Overlord<…, C, …>` type parameter becomes an enum forwarding the five trait methods.
#[derive(Clone, Debug, PartialEq)]
pub enum CryptoBackend {
    Blst,
    Hip { devices: Vec<i32> },
}

impl CryptoBackend {
    pub fn from_config(backend: &str, devices: &[i32]) -> Option<Self> {
        match backend {
            "" | "blst" => Some(CryptoBackend::Blst),
            "hip" => Some(CryptoBackend::Hip { devices: devices.to_vec() }),
            _ => None,
        }
    }
}

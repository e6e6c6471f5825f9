//! Raw bindings of include/ovhip.h (the C ABI of libovhip.so). One declaration per prototype of
//! the header, same names, same argument order; tests/test_crate_ffi.py compares the two
//! mechanically. Type mapping: int -> i32, size_t -> usize, uintN_t -> uN, int32_t -> i32,
//! float -> f32, `const T*` -> `*const T`, `T*` and `T out[k]` -> `*mut T`, void* -> *mut c_void.
#![allow(non_camel_case_types)]
use std::os::raw::{c_char, c_void};

/// Opaque context (`ovh_ctx` in the header): device buffers, HIP streams, the vote pool and the
/// validator table of one or more GPUs.
#[repr(C)]
pub struct OvhCtx {
    _p: [u8; 0],
}

pub const OVH_OK: i32 = 0;
pub const OVH_ERR_HASH_LEN: i32 = 100;
pub const OVH_ERR_LEN_MISMATCH: i32 = 101;
pub const OVH_ERR_PUBKEY: i32 = 102;
pub const OVH_ERR_ARG: i32 = 103;
pub const OVH_ERR_DEVICE: i32 = 200;
pub const OVH_ERR_RNG: i32 = 201;

pub const OVH_FLAG_AGG_NO_GROUPCHECK: u32 = 0x1;
pub const OVH_FLAG_PROFILE: u32 = 0x2;
pub const OVH_FLAG_VM_TRACE: u32 = 0x4;
pub const OVH_FLAG_TEST_RLC: u32 = 0x8;
pub const OVH_FLAG_SK_RAW: u32 = 0x10;
pub const OVH_FLAG_VM_CLOCK: u32 = 0x20;
/// The vote pool on CU-masked streams leaving 8 CUs to other kernels (RCCL between shard batches).
pub const OVH_FLAG_POOL_RESERVE: u32 = 0x40;

pub const OVH_NSTAGES: usize = 6;
pub const OVH_VOTE_HASH_MAX: usize = 64;
pub const OVH_PARTIAL_BYTES: usize = 864;
pub const OVH_BATCH_SLOTS: usize = 6;

extern "C" {
    pub fn ovh_create(device: i32, dst: *const u8, dst_len: usize, flags: u32) -> *mut OvhCtx;
    pub fn ovh_create_multi(devices: *const i32, ndev: i32, dst: *const u8, dst_len: usize, flags: u32) -> *mut OvhCtx;
    pub fn ovh_multi_peer_matrix(ctx: *mut OvhCtx, out: *mut u8, cap: usize) -> i32;
    pub fn ovh_destroy(ctx: *mut OvhCtx);
    pub fn ovh_device_count(ctx: *mut OvhCtx) -> i32;
    pub fn ovh_stream(ctx: *mut OvhCtx) -> *mut c_void;
    pub fn ovh_sm3(msg: *const u8, len: usize, out: *mut u8) -> i32;
    pub fn ovh_vote_digests_device(ctx: *mut OvhCtx, n: usize, heights: *const u64, rounds: *const u64, vote_types: *const u8, block_hashes: *const u8, hash_lens: *const u8, digests: *mut u8) -> i32;
    pub fn ovh_vote_digests(ctx: *mut OvhCtx, n: usize, heights: *const u64, rounds: *const u64, vote_types: *const u8, block_hashes: *const u8, hash_lens: *const u8, digests: *mut u8) -> i32;
    pub fn ovh_sk_parse(ctx: *mut OvhCtx, key: *const u8, key_len: usize, out_scalar: *mut u8) -> i32;
    pub fn ovh_sign(ctx: *mut OvhCtx, key: *const u8, key_len: usize, hash: *const u8, hash_len: usize, out: *mut u8) -> i32;
    pub fn ovh_sk_to_pk(ctx: *mut OvhCtx, key: *const u8, key_len: usize, out: *mut u8) -> i32;
    pub fn ovh_verify(ctx: *mut OvhCtx, sig: *const u8, sig_len: usize, hash: *const u8, hash_len: usize, pk: *const u8, pk_len: usize) -> i32;
    pub fn ovh_aggregate_sigs(ctx: *mut OvhCtx, sigs: *const u8, sig_lens: *const usize, n_sigs: usize, pks: *const u8, pk_lens: *const usize, n_pks: usize, out: *mut u8) -> i32;
    pub fn ovh_aggregate_pks(ctx: *mut OvhCtx, pks: *const u8, pk_lens: *const usize, n: usize, out: *mut u8) -> i32;
    pub fn ovh_verify_aggregated(ctx: *mut OvhCtx, agg_sig: *const u8, agg_len: usize, hash: *const u8, hash_len: usize, pks: *const u8, pk_lens: *const usize, n: usize) -> i32;
    pub fn ovh_set_validators(ctx: *mut OvhCtx, pks: *const u8, n: usize) -> i32;
    pub fn ovh_verify_batch(ctx: *mut OvhCtx, n: usize, sigs: *const u8, hashes: *const u8, pks: *const u8, codes: *mut i32) -> i32;
    pub fn ovh_prefetch(ctx: *mut OvhCtx, n: usize, sigs: *const u8, hashes: *const u8, pks: *const u8) -> i32;
    pub fn ovh_cache_config(ctx: *mut OvhCtx, capacity: usize) -> i32;
    pub fn ovh_cache_stats(ctx: *mut OvhCtx, stats: *mut u64) -> i32;
    pub fn ovh_samemsg_stats(ctx: *mut OvhCtx, stats: *mut u64) -> i32;
    pub fn ovh_msg_cache_stats(ctx: *mut OvhCtx, stats: *mut u64) -> i32;
    pub fn ovh_verify_qc_batch(ctx: *mut OvhCtx, nq: usize, sigs: *const u8, hashes: *const u8, bitmaps: *const u8, bitmap_len: usize, codes: *mut i32) -> i32;
    pub fn ovh_set_test_rlc(ctx: *mut OvhCtx, seed: u64, index_base: u64) -> i32;
    pub fn ovh_verify_batch_device(ctx: *mut OvhCtx, n: usize, d_sigs: *const u8, d_hashes: *const u8, d_pks: *const u8, d_codes: *mut i32) -> i32;
    pub fn ovh_batch_partial_device(ctx: *mut OvhCtx, n: usize, d_sigs: *const u8, d_hashes: *const u8, d_pks: *const u8, d_codes: *mut i32, d_partial: *mut u8, stream: *mut c_void) -> i32;
    pub fn ovh_combine_partials_device(ctx: *mut OvhCtx, k: usize, d_partials: *const u8, verdict: *mut i32) -> i32;
    pub fn ovh_batch_fallback_device(ctx: *mut OvhCtx, n: usize, d_codes: *mut i32) -> i32;
    pub fn ovh_verify_batch_device_async(ctx: *mut OvhCtx, n: usize, d_sigs: *const u8, d_hashes: *const u8, d_pks: *const u8, d_codes: *mut i32) -> i32;
    pub fn ovh_verify_samemsg_device_async(ctx: *mut OvhCtx, n: usize, d_sigs: *const u8, hash: *const u8, d_pks: *const u8, d_codes: *mut i32) -> i32;
    pub fn ovh_verify_batch_async(ctx: *mut OvhCtx, n: usize, sigs: *const u8, hashes: *const u8, pks: *const u8, codes: *mut i32) -> i32;
    pub fn ovh_batch_wait(ctx: *mut OvhCtx) -> i32;
    pub fn ovh_combine_partials_device_async(ctx: *mut OvhCtx, k: usize, d_partials: *const u8, n: usize, d_codes: *mut i32, stream: *mut c_void) -> i32;
    pub fn ovh_stage_times(ctx: *mut OvhCtx, ms: *mut f32, max: usize) -> i32;
    pub fn ovh_stage_name(stage: i32) -> *const c_char;
    pub fn ovh_vote_spans(ctx: *mut OvhCtx, ms: *mut f32, max: usize) -> i32;
    pub fn ovh_vm_trace(ctx: *mut OvhCtx, prog: i32, stamps: *mut u64, max: usize) -> i32;
    pub fn ovh_diag_vm_occupancy(ctx: *mut OvhCtx, prog: i32, n: usize, reps: i32, streams: i32, ms: *mut f32) -> i32;
    pub fn ovh_vm_clock(ctx: *mut OvhCtx, stamps: *mut u64, max: usize) -> i32;
    pub fn ovh_pool_log(ctx: *mut OvhCtx, words: *mut u64, max: usize) -> i32;
    pub fn ovh_sign_batch_device(ctx: *mut OvhCtx, n: usize, d_sks: *const u8, d_hashes: *const u8, d_sigs: *mut u8) -> i32;
    pub fn ovh_sk_to_pk_batch_device(ctx: *mut OvhCtx, n: usize, d_sks: *const u8, d_pks: *mut u8) -> i32;
}

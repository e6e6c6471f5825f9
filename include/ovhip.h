/*
 * libovhip — MI355X (gfx950) BLS12-381 signature backend for the overlord `Crypto` trait of
 * cita-cloud/consensus_overlord. C ABI: plain pointers and sizes, caller-owned host buffers,
 * no pointer is retained after a call returns. All arithmetic runs in HIP kernels; there is
 * no CPU fallback (a missing/failed device returns OVH_ERR_DEVICE).
 *
 * Return codes (int):
 *   0        OK
 *   1..7     BLST_ERROR of the failing signature parse / aggregate / verify
 *            (BAD_ENCODING, POINT_NOT_ON_CURVE, POINT_NOT_IN_GROUP, AGGR_TYPE_MISMATCH,
 *             VERIFY_FAIL, PK_IS_INFINITY, BAD_SCALAR)   -> ConsensusError::CryptoErr
 *   100      hash is not 32 bytes      -> ConsensusError::Other("failed to convert hash value")
 *   101      len(signatures) != len(voters)
 *                                     -> Other("signatures length does not match voters length")
 *   102      a public key does not parse -> Other("lose public key")
 *   103      invalid argument (NULL pointer, n too large)
 *   200      HIP device error
 *
 * Variable-length lists (Rust `Vec<Bytes>`) are passed as one concatenated byte buffer plus
 * an array of item lengths.
 */
#ifndef OVHIP_H
#define OVHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ovh_ctx ovh_ctx;

#define OVH_OK 0
#define OVH_ERR_HASH_LEN 100
#define OVH_ERR_LEN_MISMATCH 101
#define OVH_ERR_PUBKEY 102
#define OVH_ERR_ARG 103
#define OVH_ERR_DEVICE 200

/* Flags for ovh_create. */
#define OVH_FLAG_AGG_NO_GROUPCHECK 0x1u /* aggregate_signatures without the G2 subgroup check */
#define OVH_FLAG_PROFILE 0x2u           /* record HIP events around every batch stage */
#define OVH_FLAG_VM_TRACE 0x4u          /* diagnostics: per-phase clock of the VM kernels' workgroup 0 */

/* Batch stages (ovh_stage_name gives the label). Each stage is one or more kernels enqueued
 * back to back on ovh_stream. */
#define OVH_NSTAGES 5

/* Create a context on HIP device `device` with hash-to-curve domain separation tag `dst`
 * (NULL -> "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_", the believed ophelia-blst DST).
 * Replaces ConsensusCrypto::new's crypto state (src/consensus.rs:347-359). NULL on failure. */
ovh_ctx* ovh_create(int device, const uint8_t* dst, size_t dst_len, uint32_t flags);
void ovh_destroy(ovh_ctx* ctx);
/* The HIP stream (hipStream_t) all of the context's kernels run on. */
void* ovh_stream(ovh_ctx* ctx);

/* Crypto::hash -> util.rs:83-87 sm3_hash. */
int ovh_sm3(const uint8_t* msg, size_t len, uint8_t out[32]);

/* Crypto::sign (consensus.rs:390-395): sigma = sk * H(hash), 96-byte compressed.
 * sk: 32-byte big-endian scalar, 0 < sk < r (else BLST_BAD_ENCODING). */
int ovh_sign(ovh_ctx* ctx, const uint8_t* sk, size_t sk_len, const uint8_t* hash, size_t hash_len, uint8_t out[96]);
/* BlsPrivateKey::pub_key + to_bytes (consensus.rs:352,357): 48-byte compressed pk. */
int ovh_sk_to_pk(ovh_ctx* ctx, const uint8_t* sk, size_t sk_len, uint8_t out[48]);

/* Crypto::verify_signature (consensus.rs:397-416). */
int ovh_verify(ovh_ctx* ctx, const uint8_t* sig, size_t sig_len, const uint8_t* hash, size_t hash_len,
               const uint8_t* pk, size_t pk_len);

/* Crypto::aggregate_signatures (consensus.rs:418-444): 96-byte compressed sum. */
int ovh_aggregate_sigs(ovh_ctx* ctx, const uint8_t* sigs, const size_t* sig_lens, size_t n_sigs,
                       const uint8_t* pks, const size_t* pk_lens, size_t n_pks, uint8_t out[96]);

/* BlsPublicKey::aggregate (consensus.rs:371): 48-byte compressed sum. */
int ovh_aggregate_pks(ovh_ctx* ctx, const uint8_t* pks, const size_t* pk_lens, size_t n, uint8_t out[48]);

/* Crypto::verify_aggregated_signature (consensus.rs:446-462, 365-382). */
int ovh_verify_aggregated(ovh_ctx* ctx, const uint8_t* agg_sig, size_t agg_len, const uint8_t* hash, size_t hash_len,
                          const uint8_t* pks, const size_t* pk_lens, size_t n);

/* Batched verify_signature over n votes (fixed-size compressed encodings):
 * sigs n x 96 B, hashes n x 32 B, pks n x 48 B -> codes[n] with exactly the per-vote
 * ovh_verify result. Random-linear-combination check (64-bit scalars from `seed`) with a
 * per-vote fallback when the combined check fails. Returns 0 if the batch ran (the verdicts
 * are in codes), else an error. Host buffers. */
int ovh_verify_batch(ovh_ctx* ctx, size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks,
                     uint64_t seed, int32_t* codes);

/* The same with device-resident inputs/outputs (pointers into HBM), enqueued on ovh_stream;
 * the call returns after the batch completed. */
int ovh_verify_batch_device(ovh_ctx* ctx, size_t n, const uint8_t* d_sigs, const uint8_t* d_hashes,
                            const uint8_t* d_pks, uint64_t seed, int32_t* d_codes);

/* Multi-GPU split of ovh_verify_batch_device: per-shard partial = {Fp12 product of the
 * shard's Miller outputs (576 B), projective G2 sum of r_i sigma_i (288 B)} = 864 bytes,
 * written to d_partial (device memory). Per-vote parse/subgroup codes go to d_codes.
 * The G2 sum is in homogeneous projective coordinates (X : Y : Z), O = (0 : 1 : 0). */
#define OVH_PARTIAL_BYTES 864
int ovh_batch_partial_device(ovh_ctx* ctx, size_t n, const uint8_t* d_sigs, const uint8_t* d_hashes,
                             const uint8_t* d_pks, uint64_t seed, int32_t* d_codes, uint8_t* d_partial);
/* Combine k partials (device memory, k x 864 B): returns 1 if prod f * e(-G1, sum S) == 1
 * after the final exponentiation, 0 if not, <0 on device error. */
int ovh_combine_partials_device(ovh_ctx* ctx, size_t k, const uint8_t* d_partials);
/* Per-vote fallback for a shard whose combined check failed: codes[i] (device) updated to the
 * exact per-vote verify result for every vote whose code is still 0. */
int ovh_batch_fallback_device(ovh_ctx* ctx, size_t n, int32_t* d_codes);

/* Pipelined batches. ovh_verify_batch_device_async enqueues one batch and returns without
 * waiting: the per-vote stages run on ovh_stream, the combined check and (device-gated) per-vote
 * fallback on a second, lower-priority stream, so batch k's final exponentiation overlaps batch
 * k + 1's per-vote work. Up to OVH_BATCH_SLOTS batches may be in flight per context; the
 * d_codes of a batch must stay untouched until ovh_batch_wait returns, after which they hold
 * exactly the per-vote ovh_verify results. ovh_verify_batch_device = the async call +
 * ovh_batch_wait. */
#define OVH_BATCH_SLOTS 2 /* batches in flight per context (state slots) */
int ovh_verify_batch_device_async(ovh_ctx* ctx, size_t n, const uint8_t* d_sigs, const uint8_t* d_hashes,
                                  const uint8_t* d_pks, uint64_t seed, int32_t* d_codes);
int ovh_batch_wait(ovh_ctx* ctx);
/* Multi-GPU form: after ovh_batch_partial_device (n votes of this rank) and the all-gather of
 * the k <= 16 partials, enqueue the combined check and, if it fails, the per-vote fallback of
 * this rank's n votes into d_codes, on the second stream; ovh_batch_wait completes it. */
int ovh_combine_partials_device_async(ovh_ctx* ctx, size_t k, const uint8_t* d_partials, size_t n,
                                      int32_t* d_codes);

/* Device time (ms, HIP events on ovh_stream) of each stage of the most recent batch call
 * (ovh_verify_batch_device / ovh_batch_partial_device / ovh_combine_partials_device /
 * ovh_batch_fallback_device) on a context created with OVH_FLAG_PROFILE; stages that did not
 * run read 0. Fills min(max, OVH_NSTAGES) entries and returns that count (0 without the
 * flag, <0 on error). */
int ovh_stage_times(ovh_ctx* ctx, float* ms, size_t max);
const char* ovh_stage_name(int stage);

/* Diagnostics (context created with OVH_FLAG_VM_TRACE): the wall clock (100 MHz counter)
 * workgroup 0 of the last launch of VM program `prog` (0 vote, 1 fold, 2 final, 3 pairchk)
 * read after each phase barrier: copies min(max, nphases + 1) stamps, returns nphases + 1
 * (0 without the flag, <0 on error). */
int ovh_vm_trace(ovh_ctx* ctx, int prog, uint64_t* stamps, size_t max);

/* Batched helpers used to synthesise workloads on the device. */
int ovh_sign_batch_device(ovh_ctx* ctx, size_t n, const uint8_t* d_sks, const uint8_t* d_hashes, uint8_t* d_sigs);
int ovh_sk_to_pk_batch_device(ovh_ctx* ctx, size_t n, const uint8_t* d_sks, uint8_t* d_pks);

#ifdef __cplusplus
}
#endif

#endif /* OVHIP_H */

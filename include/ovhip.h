/*
 * libovhip — MI355X (gfx950) BLS12-381 signature backend for the overlord `Crypto` trait of
 * cita-cloud/consensus_overlord. C ABI: plain pointers and sizes, caller-owned host buffers,
 * no pointer is retained after a call returns. All curve arithmetic runs in HIP kernels; there
 * is no CPU fallback (a missing/failed device returns OVH_ERR_DEVICE). Every entry point is
 * thread-safe: a context serialises its device work internally (the trait object is Send +
 * Sync and is called concurrently by overlord and the gRPC check_block handler,
 * src/main.rs:107-127 -> src/consensus.rs:176).
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
 *   103      invalid argument (NULL pointer, n too large, wrong context kind)
 *   200      HIP device error
 *   201      the OS random source (getrandom) failed
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
/* A HIP error, or a batch's final stream gave up waiting for the vote pool. The latter is
 * sticky: every later synchronising call of the context (ovh_batch_wait, the synchronous batch
 * and partial / combine / fallback entry points) returns it, and the context must be destroyed. */
#define OVH_ERR_DEVICE 200
#define OVH_ERR_RNG 201

/* Flags for ovh_create / ovh_create_multi. */
#define OVH_FLAG_AGG_NO_GROUPCHECK 0x1u /* aggregate_signatures without the G2 subgroup check */
#define OVH_FLAG_PROFILE 0x2u           /* record HIP events around every batch stage */
#define OVH_FLAG_VM_TRACE 0x4u          /* diagnostics: per-phase clock of the VM kernels' workgroup 0 */
#define OVH_FLAG_TEST_RLC 0x8u          /* TESTS ONLY: batch coefficients from ovh_set_test_rlc (predictable) */
#define OVH_FLAG_SK_RAW 0x10u           /* private key = 32-byte big-endian scalar 0 < sk < r (blst
                                           SecretKey::from_bytes) instead of KeyGen (see ovh_sk_parse) */
#define OVH_FLAG_VM_CLOCK 0x20u         /* diagnostics: shader / wall clock stamps around every vote
                                           workgroup's program (ovh_vm_clock) */
#define OVH_FLAG_POOL_RESERVE 0x40u     /* the vote pool leaves 8 compute units (one per XCD; env
                                           OVH_POOL_RESERVE: another multiple of 8, <= 64) free for
                                           other kernels -- the caller's collective between shard
                                           batches -- and shard batches (ovh_batch_partial_device*,
                                           ovh_create_multi) share the persistent pool instead of a grid
                                           per batch. Use for a context whose partials cross RCCL. */

/* Batch stages (ovh_stage_name gives the label). Each stage is one or more kernels. */
#define OVH_NSTAGES 6

/* Create a context on HIP device `device` with hash-to-curve domain separation tag `dst`
 * (NULL -> "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_", the believed ophelia-blst DST).
 * Replaces ConsensusCrypto::new's crypto state (src/consensus.rs:347-359). NULL on failure. */
ovh_ctx* ovh_create(int device, const uint8_t* dst, size_t dst_len, uint32_t flags);
/* One context over several GPUs of this process: ovh_verify_batch and
 * ovh_prefetch split a batch into contiguous shards, one per device; each device computes its
 * shard's 864-byte partial, the partials are copied peer-to-peer (xGMI) to devices[0], which
 * runs the one combined check; on failure every device bisects its own shard. Single-call
 * entry points rotate over the devices. Devices may repeat (tests use {0, 0}); 1 <= ndev <= 8. */
ovh_ctx* ovh_create_multi(const int* devices, int ndev, const uint8_t* dst, size_t dst_len, uint32_t flags);
/* Peer access of a context's devices: out[a * n + b] = 1 when device a reaches device b's memory
 * directly (xGMI; enabled by ovh_create_multi for every pair hipDeviceCanAccessPeer allows) or a
 * and b are one device, 0 when copies between them stage through the host. Returns n (the
 * device count), or OVH_ERR_ARG when cap < n * n. The pipelined combined check
 * (ovh_verify_batch_async) rotates over the devices with peer access to and from every other. */
int ovh_multi_peer_matrix(ovh_ctx* ctx, uint8_t* out, size_t cap);
/* Synchronises every stream of the context and frees its device memory. The streams themselves
 * are not destroyed: they are parked per device and priority and handed to later contexts of
 * that device, so an ovh_stream handle -- and any event a caller recorded on it, e.g. torch's
 * pinned-host allocator after a non-blocking copy issued on ExternalStream(ovh_stream(ctx)) --
 * stays valid for the life of the process. Work a caller enqueued on ovh_stream before
 * ovh_destroy completes before the call returns. */
void ovh_destroy(ovh_ctx* ctx);
/* Number of devices of the context (1 for ovh_create). */
int ovh_device_count(ovh_ctx* ctx);
/* The HIP stream (hipStream_t) the context's per-vote kernels run on (first device). */
void* ovh_stream(ovh_ctx* ctx);

/* Crypto::hash -> util.rs:83-87 sm3_hash. */
int ovh_sm3(const uint8_t* msg, size_t len, uint8_t out[32]);

/* Vote digests on the device: digest i = SM3(rlp(Vote{height, round,
 * vote_type, block_hash})), the hash overlord signs and Consensus::check_block rebuilds
 * (consensus.rs:169-175 -> util.rs:83-87), so the batching shim can ship raw votes and feed the
 * digests straight to ovh_verify_batch_device. Vote i's block hash is the first hash_lens[i]
 * (<= OVH_VOTE_HASH_MAX; 0 = the empty hash of a nil vote) bytes at block_hashes + 64 i.
 * _device: every pointer is device memory, the kernel is enqueued on ovh_stream and the call
 * returns without waiting (stream order). Host form: host buffers, synchronous. */
#define OVH_VOTE_HASH_MAX 64
int ovh_vote_digests_device(ovh_ctx* ctx, size_t n, const uint64_t* heights, const uint64_t* rounds,
                            const uint8_t* vote_types, const uint8_t* block_hashes, const uint8_t* hash_lens,
                            uint8_t* digests);
int ovh_vote_digests(ovh_ctx* ctx, size_t n, const uint64_t* heights, const uint64_t* rounds, const uint8_t* vote_types,
                     const uint8_t* block_hashes, const uint8_t* hash_lens, uint8_t* digests);

/* BlsPrivateKey::try_from (consensus.rs:349-350, ophelia-blst [dep]): the 32-byte scalar the
 * context signs with, big-endian. Default: IETF KeyGen (blst SecretKey::key_gen(key, ""):
 * HKDF-SHA256, key >= 32 bytes) -- the reference's own example/private_key is >= r, so the
 * parse cannot be blst's strict from_bytes. With OVH_FLAG_SK_RAW: 32 bytes, 0 < sk < r.
 * BLST_BAD_ENCODING (1) when the key does not parse. Host only (no device work). */
int ovh_sk_parse(ovh_ctx* ctx, const uint8_t* key, size_t key_len, uint8_t out_scalar[32]);

/* Crypto::sign (consensus.rs:390-395): sigma = sk * H(hash), 96-byte compressed; `key` is the
 * private key bytes as ConsensusCrypto::new reads them (ovh_sk_parse). */
int ovh_sign(ovh_ctx* ctx, const uint8_t* key, size_t key_len, const uint8_t* hash, size_t hash_len, uint8_t out[96]);
/* BlsPrivateKey::pub_key + to_bytes (consensus.rs:352,357): 48-byte compressed pk. */
int ovh_sk_to_pk(ovh_ctx* ctx, const uint8_t* key, size_t key_len, uint8_t out[48]);

/* Crypto::verify_signature (consensus.rs:397-416). Answers from the verdict cache when the
 * (sig, hash, voter) triple was batch-verified by ovh_prefetch; otherwise one device check. */
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

/* ConsensusCrypto::update_pubkeys (consensus.rs:361-363; callers proc_reconfigure :131-136 and
 * Brain::commit :622-629): n x 48-byte compressed validator keys, in the order the node's config
 * lists them. Each key is decompressed and group-checked once on the device and kept as a
 * point in HBM. ovh_verify_batch / ovh_prefetch then skip the per-vote key decompression for
 * voters found in the table, and ovh_verify_qc_batch selects QC voters from it. Keys that do
 * not parse are kept (their votes answer 102, as the reference's per-call parse would). */
int ovh_set_validators(ovh_ctx* ctx, const uint8_t* pks, size_t n);

/* Batched verify_signature over n votes (fixed-size compressed encodings):
 * sigs n x 96 B, hashes n x 32 B, pks n x 48 B -> codes[n], codes[i] == the ovh_verify result
 * for vote i. One random-linear-combination check with secret 64-bit coefficients (a fresh
 * getrandom seed per batch) and, when it fails, a bisection: 16-vote groups, then per-vote
 * checks in the failing groups on the device-resident Miller outputs. Host buffers. */
int ovh_verify_batch(ovh_ctx* ctx, size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks,
                     int32_t* codes);

/* Vote-batching ingress: batch-verify n votes as they arrive at
 * proc_network_msg (consensus.rs:210-262) and keep each verdict in the context's cache, keyed
 * by the exact (sig, hash, voter) bytes; overlord's later serial verify_signature calls
 * (ovh_verify) are then answered from the cache. Bounded FIFO cache (ovh_cache_config). */
int ovh_prefetch(ovh_ctx* ctx, size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks);
/* Cache capacity in entries (0 disables the cache and empties it). Default 65536. */
int ovh_cache_config(ovh_ctx* ctx, size_t capacity);
/* stats[0] = hits, stats[1] = misses (fixed-size triples not in the cache), stats[2] = entries. */
int ovh_cache_stats(ovh_ctx* ctx, uint64_t stats[3]);
/* Same-message batches (ovh_verify_batch / ovh_prefetch on one device): when the n votes of a
 * call sign at most n / 2 distinct hashes (a round's votes all sign hash(rlp(Vote)), which has no
 * voter field: consensus.rs:169-175), the batch is checked as prod_g e(sum_{i in g} r_i pk_i, H_g)
 * e(-G1, sum_i r_i sigma_i) == 1 with one hash_to_G2 and one Miller loop per distinct hash
 * (per vote only the key and signature checks and r_i pk_i), then bisected per vote on failure;
 * the codes are the per-call codes as for any batch. By default the path takes batches of more
 * than OVH_SMALL_MAX (1,024) votes: below that the small-batch path (one wave per vote, one final
 * exponentiation) has the lower latency. The environment variable
 * OVH_SAMEMSG (read at ovh_create) selects 0 = never, 1 = above the small-batch size (default),
 * 2 = every batch with at most n / 2 distinct hashes (the least device work per vote). Counters
 * since ovh_create: stats[0] such batches, stats[1] their votes, stats[2] their distinct hashes. */
int ovh_samemsg_stats(ovh_ctx* ctx, uint64_t stats[3]);
/* Message cache of the per-call verify (ovh_verify, ovh_verify_batch with n = 1): H =
 * hash_to_G2(hash) of the last 256 hashes verified per call, so every later vote on a hash (all
 * votes of a round sign the same hash, consensus.rs:397-416) skips hash_to_G2. stats[0] = hits,
 * stats[1] = misses, summed over a multi-device context's devices. */
int ovh_msg_cache_stats(ovh_ctx* ctx, uint64_t stats[2]);

/* Batched QC verification for block sync (check_block, consensus.rs:143-207): QC j = aggregated
 * signature sigs[j] (96 B) over hashes[j] (32 B, the SM3 of rlp(Vote{h, r, Precommit, block})),
 * signed by the validators whose bits are set in bitmaps[j] (bitmap_len bytes, MSB first) over
 * the validator table sorted by key bytes (overlord extract_voters over the address-sorted
 * authority list; validators_to_nodes uses the key bytes as the address, util.rs:69-77).
 * codes[j] == ovh_verify_aggregated(sigs[j], hashes[j], those voters). One RLC batch over all
 * QCs. Needs ovh_set_validators. */
int ovh_verify_qc_batch(ovh_ctx* ctx, size_t nq, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* bitmaps,
                        size_t bitmap_len, int32_t* codes);

/* TESTS ONLY (context created with OVH_FLAG_TEST_RLC, else OVH_ERR_ARG): vote i of every
 * following batch gets the coefficient SplitMix64(seed, index_base + i). Predictable
 * coefficients let an adversary cancel invalid signatures inside the combined check
 * (tests/test_rlc_soundness.py); production contexts never use this. */
int ovh_set_test_rlc(ovh_ctx* ctx, uint64_t seed, uint64_t index_base);

/* The same as ovh_verify_batch with device-resident inputs/outputs (pointers into HBM), enqueued
 * on the context's streams; returns after the batch completed. */
int ovh_verify_batch_device(ovh_ctx* ctx, size_t n, const uint8_t* d_sigs, const uint8_t* d_hashes,
                            const uint8_t* d_pks, int32_t* d_codes);

/* Multi-GPU split of ovh_verify_batch_device (one process per GPU): per-shard partial =
 * {Fp12 product of the shard's Miller outputs (576 B), projective G2 sum of r_i sigma_i
 * (288 B)} = 864 bytes, written to d_partial (device memory); per-vote parse/subgroup codes go
 * to d_codes. The G2 sum is in homogeneous projective coordinates (X : Y : Z), O = (0 : 1 : 0).
 * Stream order: `stream` (a hipStream_t of the caller, e.g. torch's current stream) -- the
 * partial is written after the work already on `stream` (so a gather buffer can be reused) and
 * `stream` waits for the write; the call returns without blocking. stream NULL: the call
 * returns once d_partial is written. The inputs (d_sigs, d_hashes, d_pks) are read in
 * ovh_stream(ctx) order: a caller that produced them on another stream first makes ovh_stream
 * wait for it (shard.py does, through an event). */
#define OVH_PARTIAL_BYTES 864
int ovh_batch_partial_device(ovh_ctx* ctx, size_t n, const uint8_t* d_sigs, const uint8_t* d_hashes,
                             const uint8_t* d_pks, int32_t* d_codes, uint8_t* d_partial, void* stream);
/* Combine k partials (device memory, k x 864 B): *verdict = 1 if prod f * e(-G1, sum S) == 1
 * after the final exponentiation, else 0. Synchronous; returns 0 or an error code. */
int ovh_combine_partials_device(ovh_ctx* ctx, size_t k, const uint8_t* d_partials, int32_t* verdict);
/* Bisection of the last ovh_batch_partial_device shard (its combined check failed): d_codes[i]
 * still 0 -> the exact per-vote verify result. Synchronous. */
int ovh_batch_fallback_device(ovh_ctx* ctx, size_t n, int32_t* d_codes);

/* Pipelined batches. ovh_verify_batch_device_async enqueues one batch and returns without
 * waiting: the batch is staged and published on ovh_stream (its signatures and keys copied into
 * the library's own buffer, its hashes through hash_to_field), its per-vote work runs in the
 * context's vote pool (persistent workgroups that take 4-vote quads of the published batches in
 * order), and its combined check and (device-gated) bisection on a lower-priority final stream,
 * so batch k's final exponentiation overlaps later batches' per-vote work. The inputs are read
 * in ovh_stream order: they must be ready when the work enqueued there before the call is done,
 * and work enqueued there after the call may overwrite them. Up to OVH_BATCH_SLOTS batches may be
 * in flight per context; the d_codes of a batch must stay untouched until ovh_batch_wait
 * returns, after which they hold exactly the per-vote ovh_verify results. */
#define OVH_BATCH_SLOTS 6 /* batches in flight per context (state slots) */
int ovh_verify_batch_device_async(ovh_ctx* ctx, size_t n, const uint8_t* d_sigs, const uint8_t* d_hashes,
                                  const uint8_t* d_pks, int32_t* d_codes);
/* The pipelined same-message form: n votes in device memory that all sign the 32-byte `hash`
 * (host memory, read before the call returns) -- a round's precommits. One hash_to_G2 and one
 * key-sum Miller loop for the batch, the per-vote key and signature checks and RLC products on
 * two per-vote streams in turn (consecutive batches co-resident); codes
 * as ovh_verify_batch_device_async (exactly the per-vote ovh_verify results after
 * ovh_batch_wait, the same OVH_BATCH_SLOTS limit). The inputs are read after the caller's work
 * enqueued on ovh_stream before the call, and -- unlike that API's -- must stay untouched until
 * ovh_batch_wait returns, like the codes. Replaces,
 * for a round's votes, overlord calling Crypto::verify_signature (consensus.rs:397-416) once per
 * SignedVote. Single-device contexts. */
int ovh_verify_samemsg_device_async(ovh_ctx* ctx, size_t n, const uint8_t* d_sigs, const uint8_t* hash,
                                    const uint8_t* d_pks, int32_t* d_codes);
/* The pipelined form with host buffers, for single- and multi-device contexts (a node with no
 * torch; ovh_create_multi is its multi-GPU path): the inputs are copied into pinned staging
 * before the call returns (the caller may reuse them at once); `codes` (host, n entries) must
 * stay valid and is written by a later call of this function or ovh_batch_wait. Per batch each
 * device runs its shard's per-vote stages on its own pipeline, the partials go peer-to-peer
 * (xGMI) to the batch's final device, which rotates over the devices batch by batch, and each
 * device bisects its own shard when the combined check fails. At most OVH_BATCH_SLOTS batches
 * are in flight: a further call first completes the oldest. The caller's current HIP device is
 * unchanged on return. */
int ovh_verify_batch_async(ovh_ctx* ctx, size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks,
                           int32_t* codes);
/* Completes every batch in flight on the context (device or host form, any context kind). */
int ovh_batch_wait(ovh_ctx* ctx);
/* Multi-GPU form: after ovh_batch_partial_device (n votes of this rank) and the all-gather of
 * the k <= 16 partials on `stream`, enqueue (stream-ordered after the gather) the combined check
 * and, if it fails, the bisection of this rank's n votes into d_codes; `stream` waits until the
 * partials were read. ovh_batch_wait completes it. */
int ovh_combine_partials_device_async(ovh_ctx* ctx, size_t k, const uint8_t* d_partials, size_t n,
                                      int32_t* d_codes, void* stream);

/* Device time (ms, HIP events) of each stage of the most recent batch call on a context created
 * with OVH_FLAG_PROFILE; stages that did not run read 0. Fills min(max, OVH_NSTAGES) entries
 * and returns that count (0 without the flag, <0 on error). */
int ovh_stage_times(ovh_ctx* ctx, float* ms, size_t max);
const char* ovh_stage_name(int stage);
/* Diagnostics (context created with OVH_FLAG_PROFILE): (start, end) in ms, relative to the
 * first, of the vote kernels of the last batches (up to 256, oldest first) -- pipelined vote
 * grids of consecutive batches overlap, so their device-level rate is the work over the union of
 * these spans. Writes min(count, max / 2) pairs and returns that number; max = 0 forgets the
 * batches recorded so far. */
int ovh_vote_spans(ovh_ctx* ctx, float* ms, size_t max);

/* Diagnostics (context created with OVH_FLAG_VM_TRACE): the wall clock (100 MHz counter) of
 * workgroup 0 of the last launch of VM program `prog` (0 vote, 1 fold, 2 final, 3 vote_t)
 * read after each phase barrier: copies min(max, nphases + 1) stamps, returns nphases + 1
 * (0 without the flag, <0 on error). */
int ovh_vm_trace(ovh_ctx* ctx, int prog, uint64_t* stamps, size_t max);
/* Diagnostics: `reps` batches of n zero votes through a VM program, *ms = wall time. prog 0:
 * vsame launches on one stream (streams = 1) or alternating over two (streams = 2: two
 * launches co-resident when the LDS allows, i.e. two waves per SIMD). prog 1: the vote pool,
 * batches published back to back (staging, hash_to_field, publication; no final-stream work).
 * prog 2: the vote pool with all reps <= OVH_BATCH_SLOTS batches published before its grids
 * start (no gap: the PMC passes' counters cover the batches and no idle wait). */
int ovh_diag_vm_occupancy(ovh_ctx* ctx, int prog, size_t n, int reps, int streams, float* ms);
/* Diagnostics (context created with OVH_FLAG_VM_CLOCK): per workgroup of the last vote / vote_t
 * launch, (delta s_memtime, delta s_memrealtime) around its VM program -- shader cycles and
 * 100 MHz ticks, so the clock the kernel held is delta_memtime / delta_realtime x 100 MHz
 * (MI355X_MICROARCH.md, DVFS give-back). Copies min(max, 2 x workgroups) values, returns
 * 2 x workgroups (0 without the flag, <0 on error). The stamps go to a buffer nothing else
 * reads; without the flag no stamp executes. */
int ovh_vm_clock(ovh_ctx* ctx, uint64_t* stamps, size_t max);

/* Diagnostics (context created with OVH_FLAG_VM_CLOCK): the vote pool's log, a ring of 64 batch
 * records of 2,064 words -- 100 MHz stamps of the batch's stream events (publication, pool done,
 * folds, MSM, final, bisection; word 15 its sequence number), then per quad (< 1,024) its start
 * (bits 0..47; bits 48..59 the SIMD it ran on: XCC, SE, SA, CU, SIMD as 3+2+1+4+2 bits; bits 60..63 how
 * its claim went: 1 last published batch, 2 its SIMD busy, 4 deferred, 8 busy and not deferred) and end. Copies up to `max` words after synchronising;
 * returns the log's size in words (0 without the flag, <0 on error). */
int ovh_pool_log(ovh_ctx* ctx, uint64_t* words, size_t max);

/* Batched helpers used to synthesise workloads on the device; d_sks are 32-byte big-endian
 * scalars (not key files). */
int ovh_sign_batch_device(ovh_ctx* ctx, size_t n, const uint8_t* d_sks, const uint8_t* d_hashes, uint8_t* d_sigs);
int ovh_sk_to_pk_batch_device(ovh_ctx* ctx, size_t n, const uint8_t* d_sks, uint8_t* d_pks);

#ifdef __cplusplus
}
#endif

#endif /* OVHIP_H */

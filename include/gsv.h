/*
 * gsv.h — C ABI of the MI355X-native batch validation engine for geth-sharding's
 * collation-validation hot path (libgsv.so, HIP for gfx950).
 *
 * Plain C linkage, plain pointers and sizes, no torch / HIP types in the signatures, so
 * the reference's Go side can bind it with a cgo preamble exactly as it binds
 * crypto/secp256k1/ext.h today (see INTEGRATION.md for the stub).
 *
 * Every entry point replaces a per-item reference call with a batch:
 *   gsv_ecrecover_batch        <- secp256k1_ext_ecdsa_recover (crypto/secp256k1/ext.h:30-47)
 *                                 via secp256k1.RecoverPubkey (crypto/secp256k1/secp256.go:105-122)
 *                                 / crypto.Ecrecover (crypto/signature_cgo.go:31)
 *   gsv_sender_batch           <- recoverPlain (core/types/transaction_signing.go:222-247)
 *                                 + crypto.ValidateSignatureValues (crypto/crypto.go:181-192)
 *   gsv_tx_sender_batch        <- types.Sender(signer, tx) (core/types/transaction_signing.go:72-89,
 *                                 127-137, 182-184, 218-220) over RLP-encoded txs
 *   gsv_keccak256_batch        <- crypto.Keccak256 (crypto/crypto.go:43-49; crypto/sha3/hashes.go:16)
 *   gsv_chunk_root_batch       <- Collation.CalculateChunkRoot (sharding/collation.go:115-119)
 *                                 = types.DeriveSha(Chunks(body)) (core/types/derive_sha.go:32-41)
 *   gsv_bn256_pairing_check_batch <- bn256.PairingCheck (crypto/bn256/cloudflare/bn256.go:313-327)
 *                                 as driven by the bn256Pairing precompile (core/vm/contracts.go:333-360)
 *   gsv_notary_validate_shards <- the notary's per-collation validation (sharding/notary/notary.go:413-496
 *                                 + sharding/collation.go:193-206 DeserializeBlobToTx + Sender)
 *   gsv_derive_sha_batch       <- types.DeriveSha(list) (core/types/derive_sha.go:32-41) for any
 *                                 DerivableList: tx root (core/block_validator.go:70), receipt root (:92)
 *   gsv_collation_poc_batch    <- Collation.CalculatePOC(salt) (sharding/collation.go:124-136)
 *   gsv_collation_header_verify_batch <- CollationHeader.Hash (sharding/collation.go:66-71) and the
 *                                 proposer signature made by SMCClient.Sign (sharding/mainchain/
 *                                 smc_client.go:245-248, signed at sharding/proposer/proposer.go:83)
 *
 *   gsv_ecrecover_precompile_batch <- the ecrecover precompile's Run (core/vm/contracts.go:78-101)
 *
 * Conventions
 *   - Return value: GSV_SUCCESS (0) or a negative GSV_E_* API/HIP error. A bad ITEM never fails
 *     the batch: it gets a per-item status code (GSV_ST_*) mirroring the reference's errors.
 *   - Host-pointer entry points copy inputs to HBM, run, and copy results back (synchronous).
 *   - *_dev entry points take DEVICE pointers already resident in HBM and a hipStream_t passed
 *     as void*; they only enqueue: they never allocate device memory and never synchronize, so a
 *     *_dev call can be captured into a HIP graph (hipStreamBeginCapture).
 *   - *_dev entry points whose launch depends on host-side arguments (offset tables, chain id,
 *     salt, batch size: chunk root, pairing, notary, DeriveSha, POC, headers) need that exact
 *     argument set PREPARED first by the matching gsv_*_prepare call, which builds the trie plans
 *     and lane tables, uploads them to HBM and sizes the workspace (it may allocate and
 *     synchronize).  Unprepared -> GSV_E_NOT_PREPARED, nothing enqueued.  A context keeps its 32
 *     most recently used prepared shapes (<= 32 GiB); a HIP graph captured from a shape must not
 *     be replayed after that shape was dropped, and the caller orders graph replays against other
 *     uses of the same shape (non-captured calls on different streams are ordered by the library).
 *   - One gsv_ctx per device; a context is safe to use from several threads on distinct streams
 *     for the *_dev calls; host-pointer calls serialize on the context's internal stream.
 *   - stream = NULL selects the context stream, a blocking stream: it is ordered both ways with work
 *     on the process's legacy default (NULL) stream, such as PyTorch's default stream.  Work on other
 *     non-blocking streams is the caller's to order (events), as for any stream argument.  Capture
 *     HIP graphs on an explicit stream (a NULL-stream capture would join that implicit ordering).
 */
#ifndef GSV_H
#define GSV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSV_ABI_VERSION 2 /* 2: streams owned by the context (gsv_stream_create) */

/* ---- API / HIP errors (return values) ---- */
#define GSV_SUCCESS 0
#define GSV_E_INVALID_ARG (-1)
#define GSV_E_HIP (-2)
#define GSV_E_NOMEM (-3)
#define GSV_E_NO_DEVICE (-4)
#define GSV_E_TOO_LARGE (-5) /* e.g. collation body > 2^20 (sharding/collation.go:45) */
#define GSV_E_RCCL (-6)
#define GSV_E_NOT_PREPARED (-7) /* *_dev call whose host-side arguments were not gsv_*_prepare'd */

/* ---- per-item status codes (mirror the reference's error values) ---- */
#define GSV_ST_OK 0
#define GSV_ST_INVALID_MSG_LEN 1   /* secp256k1.ErrInvalidMsgLen       secp256.go:55 */
#define GSV_ST_INVALID_SIG_LEN 2   /* secp256k1.ErrInvalidSignatureLen secp256.go:56 */
#define GSV_ST_INVALID_RECID 3     /* secp256k1.ErrInvalidRecoveryID   secp256.go:57 */
#define GSV_ST_RECOVER_FAILED 4    /* secp256k1.ErrRecoverFailed       secp256.go:61 */
#define GSV_ST_INVALID_SIG 5       /* types.ErrInvalidSig              transaction.go:35 */
#define GSV_ST_INVALID_CHAIN_ID 6  /* types.ErrInvalidChainId          transaction_signing.go */
#define GSV_ST_INVALID_PUBKEY 7    /* "invalid public key"             transaction_signing.go:240 */
#define GSV_ST_BAD_RLP 8           /* rlp decode error of the tx */
#define GSV_ST_BN_BAD_INPUT 9      /* bn256 unmarshal / curve / subgroup failure */
#define GSV_ST_PROPOSER_MISMATCH 10 /* recovered signer != header ProposerAddress */

/* signer kinds for gsv_tx_sender_batch (core/types/transaction_signing.go) */
#define GSV_SIGNER_EIP155 0
#define GSV_SIGNER_HOMESTEAD 1
#define GSV_SIGNER_FRONTIER 2

/* pairing verdicts (core/vm/contracts.go:333-360: true32 / false32 / errBadPairingInput) */
#define GSV_PAIRING_FALSE 0
#define GSV_PAIRING_TRUE 1
#define GSV_PAIRING_BAD_INPUT 2

typedef struct gsv_ctx gsv_ctx;

/* ---- context ---- */
int gsv_device_count(void);
/* Creates a context on HIP device `device`; builds the device-resident precomputed tables
 * (secp256k1 fixed-base comb, Keccak round constants). ~once per process, like the reference's
 * global secp256k1 context (crypto/secp256k1/secp256.go:45-52). */
int gsv_ctx_create(int device, gsv_ctx **out);
void gsv_ctx_destroy(gsv_ctx *ctx);
const char *gsv_error_string(int err);
int gsv_abi_version(void);

/* Kernel timing (HIP events around each launch on the launching stream; off by default). */
int gsv_ctx_set_timing(gsv_ctx *ctx, int enable);
/* kernel ids for gsv_ctx_kernel_time */
#define GSV_K_KECCAK 0
#define GSV_K_ECRECOVER 1
#define GSV_K_CHUNK_LEAF 2
#define GSV_K_CHUNK_LEVEL 3
#define GSV_K_PAIRING 4
#define GSV_K_SENDER_PREP 5
#define GSV_K_BN_PREPARE 6 /* pair decode + G1 curve + G2 subgroup checks */
#define GSV_K_BN_FINAL 7   /* per-check product + final exponentiation */
#define GSV_K_NOTARY 8     /* blob index + per-tx decode/sighash/recover of the notary path */
#define GSV_K_DERIVE_LEAF 9 /* generic DeriveSha leaf encode + hash */
#define GSV_K_HEADER 10    /* collation header hashing + signer comparison */
#define GSV_K_COUNT 12
/* total milliseconds and launch count accumulated for kernel `kid` since the last reset */
int gsv_ctx_kernel_time(gsv_ctx *ctx, int kid, double *total_ms, long *launches);
int gsv_ctx_reset_timing(gsv_ctx *ctx);
/* prepared *_dev shapes currently cached and their device bytes */
int gsv_ctx_prepared_shapes(gsv_ctx *ctx, size_t *count, size_t *device_bytes);
/* Pipeline depth D (1..GSV_MAX_PIPELINE_DEPTH, default 1) of the shapes prepared from now on: each
 * holds D instances of its device memory (tables and workspace), so *_dev calls of ONE shape on up to
 * D different streams run concurrently instead of being ordered after each other (a stream keeps
 * the instance it last used).  A shape prepared at a lower depth is replaced by its next prepare
 * (including the implicit prepare of a binding's *_dev wrapper): the new, deeper shape serves the
 * later calls, and the old one is retired, not freed — its memory stays valid (a HIP graph captured
 * from it can still be replayed) until the shape cache's LRU bound evicts it, after its queued work.
 * Use: validating consecutive batches of equal shape on two streams overlaps one batch's
 * latency-bound tail (trie top, final exponentiation) with the next batch's bulk kernels. */
#define GSV_MAX_PIPELINE_DEPTH 8
int gsv_ctx_set_pipeline_depth(gsv_ctx *ctx, int depth);
/* A stream for a pipelining caller, on a hardware (HSA) queue of its own.  HIP multiplexes ordinary
 * streams over GPU_MAX_HW_QUEUES (4) in-order queues, so two of a caller's streams can share one, and
 * batches issued on them then run one after the other (including every event wait placed on them): a
 * pipeline of D batches needs D streams on D queues.  The stream is created with a CU mask of every CU
 * of the context's device (hipExtStreamCreateWithCUMask: HIP backs such a stream by a dedicated queue);
 * it is ordered with the legacy NULL stream like a hipStreamDefault stream (a BLOCKING stream).
 * The context owns the stream: at most GSV_MAX_STREAMS are live per context (the next create returns
 * GSV_E_INVALID_ARG: more queues oversubscribe the hardware scheduler), gsv_stream_destroy (after the
 * stream's work) releases one and refuses a stream this context did not create, and gsv_ctx_destroy
 * destroys those still live, so a process that exits without destroying its streams tears nothing down
 * in the runtime's static-destructor order. */
#define GSV_MAX_STREAMS 8
int gsv_stream_create(gsv_ctx *ctx, void **stream_out);
int gsv_stream_destroy(gsv_ctx *ctx, void *stream);
/* Live dedicated-queue streams of the context: the caller's (gsv_stream_create) and the prepared
 * shapes' side streams.  A prepared notary shape (and the notary partition) forks its chunk roots onto
 * side streams of its OWN, one per pipeline instance, each a blocking stream on a queue of its own, freed
 * when the shape is evicted or retired.  At most 8 side streams are live per context: a prepare past
 * that takes them from the least recently used shapes holding some, which then run their chunk roots
 * after their transactions on the caller's stream until prepared again (same results; the prepare
 * succeeds; a shape whose side stream has a graph capture open keeps it). */
int gsv_ctx_stream_count(gsv_ctx *ctx, int *user_streams, int *side_streams);

/* ---- Keccak-256 (A10) ----
 * Message i is data[off[i] .. off[i+1]); out32[32*i .. +32) = Keccak256(message i). */
int gsv_keccak256_batch(gsv_ctx *ctx, const uint8_t *data, const uint64_t *off, size_t n,
                        uint8_t *out32);
int gsv_keccak256_batch_dev(gsv_ctx *ctx, const uint8_t *d_data, const uint64_t *d_off, size_t n,
                            uint8_t *d_out32, void *stream);

/* ---- secp256k1 public-key recovery (A5-A9) ----
 * msg32: n x 32 B message hashes; sig65: n x 65 B [R || S || recid].
 * pub65_out: n x 65 B uncompressed keys (0x04 || X || Y), zeroed for failed items.
 * status: GSV_ST_OK / GSV_ST_INVALID_RECID (recid >= 4) / GSV_ST_RECOVER_FAILED.
 * addr20_out (optional, may be NULL): Keccak256(X || Y)[12:32] for OK items. */
int gsv_ecrecover_batch(gsv_ctx *ctx, const uint8_t *msg32, const uint8_t *sig65, size_t n,
                        uint8_t *pub65_out, uint8_t *addr20_out, uint8_t *status);
int gsv_ecrecover_batch_dev(gsv_ctx *ctx, const uint8_t *d_msg32, const uint8_t *d_sig65, size_t n,
                            uint8_t *d_pub65_out, uint8_t *d_addr20_out, uint8_t *d_status,
                            void *stream);

/* ---- the ecrecover precompile (core/vm/contracts.go:78-101) ----
 * Input i = in[off[i] .. off[i+1]) = hash(32) || v(32) || r(32) || s(32), right-padded with zeros to
 * 128 bytes (longer inputs: only the first 128 bytes are read).  ok[i] = 1 and out32[i] =
 * LeftPadBytes(Keccak256(pub[1:])[12:], 32) on success; ok[i] = 0 and out32[i] zero where the
 * reference returns (nil, nil): input[32:63] not all zero, ValidateSignatureValues(v - 27, r, s,
 * homestead = false) false (crypto/crypto.go:181-192), or recovery failing. */
int gsv_ecrecover_precompile_batch(gsv_ctx *ctx, const uint8_t *in, const uint64_t *off, size_t n,
                                   uint8_t *out32, uint8_t *ok);
/* Device-resident form over padded records: d_in128 = n x 128 bytes in HBM. */
int gsv_ecrecover_precompile_batch_dev(gsv_ctx *ctx, const uint8_t *d_in128, size_t n, uint8_t *d_out32,
                                       uint8_t *d_ok, void *stream);

/* ---- recoverPlain (A4): sighash + (R, S, V) -> sender address ----
 * r32/s32: n x 32 B big-endian; v: per-item V already reduced by the signer
 * (27/28 for Homestead/Frontier, tx.V - 2*chainId - 8 for EIP-155) as a uint64 with
 * v_big[i] != 0 meaning "V had more than 8 bits" (-> GSV_ST_INVALID_SIG).
 * homestead: 1 = reject s > n/2 (crypto/crypto.go:188). */
int gsv_sender_batch(gsv_ctx *ctx, const uint8_t *sighash32, const uint8_t *r32, const uint8_t *s32,
                     const uint64_t *v, const uint8_t *v_big, size_t n, int homestead,
                     uint8_t *addr20_out, uint8_t *status);

/* ---- types.Sender over RLP-encoded transactions (A1-A4) ----
 * tx i = rlp[off[i] .. off[i+1]); chain_id big-endian (len 0 = 0). */
int gsv_tx_sender_batch(gsv_ctx *ctx, const uint8_t *rlp, const uint64_t *off, size_t n,
                        const uint8_t *chain_id, size_t chain_id_len, int signer_kind,
                        uint8_t *addr20_out, uint8_t *status);

/* ---- collation chunk root (B1-B5) ----
 * body i = bodies[off[i] .. off[i+1]), each <= 2^20 bytes (else GSV_E_TOO_LARGE).
 * root32_out[i] = DeriveSha(Chunks(body i)); an empty body gives emptyRoot. */
int gsv_chunk_root_batch(gsv_ctx *ctx, const uint8_t *bodies, const uint64_t *off, size_t n,
                         uint8_t *root32_out);
/* Prepares gsv_chunk_root_batch_dev for exactly these host offsets h_off[0..n] (trie plans per body
 * length, device offset table, workspace). */
int gsv_chunk_root_prepare(gsv_ctx *ctx, const uint64_t *h_off, size_t n);
int gsv_chunk_root_batch_dev(gsv_ctx *ctx, const uint8_t *d_bodies, const uint64_t *h_off, size_t n,
                             uint8_t *d_root32_out, void *stream);

/* ---- BN254 pairing check (C1-C6) ----
 * check i = in[off[i] .. off[i+1]) in the precompile encoding (k x 192 B);
 * verdict[i] = GSV_PAIRING_TRUE / FALSE / BAD_INPUT. */
int gsv_bn256_pairing_check_batch(gsv_ctx *ctx, const uint8_t *in, const uint64_t *off, size_t n,
                                  uint8_t *verdict);
/* Device-resident form: d_in in HBM, h_off on the host (n+1 offsets into d_in), d_verdict in HBM.
 * Enqueues on `stream` (NULL = the context stream); returns after the launches are queued.
 * gsv_bn256_pairing_prepare builds the lane tables for exactly these offsets. */
int gsv_bn256_pairing_prepare(gsv_ctx *ctx, const uint64_t *h_off, size_t n);
int gsv_bn256_pairing_check_batch_dev(gsv_ctx *ctx, const uint8_t *d_in, const uint64_t *h_off, size_t n,
                                      uint8_t *d_verdict, void *stream);

/* ---- synthetic signed workload (bench / test data generator; signing is not on the path) ----
 * key_i, msg_i, nonce_i = Keccak256(le64(seed) || le64(i) || "key"/"msg"/"nce"), key and nonce
 * reduced mod n (0 -> 1); sig_i = ECDSA(key_i, msg_i, nonce_i), low-s normalised, recid in sig[64].
 * pub65/addr20 (optional) receive the signer's key and address (the expected recovery result). */
int gsv_synth_sign(gsv_ctx *ctx, uint64_t seed, size_t n, uint8_t *msg32, uint8_t *sig65,
                   uint8_t *pub65, uint8_t *addr20);
int gsv_synth_sign_dev(gsv_ctx *ctx, uint64_t seed, size_t n, uint8_t *d_msg32, uint8_t *d_sig65,
                       uint8_t *d_pub65, uint8_t *d_addr20, void *stream);

/* ---- synthetic pairing workload (bench / test data; configs[4]) ----
 * nchecks x 768 B precompile inputs: check i = e(aP,bQ) e(-bP,aQ) e(cP,dQ) e(-dP,cQ) (true) with
 * a..d = Keccak256(le64(seed) || le64(i) || tag) mod 2^253; i % 8 == 7 perturbs d (false);
 * i % 1024 == 1023 also sets a coordinate to p (bad input).  expect (optional) gets the verdicts. */
int gsv_bn256_synth_checks_dev(gsv_ctx *ctx, uint64_t seed, size_t nchecks, uint8_t *d_out768,
                               uint8_t *d_expect, void *stream);

/* ---- notary validation of whole collations (configs[3]) ----
 * Shard s body = bodies[off[s] .. off[s+1]), at most 2^20 bytes (sharding/collation.go:45).  On the
 * GPU: blob-deserialize (sharding/utils/marshal.go:144-198), decode every blob as an RLP transaction
 * and recover its sender with the signer (GSV_SIGNER_*, chain_id big-endian; the reference notary's
 * chain uses EIP-155), and compute the chunk root (sharding/collation.go:115-119).
 * Per shard: root32_out[32], ntx_out = number of blobs, valid_bitmap_out[(max_txs+7)/8] with bit t
 * (LSB first) set when tx t's sender recovered (GSV_ST_OK).  Optional per tx, laid out
 * [n_shards][max_txs]: senders_out (20 B, zero when not OK) and status_out (GSV_ST_*).
 * A shard with more than max_txs blobs: only the first max_txs are validated; the host entry point
 * returns GSV_E_TOO_LARGE for it (the _dev one reports it through ntx > max_txs).
 * 1 <= max_txs <= GSV_MAX_TXS_PER_SHARD (every blob takes at least one 32-byte chunk of a body of at
 * most 2^20 bytes), else GSV_E_INVALID_ARG; at most 65,535 shards per call. */
#define GSV_MAX_TXS_PER_SHARD 32768
int gsv_notary_validate_shards(gsv_ctx *ctx, const uint8_t *bodies, const uint64_t *off, size_t n_shards,
                               const uint8_t *chain_id, size_t chain_id_len, int signer_kind, uint32_t max_txs,
                               uint8_t *root32_out, uint32_t *ntx_out, uint8_t *valid_bitmap_out,
                               uint8_t *senders_out, uint8_t *status_out);
/* Device-resident form: d_bodies/outputs in HBM, h_off on the host; enqueues on `stream`.
 * gsv_notary_prepare prepares it for exactly (h_off, chain id, signer_kind, max_txs). */
int gsv_notary_prepare(gsv_ctx *ctx, const uint64_t *h_off, size_t n_shards, const uint8_t *chain_id,
                       size_t chain_id_len, int signer_kind, uint32_t max_txs);
int gsv_notary_validate_shards_dev(gsv_ctx *ctx, const uint8_t *d_bodies, const uint64_t *h_off, size_t n_shards,
                                   const uint8_t *chain_id, size_t chain_id_len, int signer_kind,
                                   uint32_t max_txs, uint8_t *d_root32, uint32_t *d_ntx, uint8_t *d_bitmap,
                                   uint8_t *d_senders, uint8_t *d_status, void *stream);

/* ---- synthetic collations (bench / test data; configs[3]) ----
 * Bodies of shards shard0 .. shard0+n_shards-1 (txs_per_shard x 128 B each, contiguous): signed
 * EIP-155 txs (chain id 1) blob-serialized 4 chunks per tx; every 128th tx invalid by construction
 * (high-s / wrong chain id / r not an x-coordinate / recid flipped).  Optional expected status and
 * sender per tx; exp_sender holds the SIGNER's address, which a recid-flipped tx (status OK) does not
 * recover to. */
int gsv_notary_synth_dev(gsv_ctx *ctx, uint64_t seed, uint32_t shard0, size_t n_shards, uint32_t txs_per_shard,
                         uint8_t *d_bodies, uint8_t *d_exp_status, uint8_t *d_exp_sender, void *stream);

/* ---- DeriveSha over any DerivableList (tx root, receipt root) ----
 * List i holds items [list_off[i], list_off[i+1]) of the global item array; item k =
 * vals[voff[k] .. voff[k+1]) is list.GetRlp(j) — the RLP the reference inserts under key rlp(j)
 * (core/types/derive_sha.go:36-38; rlp(tx) for Transactions, rlp(receipt) for Receipts).
 * root32_out[i] = DeriveSha(list i); an empty list gives emptyRoot.  Lists of up to 2^24 items. */
int gsv_derive_sha_batch(gsv_ctx *ctx, const uint8_t *vals, const uint64_t *voff, const uint64_t *list_off,
                         size_t n_lists, uint8_t *root32_out);
/* Device-resident form: d_vals in HBM; voff / list_off on the host (offsets into d_vals / item
 * indices); d_root32_out in HBM; enqueues on `stream` (NULL = the context stream).
 * gsv_derive_sha_prepare prepares it for exactly (voff, list_off). */
int gsv_derive_sha_prepare(gsv_ctx *ctx, const uint64_t *voff, const uint64_t *list_off, size_t n_lists);
int gsv_derive_sha_batch_dev(gsv_ctx *ctx, const uint8_t *d_vals, const uint64_t *voff, const uint64_t *list_off,
                             size_t n_lists, uint8_t *d_root32_out, void *stream);

/* ---- Proof of Custody (sharding/collation.go:124-136) ----
 * poc32_out[i] = DeriveSha(Chunks(salt||b0||salt||b1||...)) over body i = bodies[off[i] .. off[i+1])
 * (salt alone for an empty body).  The salted body may hold up to 2^26 bytes (GSV_E_TOO_LARGE). */
int gsv_collation_poc_batch(gsv_ctx *ctx, const uint8_t *bodies, const uint64_t *off, size_t n,
                            const uint8_t *salt, size_t salt_len, uint8_t *poc32_out);
int gsv_collation_poc_prepare(gsv_ctx *ctx, const uint64_t *h_off, size_t n, const uint8_t *salt, size_t salt_len);
int gsv_collation_poc_batch_dev(gsv_ctx *ctx, const uint8_t *d_bodies, const uint64_t *h_off, size_t n,
                                const uint8_t *salt, size_t salt_len, uint8_t *d_poc32_out, void *stream);

/* ---- collation header hash + proposer signature ----
 * Header i = collationHeaderData{ShardID, ChunkRoot, Period, ProposerAddress, ProposerSignature}
 * (sharding/collation.go:35-43): shard_id32 / period32 are 32-byte big-endian integers,
 * chunk_root32, proposer20, sig65 = [R || S || V] as crypto.Sign returns it (V in {0,1}).
 * nil_flags (optional, NULL = all set): bit 0 = ChunkRoot nil, bit 1 = ProposerAddress nil,
 * bit 2 = ProposerSignature nil/empty (each then RLP-encodes as 0x80, rlp/encode.go:545-581).
 * hash32_out (optional): CollationHeader.Hash() of the header as given (signature included).
 * signer20_out (optional): crypto.Ecrecover(Hash() with ProposerSignature empty — the hash the
 * proposer signs at sharding/proposer/proposer.go:83 — , sig) -> address, zero on failure.
 * status: GSV_ST_OK when the signer equals ProposerAddress, GSV_ST_PROPOSER_MISMATCH when not,
 * else the recovery status (GSV_ST_INVALID_RECID / GSV_ST_RECOVER_FAILED). */
int gsv_collation_header_verify_batch(gsv_ctx *ctx, const uint8_t *shard_id32, const uint8_t *chunk_root32,
                                      const uint8_t *period32, const uint8_t *proposer20, const uint8_t *sig65,
                                      const uint8_t *nil_flags, size_t n, uint8_t *hash32_out,
                                      uint8_t *signer20_out, uint8_t *status);
/* Device-resident form: every array in HBM (d_nil_flags / d_hash32_out / d_signer20_out may be NULL);
 * enqueues on `stream` (NULL = the context stream) and returns.  gsv_collation_header_prepare sizes
 * its workspace for batches of n headers. */
int gsv_collation_header_prepare(gsv_ctx *ctx, size_t n);
int gsv_collation_header_verify_batch_dev(gsv_ctx *ctx, const uint8_t *d_shard_id32, const uint8_t *d_chunk_root32,
                                          const uint8_t *d_period32, const uint8_t *d_proposer20,
                                          const uint8_t *d_sig65, const uint8_t *d_nil_flags, size_t n,
                                          uint8_t *d_hash32_out, uint8_t *d_signer20_out, uint8_t *d_status,
                                          void *stream);

/* ---- multi-GPU: the shard partition and its one collective ----
 * One process per GPU.  Rank r of N owns the contiguous shard block [floor(S r / N), floor(S (r+1) / N))
 * of S shards (the reference runs one shard per node, --shardid, sharding/node/backend.go:245-284;
 * S = 100 in the SMC, sharding/contracts/sharding_manager.sol:56).
 * gsv_comm_unique_id: rank 0 creates the id and hands it to the other ranks (any channel);
 * gsv_comm_init binds an RCCL communicator (xGMI within the node) to the context's device. */
#define GSV_COMM_ID_BYTES 128
int gsv_comm_unique_id(uint8_t id[GSV_COMM_ID_BYTES]);
int gsv_comm_init(gsv_ctx *ctx, const uint8_t id[GSV_COMM_ID_BYTES], int nranks, int rank);
int gsv_comm_info(gsv_ctx *ctx, int *nranks, int *rank);
/* first shard and shard count of `rank`'s block */
int gsv_shard_range(size_t n_shards, int nranks, int rank, size_t *first, size_t *count);
/* Validates this rank's block (bodies/off: its `count` shards, as gsv_notary_validate_shards) and
 * all-gathers the fixed-size per-shard records over RCCL, so every rank returns the records of all
 * n_total_shards shards in shard order: root32_all[32 S], ntx_all[S], valid_bitmap_all[S ceil(max_txs/8)].
 * senders_out / status_out (optional) cover this rank's own shards only ([count][max_txs]).
 * Needs gsv_comm_init (a context without one behaves as N = 1).
 * Collective contract (as for RCCL itself): every rank calls it with the same n_total_shards, chain id,
 * signer and max_txs.  An error in those returns on every rank before the collective.  A failure local
 * to one rank (its bodies, a body > 2^20 bytes, device memory, a HIP error) does NOT skip the
 * collective: the rank all-gathers an empty block carrying its status, and EVERY rank returns the
 * status of the lowest failing rank (the records of the failing ranks' shards are zero). */
int gsv_notary_validate_partition(gsv_ctx *ctx, const uint8_t *bodies, const uint64_t *off, size_t n_total_shards,
                                  const uint8_t *chain_id, size_t chain_id_len, int signer_kind, uint32_t max_txs,
                                  uint8_t *root32_all, uint32_t *ntx_all, uint8_t *valid_bitmap_all,
                                  uint8_t *senders_out, uint8_t *status_out);
/* Device-resident form (the one bench.py times at N > 1): d_bodies holds this rank's block in HBM at the
 * host offsets h_off (count + 1 entries, count from gsv_shard_range); outputs in HBM; enqueues the block's
 * validation, the record pack, one ncclAllGather and the unpack on `stream` and returns.
 * d_rank_status (optional, int32 [nranks]) receives every rank's local status (nonzero: that rank's
 * shards have zero records).  A rank-local failure joins the collective as above and returns its code
 * (the other ranks see it in d_rank_status).  gsv_notary_partition_prepare prepares it for exactly
 * (h_off, n_total_shards, nranks, rank, chain id, signer, max_txs); the context's communicator gives
 * nranks / rank.  Prepared at pipeline depth D (gsv_ctx_set_pipeline_depth), D consecutive calls may be
 * in flight on D streams: their validations overlap, and the library makes each call's all-gather wait
 * for the previous one on the communicator (an event chain; outside a graph capture), so collectives
 * never overlap and every rank issues them in call order. */
int gsv_notary_partition_prepare(gsv_ctx *ctx, const uint64_t *h_off, size_t n_total_shards, int nranks, int rank,
                                 const uint8_t *chain_id, size_t chain_id_len, int signer_kind, uint32_t max_txs);
int gsv_notary_validate_partition_dev(gsv_ctx *ctx, const uint8_t *d_bodies, const uint64_t *h_off,
                                      size_t n_total_shards, const uint8_t *chain_id, size_t chain_id_len,
                                      int signer_kind, uint32_t max_txs, uint8_t *d_root32_all, uint32_t *d_ntx_all,
                                      uint8_t *d_valid_bitmap_all, uint8_t *d_senders, uint8_t *d_status,
                                      int32_t *d_rank_status, void *stream);
/* The same two halves for a caller with its own transport (e.g. records gathered across nodes, one
 * shard per node as the reference runs): pack validates rank `rank`'s block and writes its record block
 * (gsv_partition_block_bytes: header {int32 status, uint32 shards} + ceil(S/N) records of
 * root 32 | ntx 4 | bitmap, padded to 8) into d_block; unpack takes the nranks blocks in rank order and
 * writes the per-shard outputs in shard order (+ d_rank_status).  pack needs
 * gsv_notary_partition_prepare with the same (nranks, rank). */
size_t gsv_partition_block_bytes(size_t n_total_shards, int nranks, uint32_t max_txs);
int gsv_notary_partition_pack_dev(gsv_ctx *ctx, const uint8_t *d_bodies, const uint64_t *h_off, size_t n_total_shards,
                                  int nranks, int rank, const uint8_t *chain_id, size_t chain_id_len, int signer_kind,
                                  uint32_t max_txs, uint8_t *d_block, uint8_t *d_senders, uint8_t *d_status,
                                  void *stream);
int gsv_notary_partition_unpack_dev(gsv_ctx *ctx, const uint8_t *d_blocks, size_t n_total_shards, int nranks,
                                    uint32_t max_txs, uint8_t *d_root32_all, uint32_t *d_ntx_all,
                                    uint8_t *d_valid_bitmap_all, int32_t *d_rank_status, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* GSV_H */

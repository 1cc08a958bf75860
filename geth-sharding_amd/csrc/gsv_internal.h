// Internal declarations shared by the HIP translation units of libgsv.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gsv.h"

namespace gsv {

// ecrecover.hip
hipError_t launch_gtable_init(uint4* gtab, hipStream_t st);
hipError_t launch_ecrecover(const uint8_t* msg32, const uint8_t* sig65, uint32_t n, const uint4* gtab,
                            uint8_t* pub65, uint8_t* addr20, uint8_t* status, hipStream_t st);
hipError_t launch_sender(const uint8_t* sighash32, const uint8_t* r32, const uint8_t* s32,
                         const uint64_t* v, const uint8_t* vbig, uint32_t n, int homestead,
                         const uint4* gtab, uint8_t* addr20, uint8_t* status, hipStream_t st);
hipError_t launch_ecrecover_precompile(const uint8_t* in128, uint32_t n, const uint4* gtab, uint8_t* out32,
                                       uint8_t* ok, hipStream_t st);
hipError_t launch_synth_sign(uint64_t seed, uint32_t n, const uint4* gtab, uint8_t* msg32,
                             uint8_t* sig65, uint8_t* pub65, uint8_t* addr20, hipStream_t st);

// keccak.hip
hipError_t launch_keccak256(const uint8_t* data, const uint64_t* off, uint32_t n, uint8_t* out32,
                            hipStream_t st);

// Launchers call timer_begin(tctx, GSV_HOOK_TAIL) (no launch follows it directly) where the call's
// bulk kernels end and its latency-bound tail begins (trie top, Miller loop + final exponentiation):
// with pipelined shape instances the next call's bulk kernels start there (gsv_api.hip shape_run).
constexpr int GSV_HOOK_TAIL = -1;

// chunk_root.hip
struct TriePlan;  // host-built, device-resident trie shape for one body length N
size_t chunk_root_scratch_bytes(const TriePlan* plan, uint32_t nbodies);
hipError_t launch_chunk_root_plan(const TriePlan* plan, const uint8_t* d_bodies, const uint64_t* d_body_off,
                                  uint32_t nbodies, uint8_t* d_scratch, uint8_t* d_roots, hipStream_t st,
                                  void (*timer_begin)(void*, int), void (*timer_end)(void*, int),
                                  void* tctx);

// generic DeriveSha (any DerivableList) and the Proof-of-Custody salted body
size_t derive_sha_scratch_bytes(const TriePlan* plan, uint32_t nlists);
hipError_t launch_derive_sha_plan(const TriePlan* plan, uint32_t nlists, const uint8_t* d_vals,
                                  const uint64_t* d_voff, uint64_t vend, const uint64_t* d_leaf_base, uint8_t* d_lmsg, uint8_t* d_leafrefs, uint8_t* d_scratch, uint8_t* d_roots,
                                  hipStream_t st, void (*timer_begin)(void*, int), void (*timer_end)(void*, int),
                                  void* tctx);
hipError_t launch_poc_expand(const uint8_t* d_bodies, const uint64_t* d_in_off, const uint64_t* d_out_off,
                             uint32_t nbodies, uint64_t max_out, const uint8_t* d_salt, uint32_t slen, uint8_t* d_out,
                             hipStream_t st);

// collation.hip: header hashes + proposer signature (ecrecover of the unsigned header hash)
size_t header_scratch_bytes(uint32_t n);
hipError_t launch_header_verify(const uint8_t* d_sid32, const uint8_t* d_root32, const uint8_t* d_per32,
                                const uint8_t* d_prop20, const uint8_t* d_sig65, const uint8_t* d_nil, uint32_t n,
                                const uint4* gtab, uint8_t* d_scratch, uint8_t* d_hash32, uint8_t* d_signer20,
                                uint8_t* d_status, hipStream_t st);

// layout flags of launch_bn256_pairing: the final exponentiation on three lanes per check and the Miller
// loop on two lanes per Miller lane (batches below one wave per SIMD), the two-wave lines kernel
// (LINESW2, large batches; else the one-wave k_bn_lines), and the two-wave Miller kernels kept for A/B
// (MILLERW2, MILLERL; off by default)
constexpr int GSV_BN_LAYOUT_FINAL3 = 1, GSV_BN_LAYOUT_MILLER2 = 2, GSV_BN_LAYOUT_MILLERW2 = 8,
              GSV_BN_LAYOUT_LINESW2 = 16, GSV_BN_LAYOUT_MILLERL = 32;
// bn256.hip: pairs in slot-major order (the j-th pairs of all checks contiguous): pair_src[p] = byte
// offset of pair p in d_in.  A check's pairs are split into Miller lanes of <= k pairs each: lane l
// runs the multi-Miller loop over pidx[lane_first[l] .. lane_first[l+1]), check c owns lanes
// [check_lane[c], check_lane[c+1]); cbad[c] != 0 marks a ragged input length (no pairs, verdict
// BAD_INPUT).  Workspaces (F_p elements are 9 words, bn254_fe9.cuh): pstat[npairs],
// lines[91 * 54][npairs], lstat[nlanes], fv[108][nlanes] words, fws[BN_FINAL_SLOTS * 108][nchecks]
// words (the final exponentiation's values that outlive its registers); maxl = the most lanes any
// check has.  final3: the final exponentiation runs on three cooperating lanes per check (small batches)
constexpr int BN_FINAL_SLOTS = 8;
hipError_t launch_bn256_pairing(const uint8_t* d_in, const uint64_t* d_pair_src, uint32_t npairs,
                                const uint32_t* d_lane_first, const uint32_t* d_pidx, uint32_t nlanes,
                                const uint32_t* d_check_lane, const uint8_t* d_cbad, uint32_t nchecks,
                                uint8_t* d_pstat, uint32_t* d_lines, uint8_t* d_lstat, uint32_t* d_fv,
                                uint32_t* d_fws, uint32_t maxl, uint8_t* d_verdict, int layout, hipStream_t st, void (*timer_begin)(void*, int),
                                void (*timer_end)(void*, int), void* tctx);
hipError_t launch_bn256_synth(uint64_t seed, uint32_t nchecks, uint8_t* d_out, uint8_t* d_expect, hipStream_t st);

// notary.hip
size_t blob_rec_bytes();
hipError_t launch_partition_pack(const uint8_t* d_root, const uint32_t* d_ntx, const uint8_t* d_bm, uint32_t n,
                                 uint32_t per, uint32_t R, uint32_t bm, int32_t status, uint8_t* d_block,
                                 hipStream_t st);
hipError_t launch_partition_unpack(const uint8_t* d_all, uint32_t nranks, uint32_t n_total, uint32_t R, uint32_t bm,
                                   size_t B, uint8_t* d_root, uint32_t* d_ntx, uint8_t* d_bm, int32_t* d_rank_status,
                                   hipStream_t st);
hipError_t launch_blob_index(const uint8_t* d_bodies, const uint64_t* d_off, const uint32_t* d_len,
                             uint32_t n_shards, uint32_t max_txs, void* d_blobs, uint32_t* d_ntx, hipStream_t st);
hipError_t launch_notary_tx(const uint8_t* d_bodies, const uint64_t* d_off, const void* d_blobs,
                            const uint32_t* d_ntx, uint32_t n_shards, uint32_t max_txs, const uint8_t* d_cid64,
                            const uint8_t* d_suffix, uint32_t slen, int signer_kind, const uint4* gtab,
                            uint8_t* d_bitmap, uint32_t bm_bytes, uint8_t* d_senders, uint8_t* d_status,
                            hipStream_t st);
hipError_t launch_notary_synth(uint64_t seed, uint32_t shard0, uint32_t n_shards, uint32_t txs_per_shard,
                               const uint4* gtab, uint8_t* d_bodies, uint8_t* d_exp_status, uint8_t* d_exp_sender,
                               hipStream_t st);

// fixed-base comb for u1*G: ceil(256 / COMB_BITS) windows of 2^COMB_BITS affine entries d * 2^(COMB_BITS w) * G.
// 20-bit windows: 13 mixed adds per u1*G over a 1.09 GB table in HBM (one random 80-byte read per
// window, prefetched a window ahead); 16-bit: 16 adds, 80 MiB (Infinity-Cache resident), 1.3 % slower;
// 22-bit: 12 adds, 4 GB, within 0.1 % of 20-bit (profiles/r02/ab_comb.txt).  The table is built once
// per context (k_gtable_base + k_gtable_init).
constexpr int COMB_BITS = 20;
constexpr int COMB_WINDOWS = (256 + COMB_BITS - 1) / COMB_BITS;  // the top window may be partial
static_assert(COMB_BITS >= 4 && COMB_BITS <= 26, "comb window width");
constexpr size_t GTAB_ENTRIES = (size_t)COMB_WINDOWS << COMB_BITS;
constexpr size_t GTAB_ENTRY_BYTES = 80;  // fe9 x[9] y[9] + 2 pad words (recover_dev.cuh gtab_load)
constexpr size_t GTAB_BYTES = GTAB_ENTRIES * GTAB_ENTRY_BYTES;

}  // namespace gsv

// Notary validation of whole collation bodies on gfx950, HBM-resident end to end (configs[3]).
//
// For each shard body (<= 2^20 bytes, sharding/collation.go:45):
//   k_blob_index      blob codec: split the body into blobs (sharding/utils/marshal.go:144-198
//                     Deserialize: 32-byte chunks, indicator & 0x1F = terminal length, 0 = partial
//                     chunk, & 0x80 = skipEvm); one workgroup per shard, chunk-parallel scan.
//   k_notary_tx       one lane per blob = transaction: strict RLP decode of txdata
//                     (core/types/transaction.go:55-70 via rlp/decode.go), types.Sender semantics
//                     (core/types/transaction_signing.go:72-247: EIP-155 chain-id check, V - 2*chainId - 8,
//                     Homestead s <= n/2), the sighash Keccak streamed straight from the blob's chunks
//                     (EIP155Signer.Hash, :155-165), public-key recovery and the address Keccak.
//   chunk root        csrc/chunk_root.hip on the same bodies.
// Outputs per shard: chunk root, tx count, validity bitmap (bit t = tx t's sender recovered), and
// optionally per-tx sender addresses and status codes.
//
// The decode rules are the ones the host path uses (csrc/tx_host.hip tx_prepare), restated for one
// lane: the blob's bytes are read through the chunk map (byte k at chunk k/31, offset 1 + k%31).
#include "opcount.cuh"
#include "recover_dev.cuh"

namespace gsv {

struct BlobRec {
    uint32_t first_chunk;  // chunk index in the shard body
    uint32_t nchunks;
    uint32_t len;          // data bytes = 31 * (nchunks - 1) + terminal length
    uint32_t skip_evm;
};

// ---------------------------------------------------------------- blob index (marshal.go:144-198)
constexpr int BI_THREADS = 1024;
constexpr uint32_t BI_MAX_CHUNKS = (1u << 20) / 32;  // bodies are <= 2^20 bytes (notary_shape refuses more)
constexpr int BI_BATCH = 8;                          // indicator loads in flight per thread

// The indicator bytes (byte 0 of every chunk) are first copied to LDS by coalesced loads — thread t reads
// chunks t, t + 1,024, ..., eight loads in flight — and both passes over a thread's contiguous run of
// chunks read them from there.  r05 read them in those passes straight from HBM, one dependent byte load
// per chunk (two runs of 32 per thread at 1 MiB): 84.6 -> 40.8 us per 100-shard step, notary leg +0.5 %
// (profiles/r06/ab/blob_index_lds.txt).
__global__ __launch_bounds__(BI_THREADS) void k_blob_index(const uint8_t* __restrict__ bodies,
                                                          const uint64_t* __restrict__ body_off,
                                                          const uint32_t* __restrict__ body_len,
                                                          uint32_t max_txs, BlobRec* __restrict__ blobs,
                                                          uint32_t* __restrict__ ntx) {
    __shared__ uint32_t s_cnt[BI_THREADS];
    __shared__ int32_t s_last[BI_THREADS];
    __shared__ uint8_t s_ind[BI_MAX_CHUNKS];
    const uint32_t shard = blockIdx.x, t = threadIdx.x;
    const uint8_t* body = bodies + body_off[shard];
    // a trailing partial chunk is ignored (marshal.go:145)
    const uint32_t chunks = min(body_len[shard] / 32, BI_MAX_CHUNKS);
    for (uint32_t b = t; b < chunks; b += BI_BATCH * BI_THREADS) {
        uint8_t v[BI_BATCH];
#pragma unroll
        for (int k = 0; k < BI_BATCH; k++) {
            uint32_t c = b + k * BI_THREADS;
            v[k] = c < chunks ? body[(size_t)c * 32] : 0;
        }
#pragma unroll
        for (int k = 0; k < BI_BATCH; k++) {
            uint32_t c = b + k * BI_THREADS;
            if (c < chunks) s_ind[c] = v[k];
        }
    }
    __syncthreads();
    const uint32_t per = (chunks + BI_THREADS - 1) / BI_THREADS;
    const uint32_t c0 = t * per, c1 = min(chunks, c0 + per);
    uint32_t cnt = 0;
    int32_t last = -1;
    for (uint32_t c = c0; c < c1; c++)
        if (s_ind[c] & 0x1F) {
            cnt++;
            last = (int32_t)c;
        }
    s_cnt[t] = cnt;
    s_last[t] = last;
    __syncthreads();
    // inclusive scans (Hillis-Steele): counts (+) and last terminal (max)
    for (uint32_t d = 1; d < BI_THREADS; d <<= 1) {
        uint32_t a = t >= d ? s_cnt[t - d] : 0;
        int32_t b = t >= d ? s_last[t - d] : -1;
        __syncthreads();
        s_cnt[t] += a;
        s_last[t] = max(s_last[t], b);
        __syncthreads();
    }
    uint32_t base = s_cnt[t] - cnt;
    int32_t prev = t ? s_last[t - 1] : -1;
    for (uint32_t c = c0; c < c1; c++) {
        uint8_t ind = s_ind[c];
        uint32_t tl = ind & 0x1F;
        if (!tl) continue;
        if (base < max_txs) {
            BlobRec r;
            r.first_chunk = (uint32_t)(prev + 1);
            r.nchunks = c - (uint32_t)prev;
            r.len = 31 * (r.nchunks - 1) + tl;
            r.skip_evm = ind >> 7;
            blobs[(size_t)shard * max_txs + base] = r;
        }
        base++;
        prev = (int32_t)c;
    }
    if (t == BI_THREADS - 1) ntx[shard] = s_cnt[t];
}

// ---------------------------------------------------------------- one transaction per lane
// Measured and not kept (r05): staging each wave's chunk span in its columns of the GLV table's LDS rows
// (free until recover_core builds the table) and decoding from LDS instead of single-byte global loads:
// tx kernels 8.45-8.66 vs 8.60-8.67 ms per configs[3] step (profiles/r05/ab/recover_ab_*.json), within
// noise.  r06: the sighash preimage and R / S (~200 of a tx's byte reads) are gathered as dwords
// (BlobView::dword: two aligned loads per four bytes, issued together), which also freed registers
// (256 -> 247 VGPRs, scratch 784 -> 448 B per lane): tx kernels -1.8 to -2.0 %, 8.80 ns per tx at 128
// shards (profiles/r06/ab/notary_gather.txt).  The RLP headers stay byte reads (each depends on the last);
// reading the integer items' lead bytes together and V as two dwords measured within noise (r06,
// profiles/r06/ab/notary_lead_bytes.txt).
GSV_DI uint32_t ld_g32(uintptr_t a) { return *(const __attribute__((address_space(1))) uint32_t*)a; }

struct BlobView {
    const uint8_t* base;  // first chunk of the blob
    uintptr_t hi;         // the last 4-byte-aligned dword holding a byte of the blob's chunks
    GSV_DI uint8_t at(uint32_t k) const { return base[(size_t)(k / 31) * 32 + 1 + k % 31]; }
    // Data bytes k .. k+3 as one little-endian word (byte k lowest), read through the chunk map as two
    // aligned dwords and realigned; when the chunk ends among them the next chunk's indicator byte is
    // dropped.  Past the blob's data the bytes are unspecified (callers mask them); no dword past the
    // blob's chunks is read, so every read holds a byte of the body.
    GSV_DI uint32_t dword(uint32_t k) const {
        uint32_t c = k / 31u, r = k - 31u * c;
        uintptr_t a = (uintptr_t)base + 32u * (uintptr_t)c + 1u + r;
        uint32_t sh = (uint32_t)a & 3u;
        uintptr_t A = a & ~(uintptr_t)3;
        uint32_t x0 = ld_g32(A <= hi ? A : hi), x1 = ld_g32(A + 4 <= hi ? A + 4 : hi);
        uint32_t v = __builtin_amdgcn_alignbyte(x1, x0, sh);  // bytes a .. a+3
        // r > 27: 31 - r (1..3) data bytes, the indicator, then the next chunk's data
        uint32_t b4 = (x1 >> (8u * sh)) & 0xFFu;              // byte a+4
        uint32_t m = r > 27u ? (1u << (8u * (31u - r))) - 1u : ~0u;
        return (v & m) | (((v >> 8) | (b4 << 24)) & ~m);
    }
};

struct RItem {
    uint32_t off, n;  // payload offset / length within the blob data
    uint32_t start;   // item start (header) offset
    bool list;
};

// one RLP item at [p, p + len) of the blob data; consumed bytes or 0 on error
// (same rules as tx_host.hip rlp_item: canonical single bytes and sizes, rlp/decode.go)
GSV_DI uint32_t rlp_item(const BlobView& b, uint32_t p, uint32_t len, RItem& it) {
    if (len == 0) return 0;
    uint32_t b0 = b.at(p);
    it.start = p;
    if (b0 < 0x80) {
        it.off = p;
        it.n = 1;
        it.list = false;
        return 1;
    }
    if (b0 < 0xb8) {
        uint32_t n = b0 - 0x80;
        if (1 + n > len) return 0;
        if (n == 1 && b.at(p + 1) < 0x80) return 0;
        it.off = p + 1;
        it.n = n;
        it.list = false;
        return 1 + n;
    }
    if (b0 < 0xc0 || b0 >= 0xf8) {  // long string / long list
        bool list = b0 >= 0xf8;
        uint32_t nb = list ? b0 - 0xf7 : b0 - 0xb7;
        if (nb > 8 || 1 + nb > len || b.at(p + 1) == 0) return 0;
        uint64_t n = 0;
        for (uint32_t i = 0; i < nb; i++) n = (n << 8) | b.at(p + 1 + i);
        if (n < 56 || n > (uint64_t)(len - 1 - nb)) return 0;
        it.off = p + 1 + nb;
        it.n = (uint32_t)n;
        it.list = list;
        return 1 + nb + (uint32_t)n;
    }
    uint32_t n = b0 - 0xc0;  // short list
    if (1 + n > len) return 0;
    it.off = p + 1;
    it.n = n;
    it.list = true;
    return 1 + n;
}
GSV_DI bool uint_ok(const BlobView& b, const RItem& it, uint32_t maxlen) {
    return !it.list && it.n <= maxlen && !(it.n > 0 && b.at(it.off) == 0);
}
GSV_DI uint64_t item_u64(const BlobView& b, const RItem& it) {  // it.n <= 8
    uint64_t v = 0;
    for (uint32_t i = 0; i < it.n; i++) v = (v << 8) | b.at(it.off + i);
    return v;
}
GSV_DI uint32_t bitlen_item(const BlobView& b, const RItem& it) {  // canonical: no leading zero
    if (it.n == 0) return 0;
    return 8 * (it.n - 1) + (32 - __builtin_clz((uint32_t)b.at(it.off)));
}

// 32-bit limb w of the big-endian unsigned integer item (it.n <= 32): its bytes n-4-4w .. n-1-4w
GSV_DI uint32_t item_limb(const BlobView& b, const RItem& it, int w) {
    int32_t e = (int32_t)it.n - 4 - 4 * w;  // item position of the limb's most significant byte
    uint32_t d = b.dword(it.off + (uint32_t)(e > 0 ? e : 0));
    d = e < 0 ? (e > -4 ? d << (8u * (uint32_t)(-e)) : 0u) : d;  // positions before the item read as zero
    return __builtin_bswap32(d);
}

// Big-endian 64-byte helpers for V values longer than 8 bytes (rare; mirrors tx_host.hip be_sub)
__device__ __noinline__ uint32_t v_big_path(const uint8_t* blob_base, uint32_t voff, uint32_t vn,
                                            const uint8_t* __restrict__ cid64, uint8_t* vv_low,
                                            uint32_t* vv_big) {
    BlobView b{blob_base, 0};  // at() only
    if (vn > 64) return GSV_ST_INVALID_CHAIN_ID;  // be_sub rejects an > 64
    uint8_t V[64], t[64], chain[64];
    for (int i = 0; i < 64; i++) V[i] = 0;
    for (uint32_t i = 0; i < vn; i++) V[64 - vn + i] = b.at(voff + i);
    int br = 0;  // t = V - 35
    for (int i = 63; i >= 0; i--) {
        int d = (int)V[i] - (i == 63 ? 35 : 0) - br;
        br = d < 0;
        t[i] = (uint8_t)(d + (br ? 256 : 0));
    }
    if (br) return GSV_ST_INVALID_CHAIN_ID;
    int r = 0;  // chain = t / 2
    for (int i = 0; i < 64; i++) {
        int cur = r * 256 + t[i];
        chain[i] = (uint8_t)(cur / 2);
        r = cur % 2;
    }
    for (int i = 0; i < 64; i++)
        if (chain[i] != cid64[i]) return GSV_ST_INVALID_CHAIN_ID;
    // vv = V - 2*cid - 8
    uint8_t two[64];
    int carry = 0;
    for (int i = 63; i >= 0; i--) {
        int d = cid64[i] * 2 + carry;
        two[i] = (uint8_t)d;
        carry = d >> 8;
    }
    br = 0;
    for (int i = 63; i >= 0; i--) {
        int d = (int)V[i] - two[i] - (i == 63 ? 8 : 0) - br;
        br = d < 0;
        t[i] = (uint8_t)(d + (br ? 256 : 0));
    }
    if (br) return GSV_ST_INVALID_SIG;
    uint32_t big = 0;
    for (int i = 0; i < 63; i++) big |= t[i];
    *vv_big = big ? 1u : 0u;
    *vv_low = t[63];
    return GSV_ST_OK;
}

// The sighash preimage as a byte stream: [list header][blob bytes seg_lo .. seg_hi)[suffix]
struct PreStream {
    BlobView b;
    uint64_t hdr;       // header bytes, big-endian in the low hlen (<= 5) bytes
    uint32_t hlen;
    uint32_t seg_lo, seg_len;
    const uint8_t* suffix;  // uniform; zero bytes at [-8, 0) and [slen, slen + 8) (notary_shape layout)
    uint32_t slen;
    GSV_DI uint32_t total() const { return hlen + seg_len + slen; }
    // stream bytes sp .. sp+3 (sp a multiple of 4) as one little-endian word, zero past the stream
    GSV_DI uint32_t dword(uint32_t sp, uint64_t hle) const {
        uint32_t out = sp < 8u ? (uint32_t)(hle >> (8u * sp)) : 0u;  // header (stream bytes < hlen <= 5)
        int32_t e = (int32_t)sp - (int32_t)hlen;                       // segment position of byte 0
        // every read is unconditional (clamped into the blob's chunks / the padded suffix buffer) and
        // masked afterwards, so a block's loads issue back to back
        uint32_t d = b.dword(seg_lo + (uint32_t)(e > 0 ? e : 0));
        d = e < 0 ? (e > -4 ? d << (8u * (uint32_t)(-e)) : 0u) : d;  // the first -e bytes are header
        int32_t vh = (int32_t)seg_len - e;                             // bytes before the segment's end
        d = vh >= 4 ? d : vh > 0 ? d & ((1u << (8u * (uint32_t)vh)) - 1u) : 0u;
        out |= d;
        int32_t f = e - (int32_t)seg_len;  // suffix position of byte 0 (zero-padded buffer)
        int32_t fc = f < -4 ? -4 : f > (int32_t)slen ? (int32_t)slen : f;
        uintptr_t q = (uintptr_t)(suffix + fc);
        uintptr_t Q = q & ~(uintptr_t)3;
        uint32_t x = __builtin_amdgcn_alignbyte(ld_g32(Q + 4), ld_g32(Q), (uint32_t)q & 3u);
        int32_t vs = (int32_t)slen - f;  // bytes before the stream's end (slen is 0 for unprotected txs,
                                         // whose lanes still read the buffer's suffix)
        out |= vs >= 4 ? x : vs > 0 ? x & ((1u << (8u * (uint32_t)vs)) - 1u) : 0u;
        return out;
    }
};

// Keccak-256 over the stream (crypto/sha3/sha3.go:98-157: rate 136, dsbyte 0x01), each rate block
// gathered as 34 little-endian dwords: the blob bytes through BlobView::dword (two aligned loads per four
// bytes, all of a block's loads independent), the header from a register, the suffix from its
// zero-padded buffer.  r05 read the stream a byte at a time (136 dependent byte loads and ~6,300
// instructions per block); a timing run with the preimage reads removed bounded what the stream's reads
// cost at 1.6-2.2 % of k_notary_tx (profiles/r06/ab/notary_fake_sighash.txt).
GSV_DI void keccak_stream(uint64_t a[25], const PreStream& s) {
#pragma unroll
    for (int k = 0; k < 25; k++) a[k] = 0;
    // header bytes in stream order: byte j of hle = stream byte j (j < hlen)
    const uint64_t hle = __builtin_bswap64(s.hdr) >> (8u * (8u - s.hlen));
    uint32_t len = s.total(), pos = 0;
    while (true) {
        uint32_t rem = len - pos;  // bytes left; the final block when rem < 136
        bool final = rem < 136;
#pragma unroll
        for (int w = 0; w < 17; w++) {
            uint64_t v = (uint64_t)s.dword(pos + 8u * w, hle) | ((uint64_t)s.dword(pos + 8u * w + 4u, hle) << 32);
            if (final && (rem >> 3) == (uint32_t)w) v ^= 0x01ull << (8u * (rem & 7u));
            if (final && w == 16) v ^= 0x8000000000000000ULL;
            a[w] ^= v;
        }
        keccakf(a);
        if (final) break;
        pos += 136;
    }
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GSV_ECR_WAVES, GSV_ECR_WAVES))) void k_notary_tx(
    const uint8_t* __restrict__ bodies, const uint64_t* __restrict__ body_off, const BlobRec* __restrict__ blobs,
    const uint32_t* __restrict__ ntx, uint32_t max_txs, const uint8_t* __restrict__ cid64,
    const uint8_t* __restrict__ suffix, uint32_t slen, int signer_kind, const uint4* __restrict__ gtab,
    uint8_t* __restrict__ bitmap, uint32_t bm_bytes, uint8_t* __restrict__ senders,
    uint8_t* __restrict__ status_out) {
    GSV_LTAB_DECL;
    const uint32_t shard = blockIdx.y;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = min(ntx[shard], max_txs);
    bool active = t < n;
    const uint32_t lane = threadIdx.x & 63u;
    if (__ballot(active) == 0) {  // wave-uniform: nothing to validate here
        if ((lane & 7u) == 0 && t < max_txs && (t >> 3) < bm_bytes) bitmap[(size_t)shard * bm_bytes + (t >> 3)] = 0;
        return;
    }
    uint32_t st = GSV_ST_BAD_RLP;
    uint32_t msg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, r[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t vbyte = 0, vbig = 1, homestead = 1;
    if (active) {
        BlobRec br = blobs[(size_t)shard * max_txs + t];
        const uint8_t* bb = bodies + body_off[shard] + (size_t)br.first_chunk * 32;
        BlobView b{bb, ((uintptr_t)bb + 32u * (uintptr_t)br.nchunks - 1u) & ~(uintptr_t)3};
        RItem outer, f[9];
        uint32_t used = rlp_item(b, 0, br.len, outer);
        bool ok = used && used == br.len && outer.list;
        uint32_t p = outer.off, rem = outer.n;
        for (int i = 0; i < 9 && ok; i++) {
            uint32_t u = rlp_item(b, p, rem, f[i]);
            ok = u != 0;
            p += u;
            rem -= u;
        }
        ok = ok && rem == 0;
        ok = ok && uint_ok(b, f[0], 8) && uint_ok(b, f[2], 8) && uint_ok(b, f[1], 256) && uint_ok(b, f[4], 256) &&
             uint_ok(b, f[6], 256) && uint_ok(b, f[7], 256) && uint_ok(b, f[8], 256);
        ok = ok && !f[3].list && (f[3].n == 0 || f[3].n == 20) && !f[5].list;
        if (ok) {
            st = GSV_ST_OK;
            // signer (transaction_signing.go:127-137 EIP155, :182-184 Homestead, :218-220 Frontier)
            bool eip155 = false;
            uint32_t vb = bitlen_item(b, f[6]);
            if (signer_kind == GSV_SIGNER_EIP155) {
                bool prot = true;
                if (vb <= 8) {
                    uint64_t v = item_u64(b, f[6]);
                    prot = (v != 27 && v != 28);
                }
                if (prot) {
                    eip155 = true;
                    if (vb <= 64) {
                        // deriveChainId in uint64 arithmetic (wraps exactly like the reference)
                        uint64_t V = item_u64(b, f[6]);
                        uint64_t c = (V - 35) / 2;
                        bool match = true;
                        for (int i = 0; i < 56; i++) match = match && cid64[i] == 0;
                        uint64_t want = 0;
                        for (int i = 56; i < 64; i++) want = (want << 8) | cid64[i];
                        if (!match || c != want) st = GSV_ST_INVALID_CHAIN_ID;
                        else {
                            // vv = V - 2*chainId - 8 (big-int, non-negative or ErrInvalidSig)
                            unsigned __int128 two = (unsigned __int128)want * 2u + 8u;
                            if ((unsigned __int128)V < two) st = GSV_ST_INVALID_SIG;
                            else {
                                uint64_t vv = (uint64_t)((unsigned __int128)V - two);
                                vbig = vv > 0xFF;
                                vbyte = (uint32_t)(vv & 0xFF);
                            }
                        }
                    } else {
                        uint8_t low;
                        uint32_t big;
                        st = v_big_path(b.base, f[6].off, f[6].n, cid64, &low, &big);
                        vbig = big;
                        vbyte = low;
                    }
                }
            }
            if (!eip155) {
                homestead = signer_kind == GSV_SIGNER_FRONTIER ? 0u : 1u;
                vbig = vb > 8;
                vbyte = (uint32_t)(item_u64(b, f[6]) & 0xFF);
            }
            // sighash = Keccak(rlp([nonce, gasPrice, gas, to, value, data (, chainId, 0, 0)])):
            // the six canonical items are re-encoded byte for byte, so they are one slice of the tx
            PreStream ps;
            ps.b = b;
            ps.seg_lo = f[0].start;
            ps.seg_len = (f[5].off + f[5].n) - f[0].start;
            ps.suffix = suffix;
            ps.slen = eip155 ? slen : 0;
            uint32_t body_len = ps.seg_len + ps.slen;
            if (body_len < 56) {
                ps.hdr = 0xc0 + body_len;
                ps.hlen = 1;
            } else {
                uint32_t nb = body_len < 256 ? 1 : body_len < 65536 ? 2 : body_len < (1u << 24) ? 3 : 4;
                ps.hdr = ((uint64_t)(0xf7 + nb) << (8 * nb)) | body_len;
                ps.hlen = 1 + nb;
            }
            uint64_t a[25];
            keccak_stream(a, ps);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                msg[7 - 2 * j] = __builtin_bswap32((uint32_t)a[j]);
                msg[6 - 2 * j] = __builtin_bswap32((uint32_t)(a[j] >> 32));
            }
            // R, S (recoverPlain, :222-234): > 32 bytes cannot pass ValidateSignatureValues
            if (f[7].n > 32 || f[8].n > 32) vbig = 1;
            else {
                // limb w (little-endian 32-bit) = item bytes n-4-4w .. n-1-4w, byte-reversed; bytes before
                // the item's start are zero
#pragma unroll
                for (int w = 0; w < 8; w++) {
                    r[w] = item_limb(b, f[7], w);
                    s[w] = item_limb(b, f[8], w);
                }
            }
        }
    }
    // recoverPlain + ValidateSignatureValues (crypto/crypto.go:181-192); every lane runs the
    // recovery (dummy operands on inactive / failed lanes) so the wave stays converged
    fe qx, qy;
    uint8_t V = (uint8_t)(vbyte - 27u);
    bool valid = active && st == GSV_ST_OK && !vbig;
    sc rs, ss;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        rs.v[k] = r[k];
        ss.v[k] = s[k];
    }
    valid = valid && !sc_is_zero(rs) && !sc_is_zero(ss) && !(homestead && limbs_lt(HALF_N, s)) &&
            limbs_lt(r, SN) && limbs_lt(s, SN) && (V == 0 || V == 1);
    uint32_t rst = recover_core(qx, qy, msg, r, s, V & 1u, gtab, GSV_LTAB_LANE);
    if (st == GSV_ST_OK && !valid) st = GSV_ST_INVALID_SIG;
    if (st == GSV_ST_OK) st = rst;
    bool good = active && st == GSV_ST_OK;
    uint8_t addr[20];
    store_pub_addr(nullptr, addr, good, qx, qy);
    if (active) {
        if (senders) {
            uint8_t* o = senders + ((size_t)shard * max_txs + t) * 20;
#pragma unroll
            for (int i = 0; i < 20; i++) o[i] = addr[i];
        }
        if (status_out) status_out[(size_t)shard * max_txs + t] = (uint8_t)st;
    }
    // validity bitmap: 8 consecutive lanes (txs) own one byte; blocks start at multiples of 64
    uint64_t m = __ballot(good);
    if ((lane & 7u) == 0 && t < max_txs) {
        uint32_t byte = t >> 3;
        if (byte < bm_bytes) bitmap[(size_t)shard * bm_bytes + byte] = (uint8_t)(m >> lane);
    }
}

// ---------------------------------------------------------------- synthetic collations (bench data)
// Not on the validation path.  Shard `s`, tx j: EIP-155 transaction (chain id 1) signed with
// key_(s,j); RLP-encoded (102-105 bytes) and blob-serialized into exactly 4 chunks at body offset
// 128*j, so 8,192 txs fill a 2^20-byte body (sharding/utils/marshal.go:71-123 layout).
// Every 128th tx (j % 128 == 127) is invalid by construction, class (gi / 128) % 4: high-s
// (ErrInvalidSig), wrong chain id (ErrInvalidChainId), r not an x-coordinate (ErrRecoverFailed), and
// recid flipped: a valid signature of ANOTHER key, so its status is OK and only the recovered sender
// (!= the signer, whose address exp_sender holds) tells it apart.  The CPU
// restatement with the reference's own signer is oracle/ref_shim.c gsvref_notary_synth_body.
// Each tx is 94-124 bytes = 4 chunks.
GSV_DI uint32_t put_be_min(uint8_t* o, uint64_t v) {  // minimal big-endian bytes, returns count
    uint32_t n = 0;
    for (int i = 7; i >= 0; i--) {
        uint8_t b = (uint8_t)(v >> (8 * i));
        if (n || b) o[n++] = b;
    }
    return n;
}
GSV_DI uint32_t put_uint(uint8_t* o, uint64_t v) {  // rlp of a uint64
    uint8_t t[8];
    uint32_t n = put_be_min(t, v);
    if (n == 0) {
        o[0] = 0x80;
        return 1;
    }
    if (n == 1 && t[0] < 0x80) {
        o[0] = t[0];
        return 1;
    }
    o[0] = (uint8_t)(0x80 + n);
    for (uint32_t i = 0; i < n; i++) o[1 + i] = t[i];
    return 1 + n;
}
GSV_DI uint32_t put_u256(uint8_t* o, const uint32_t x[8]) {  // rlp of a 256-bit big int
    uint8_t t[32];
    limbs_to_be(t, x);
    uint32_t z = 0;
    while (z < 32 && t[z] == 0) z++;
    uint32_t n = 32 - z;
    if (n == 1 && t[z] < 0x80) {
        o[0] = t[z];
        return 1;
    }
    o[0] = (uint8_t)(0x80 + n);
    for (uint32_t i = 0; i < n; i++) o[1 + i] = t[z + i];
    return 1 + n;
}

__global__ __launch_bounds__(256) void k_notary_synth(uint64_t seed, uint32_t shard0, uint32_t txs_per_shard,
                                                      uint32_t ntotal, const uint4* __restrict__ gtab,
                                                      uint8_t* __restrict__ bodies, uint8_t* __restrict__ exp_status,
                                                      uint8_t* __restrict__ exp_sender) {
    uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= ntotal) return;
    uint32_t s = shard0 + id / txs_per_shard, j = id % txs_per_shard;
    uint64_t gi = (uint64_t)s * txs_per_shard + j;  // global tx id (independent of the rank split)
    // fields: nonce j mod 128, gasPrice 20 Gwei, gas 21000, to, value = gi, no data
    uint8_t body[112];
    uint32_t w = 0;
    w += put_uint(body + w, j % 128);
    w += put_uint(body + w, 20000000000ull);
    w += put_uint(body + w, 21000);
    uint32_t to[8];
    derive32(to, seed, gi, 0x6f74u);  // "to"
    uint8_t tob[32];
    limbs_to_be(tob, to);
    body[w++] = 0x94;  // 20-byte string
    for (int i = 0; i < 20; i++) body[w++] = tob[12 + i];
    w += put_uint(body + w, gi);
    body[w++] = 0x80;  // empty data
    uint32_t fields_len = w;
    // sighash preimage = rlp([6 fields, chainId=1, 0, 0])
    uint8_t pre[120];
    uint32_t plen = 0;
    uint32_t blen = fields_len + 3;
    if (blen < 56) pre[plen++] = (uint8_t)(0xc0 + blen);
    else {
        pre[plen++] = 0xf8;
        pre[plen++] = (uint8_t)blen;
    }
    for (uint32_t i = 0; i < fields_len; i++) pre[plen++] = body[i];
    pre[plen++] = 0x01;
    pre[plen++] = 0x80;
    pre[plen++] = 0x80;
    uint64_t a[25];
#pragma unroll
    for (int k = 0; k < 25; k++) a[k] = 0;
    for (uint32_t q = 0; q < plen; q++) {  // plen < 136: one block
        uint32_t wi = q >> 3;
        uint64_t v = (uint64_t)pre[q] << (8 * (q & 7));
#pragma unroll
        for (int k = 0; k < 17; k++)
            if ((uint32_t)k == wi) a[k] ^= v;
    }
#pragma unroll
    for (int k = 0; k < 17; k++) {
        if ((uint32_t)k == (plen >> 3)) a[k] ^= (uint64_t)0x01 << (8 * (plen & 7));
    }
    a[16] ^= 0x8000000000000000ULL;
    keccakf(a);
    uint32_t msg[8];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        msg[7 - 2 * q] = __builtin_bswap32((uint32_t)a[q]);
        msg[6 - 2 * q] = __builtin_bswap32((uint32_t)(a[q] >> 32));
    }
    sc d, k;
    derive32(d.v, seed, gi, 0x79656bu);  // "key"
    derive32(k.v, seed, gi, 0x65636eu);  // "nce"
    uint32_t r[8], sg[8], recid;
    fe px, py;
    ecdsa_sign(r, sg, recid, px, py, d, k, msg, gtab);
    uint32_t chain = 1, st = GSV_ST_OK;
    if (j % 128 == 127) {
        uint32_t cls = (uint32_t)((gi / 128) % 4);
        if (cls == 0) {  // high-s: n - s (still a valid signature; Homestead rule rejects it)
            sc t, u;
#pragma unroll
            for (int i = 0; i < 8; i++) t.v[i] = sg[i];
            sc_neg(u, t);
#pragma unroll
            for (int i = 0; i < 8; i++) sg[i] = u.v[i];
            recid ^= 1u;
            st = GSV_ST_INVALID_SIG;
        } else if (cls == 1) {  // signed for chain 1 but V encodes chain 5
            chain = 5;
            st = GSV_ST_INVALID_CHAIN_ID;
        } else if (cls == 2) {  // r = 2^255 + 2: r^3 + 7 is a non-residue mod p, so no point has x = r (< n)
#pragma unroll
            for (int i = 0; i < 8; i++) r[i] = i == 0 ? 2u : i == 7 ? 0x80000000u : 0u;
            st = GSV_ST_RECOVER_FAILED;
        } else {  // recid flipped: R' = -R recovers r^-1 (s R' - m G) != the signer's key
            recid ^= 1u;
        }
    }
    w += put_uint(body + w, (recid & 1u) + 35 + 2 * chain);
    w += put_u256(body + w, r);
    w += put_u256(body + w, sg);
    // tx = list header + payload
    uint8_t tx[124];
    uint32_t tlen = 0;
    tx[tlen++] = 0xf8;
    tx[tlen++] = (uint8_t)w;
    for (uint32_t i = 0; i < w; i++) tx[tlen++] = body[i];
    // blob serialisation: 4 chunks of [indicator, 31 bytes]
    uint8_t* out = bodies + ((size_t)(s - shard0) * txs_per_shard + j) * 128;
    for (uint32_t c = 0; c < 4; c++) {
        uint32_t lo = c * 31, hi = lo + 31;
        uint32_t tl = c == 3 ? tlen - 93 : 0;
        out[c * 32] = (uint8_t)tl;
        for (uint32_t q = lo; q < hi; q++) out[c * 32 + 1 + (q - lo)] = q < tlen ? tx[q] : 0;
    }
    if (exp_status) exp_status[id] = (uint8_t)st;
    if (exp_sender) store_pub_addr(nullptr, exp_sender + (size_t)id * 20, st == GSV_ST_OK, px, py);
}

// ---------------------------------------------------------------- shard-partition records
// One rank's block (gsv.h gsv_partition_block_bytes): header {int32 status, uint32 shards} then
// `per` records of R bytes: root 32 | ntx 4 | bitmap bm | zero pad (the layout of gsv/shards.py).
// A rank whose local validation failed packs its status and zero records, so every rank always
// reaches the all-gather (sharding/node/backend.go:245-284 partition; one record set per shard).
__global__ __launch_bounds__(256) void k_partition_pack(const uint8_t* __restrict__ root, const uint32_t* __restrict__ ntx,
                                                        const uint8_t* __restrict__ bitmap, uint32_t n, uint32_t per,
                                                        uint32_t R, uint32_t bm, int32_t status,
                                                        uint8_t* __restrict__ block) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        *(int32_t*)block = status;
        *(uint32_t*)(block + 4) = status ? 0u : n;
    }
    if (i >= per * R) return;
    const uint32_t k = i / R, o = i % R;
    uint8_t v = 0;
    if (k < n && status == 0) {
        if (o < 32) v = root[(size_t)k * 32 + o];
        else if (o < 36) v = (uint8_t)(ntx[k] >> (8 * (o - 32)));
        else if (o < 36 + bm) v = bitmap[(size_t)k * bm + (o - 36)];
    }
    block[8 + i] = v;
}

// all = nranks blocks of B bytes (rank order) -> per-shard outputs in shard order + rank statuses
__global__ __launch_bounds__(256) void k_partition_unpack(const uint8_t* __restrict__ all, uint32_t nranks,
                                                          uint32_t n_total, uint32_t R, uint32_t bm, size_t B,
                                                          uint8_t* __restrict__ root, uint32_t* __restrict__ ntx,
                                                          uint8_t* __restrict__ bitmap, int32_t* __restrict__ rank_status) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (rank_status && i < nranks) rank_status[i] = *(const int32_t*)(all + (size_t)i * B);
    if (i >= n_total * R) return;
    const uint32_t s = i / R, o = i % R;
    // owner rank q: first(q) = floor(S q / N) <= s < first(q + 1)
    uint32_t q = (uint32_t)(((uint64_t)s * nranks + nranks - 1) / n_total);
    while (q > 0 && (uint64_t)n_total * q / nranks > s) q--;
    while (q + 1 < nranks && (uint64_t)n_total * (q + 1) / nranks <= s) q++;
    const uint32_t k = s - (uint32_t)((uint64_t)n_total * q / nranks);
    const uint8_t* rec = all + (size_t)q * B + 8 + (size_t)k * R;
    if (o < 32) root[(size_t)s * 32 + o] = rec[o];
    else if (o == 32) ntx[s] = *(const uint32_t*)(rec + 32);
    else if (o >= 36 && o < 36 + bm) bitmap[(size_t)s * bm + (o - 36)] = rec[o];
}

hipError_t launch_partition_pack(const uint8_t* d_root, const uint32_t* d_ntx, const uint8_t* d_bm, uint32_t n,
                                 uint32_t per, uint32_t R, uint32_t bm, int32_t status, uint8_t* d_block,
                                 hipStream_t st) {
    uint32_t total = per * R;
    hipLaunchKernelGGL(k_partition_pack, dim3((total + 255) / 256 + 1), dim3(256), 0, st, d_root, d_ntx, d_bm, n, per,
                       R, bm, status, d_block);
    return hipGetLastError();
}

hipError_t launch_partition_unpack(const uint8_t* d_all, uint32_t nranks, uint32_t n_total, uint32_t R, uint32_t bm,
                                   size_t B, uint8_t* d_root, uint32_t* d_ntx, uint8_t* d_bm, int32_t* d_rank_status,
                                   hipStream_t st) {
    uint32_t total = std::max(n_total * R, nranks);
    if (!total) return hipSuccess;
    hipLaunchKernelGGL(k_partition_unpack, dim3((total + 255) / 256), dim3(256), 0, st, d_all, nranks, n_total, R, bm,
                       B, d_root, d_ntx, d_bm, d_rank_status);
    return hipGetLastError();
}

// ---------------------------------------------------------------- launchers
hipError_t launch_blob_index(const uint8_t* d_bodies, const uint64_t* d_off, const uint32_t* d_len,
                             uint32_t n_shards, uint32_t max_txs, void* d_blobs, uint32_t* d_ntx, hipStream_t st) {
    if (!n_shards) return hipSuccess;
    hipLaunchKernelGGL(k_blob_index, dim3(n_shards), dim3(BI_THREADS), 0, st, d_bodies, d_off, d_len, max_txs,
                       (BlobRec*)d_blobs, d_ntx);
    return hipGetLastError();
}

hipError_t launch_notary_tx(const uint8_t* d_bodies, const uint64_t* d_off, const void* d_blobs,
                            const uint32_t* d_ntx, uint32_t n_shards, uint32_t max_txs, const uint8_t* d_cid64,
                            const uint8_t* d_suffix, uint32_t slen, int signer_kind, const uint4* gtab,
                            uint8_t* d_bitmap, uint32_t bm_bytes, uint8_t* d_senders, uint8_t* d_status,
                            hipStream_t st) {
    if (!n_shards || !max_txs) return hipSuccess;
    dim3 grid((max_txs + 255) / 256, n_shards);
    hipLaunchKernelGGL(k_notary_tx, grid, dim3(256), 0, st, d_bodies, d_off, (const BlobRec*)d_blobs, d_ntx,
                       max_txs, d_cid64, d_suffix, slen, signer_kind, gtab, d_bitmap, bm_bytes, d_senders,
                       d_status);
    return hipGetLastError();
}

hipError_t launch_notary_synth(uint64_t seed, uint32_t shard0, uint32_t n_shards, uint32_t txs_per_shard,
                               const uint4* gtab, uint8_t* d_bodies, uint8_t* d_exp_status, uint8_t* d_exp_sender,
                               hipStream_t st) {
    uint32_t ntotal = n_shards * txs_per_shard;
    if (!ntotal) return hipSuccess;
    hipLaunchKernelGGL(k_notary_synth, dim3((ntotal + 255) / 256), dim3(256), 0, st, seed, shard0, txs_per_shard,
                       ntotal, gtab, d_bodies, d_exp_status, d_exp_sender);
    return hipGetLastError();
}

size_t blob_rec_bytes() { return sizeof(BlobRec); }

}  // namespace gsv

GSV_OPCOUNT_READER(notary)

// Collation header hashing and proposer-signature verification on gfx950.
//
// Restated semantics:
//   sharding/collation.go:35-43    collationHeaderData{ShardID *big.Int, ChunkRoot *common.Hash,
//                                  Period *big.Int, ProposerAddress *common.Address, ProposerSignature []byte}
//   sharding/collation.go:66-71    Hash() = Keccak256(rlp(data))
//   rlp/encode.go:429-440          big.Int: 0 -> 0x80, else the minimal big-endian bytes as a string
//   rlp/encode.go:545-581          nil *common.Hash / *common.Address -> 0x80; nil *big.Int -> 0 -> 0x80
//   sharding/proposer/proposer.go:77-89  the proposer signs Hash() of the header whose signature
//                                  field is still nil, then AddSig()s the [R||S||V] signature
//   crypto/signature_cgo.go:31     Ecrecover(hash, sig) -> pubkey; address = Keccak256(pub[1:])[12:]
//
// Pipeline per batch: k_header_hash (one lane per header: each RLP preimage assembled in LDS, two
// Keccak-256s) -> k_ecrecover (the shared recovery kernel, address output) -> k_header_compare
// (signer vs ProposerAddress).
#include <hip/hip_runtime.h>

#include "opcount.cuh"
#include "gsv_internal.h"
#include "keccak_dev.cuh"

namespace gsv {

constexpr int HDR_WORDS = 24;  // 8-byte words per preimage (max RLP 2 + 33 + 33 + 33 + 21 + 67 = 189 bytes)
constexpr int HDR_LANES = 256;

// A lane's preimage in LDS, word-interleaved across the block's lanes ([word][lane] of 8 bytes) so the
// Keccak absorption reads conflict-free; bytes are written at their final offsets (the payload length
// is known before any byte is written), so nothing is moved and nothing goes to HBM.
struct HdrWriter {
    uint8_t* lds;  // the block's [HDR_WORDS][HDR_LANES] u64 array
    uint32_t lane, n;
    GSV_DI void put(uint8_t b) {
        lds[((n >> 3) * HDR_LANES + lane) * 8 + (n & 7u)] = b;
        n++;
    }
    // rlp string of a 32-byte big-endian integer (writeBigInt: minimal bytes, 0 -> 0x80)
    GSV_DI void bigint32(const uint8_t* v) {
        int z = 0;
        while (z < 32 && v[z] == 0) z++;
        int L = 32 - z;
        if (L == 1 && v[31] < 0x80) {
            put(v[31]);
            return;
        }
        put((uint8_t)(0x80 + L));
        for (int k = z; k < 32; k++) put(v[k]);
    }
    GSV_DI void bytes(const uint8_t* v, int L) {  // L in {20, 32, 65}: never a single byte
        if (L < 56) {
            put((uint8_t)(0x80 + L));
        } else {
            put(0xb8);
            put((uint8_t)L);
        }
        for (int k = 0; k < L; k++) put(v[k]);
    }
};
GSV_DI uint32_t bigint32_len(const uint8_t* v) {
    int z = 0;
    while (z < 32 && v[z] == 0) z++;
    int L = 32 - z;
    return (L == 1 && v[31] < 0x80) ? 1u : 1u + (uint32_t)L;
}

// writes the RLP list of the header (with or without the signature); returns its length
GSV_DI uint32_t header_rlp(HdrWriter& w, const uint8_t* sid, const uint8_t* root, const uint8_t* per,
                           const uint8_t* prop, const uint8_t* sig, uint8_t nilf, bool with_sig) {
    bool sig_empty = !with_sig || (nilf & 4);
    uint32_t pl = bigint32_len(sid) + ((nilf & 1) ? 1u : 33u) + bigint32_len(per) + ((nilf & 2) ? 1u : 21u) +
                  (sig_empty ? 1u : 67u);
    w.n = 0;
    if (pl < 56) {
        w.put((uint8_t)(0xc0 + pl));
    } else {
        w.put(0xf8);
        w.put((uint8_t)pl);
    }
    w.bigint32(sid);
    if (nilf & 1) w.put(0x80);
    else w.bytes(root, 32);
    w.bigint32(per);
    if (nilf & 2) w.put(0x80);
    else w.bytes(prop, 20);
    if (sig_empty) w.put(0x80);
    else w.bytes(sig, 65);
    return w.n;
}

// Keccak-256 of the lane's len-byte LDS preimage (bytes past len are ignored), digest to out
GSV_DI void keccak_lds(uint8_t* out, const uint64_t* lds, uint32_t lane, uint32_t len) {
    uint64_t a[25];
#pragma unroll
    for (int k = 0; k < 25; k++) a[k] = 0;
    uint32_t w0 = 0;
    if (len >= 136) {  // len <= 189: at most one full block
#pragma unroll
        for (int k = 0; k < 17; k++) a[k] ^= lds[k * HDR_LANES + lane];
        keccakf(a);
        w0 = 17;
        len -= 136;
    }
#pragma unroll
    for (int k = 0; k < 17; k++) {
        int32_t avail = (int32_t)len - 8 * k;
        uint64_t w = 0;
        if (avail > 0 && w0 + k < (uint32_t)HDR_WORDS) w = lds[(w0 + k) * HDR_LANES + lane];
        if (avail < 8) w = avail > 0 ? w & ((1ull << (8 * avail)) - 1ull) : 0ull;
        if ((uint32_t)(len >> 3) == (uint32_t)k) w ^= 0x01ull << (8 * (len & 7u));
        if (k == 16) w ^= 0x8000000000000000ULL;
        a[k] ^= w;
    }
    keccakf_digest(a);
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int b = 0; b < 8; b++) out[8 * k + b] = (uint8_t)(a[k] >> (8 * b));
}

__global__ __launch_bounds__(HDR_LANES) void k_header_hash(const uint8_t* __restrict__ sid32,
                                                           const uint8_t* __restrict__ root32,
                                                           const uint8_t* __restrict__ per32,
                                                           const uint8_t* __restrict__ prop20,
                                                           const uint8_t* __restrict__ sig65,
                                                           const uint8_t* __restrict__ nil_flags, uint32_t n,
                                                           uint8_t* unsigned32, uint8_t* hash32) {
    __shared__ uint64_t pre[HDR_WORDS * HDR_LANES];
    uint32_t i = blockIdx.x * HDR_LANES + threadIdx.x;
    if (i >= n) return;
    uint8_t nf = nil_flags ? nil_flags[i] : 0;
    const uint8_t* sid = sid32 + (size_t)i * 32;
    const uint8_t* root = root32 + (size_t)i * 32;
    const uint8_t* per = per32 + (size_t)i * 32;
    const uint8_t* prop = prop20 + (size_t)i * 20;
    const uint8_t* sig = sig65 + (size_t)i * 65;
    HdrWriter w{(uint8_t*)pre, threadIdx.x, 0};
    uint32_t l0 = header_rlp(w, sid, root, per, prop, sig, nf, false);
    keccak_lds(unsigned32 + (size_t)i * 32, pre, threadIdx.x, l0);
    if (hash32) {  // the lane's own words only: no barrier needed between its two preimages
        uint32_t l1 = header_rlp(w, sid, root, per, prop, sig, nf, true);
        keccak_lds(hash32 + (size_t)i * 32, pre, threadIdx.x, l1);
    }
}

__global__ __launch_bounds__(256) void k_header_compare(const uint8_t* __restrict__ rec20,
                                                        const uint8_t* __restrict__ prop20,
                                                        const uint8_t* __restrict__ nil_flags, uint32_t n,
                                                        uint8_t* status, uint8_t* signer20) {
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint8_t st = status[i];
    const uint8_t* r = rec20 + (size_t)i * 20;
    const uint8_t* p = prop20 + (size_t)i * 20;
    bool eq = st == GSV_ST_OK && !(nil_flags && (nil_flags[i] & 2));
    for (int k = 0; k < 20; k++) eq = eq && r[k] == p[k];
    if (st == GSV_ST_OK && !eq) status[i] = GSV_ST_PROPOSER_MISMATCH;
    if (signer20)
        for (int k = 0; k < 20; k++) signer20[(size_t)i * 20 + k] = st == GSV_ST_OK ? r[k] : 0;
}

size_t header_scratch_bytes(uint32_t n) { return (size_t)n * (32 + 20); }

// d_scratch: header_scratch_bytes(n), 8-byte aligned
hipError_t launch_header_verify(const uint8_t* d_sid32, const uint8_t* d_root32, const uint8_t* d_per32,
                                const uint8_t* d_prop20, const uint8_t* d_sig65, const uint8_t* d_nil, uint32_t n,
                                const uint4* gtab, uint8_t* d_scratch, uint8_t* d_hash32, uint8_t* d_signer20,
                                uint8_t* d_status, hipStream_t st) {
    if (n == 0) return hipSuccess;
    uint8_t* uh = d_scratch;
    uint8_t* rec = uh + (size_t)n * 32;
    dim3 g((n + HDR_LANES - 1) / HDR_LANES);
    hipLaunchKernelGGL(k_header_hash, g, dim3(HDR_LANES), 0, st, d_sid32, d_root32, d_per32, d_prop20, d_sig65, d_nil,
                       n, uh, d_hash32);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = launch_ecrecover(uh, d_sig65, n, gtab, nullptr, rec, d_status, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_header_compare, g, dim3(256), 0, st, rec, d_prop20, d_nil, n, d_status, d_signer20);
    return hipGetLastError();
}

}  // namespace gsv

GSV_OPCOUNT_READER(collation)

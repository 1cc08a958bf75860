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
// Pipeline per batch: k_header_hash (one lane per header: both RLP preimages in a per-lane HBM
// buffer, two Keccak-256s) -> k_ecrecover (the shared recovery kernel, address output) ->
// k_header_compare (signer vs ProposerAddress).
#include <hip/hip_runtime.h>

#include "opcount.cuh"
#include "gsv_internal.h"
#include "keccak_dev.cuh"

namespace gsv {

constexpr int HDR_PRE = 256;  // bytes per preimage buffer (max RLP 3 + 33 + 33 + 33 + 21 + 67 = 190)

// Keccak-256 of len bytes at 8-byte aligned p (bytes past len are ignored), digest bytes to out
GSV_DI void keccak_aligned(uint8_t* out, const uint8_t* p, uint32_t len) {
    uint64_t a[25];
#pragma unroll
    for (int k = 0; k < 25; k++) a[k] = 0;
    const uint64_t* q = (const uint64_t*)p;
    while (len >= 136) {
#pragma unroll
        for (int k = 0; k < 17; k++) a[k] ^= q[k];
        keccakf(a);
        q += 17;
        len -= 136;
    }
#pragma unroll
    for (int k = 0; k < 17; k++) {
        int32_t avail = (int32_t)len - 8 * k;
        uint64_t w = 0;
        if (avail >= 8) w = q[k];
        else if (avail > 0) w = q[k] & ((1ull << (8 * avail)) - 1ull);
        if ((uint32_t)(len >> 3) == (uint32_t)k) w ^= 0x01ull << (8 * (len & 7u));
        if (k == 16) w ^= 0x8000000000000000ULL;
        a[k] ^= w;
    }
    keccakf(a);
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int b = 0; b < 8; b++) out[8 * k + b] = (uint8_t)(a[k] >> (8 * b));
}

struct HdrWriter {
    uint8_t* p;
    uint32_t n;
    GSV_DI void put(uint8_t b) { p[n++] = b; }
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

// writes the RLP list of the header at m (with or without the signature); returns its length
GSV_DI uint32_t header_rlp(uint8_t* m, const uint8_t* sid, const uint8_t* root, const uint8_t* per,
                           const uint8_t* prop, const uint8_t* sig, uint8_t nilf, bool with_sig) {
    HdrWriter w{m + 3, 0};  // payload first, list header prepended below
    w.bigint32(sid);
    if (nilf & 1) w.put(0x80);
    else w.bytes(root, 32);
    w.bigint32(per);
    if (nilf & 2) w.put(0x80);
    else w.bytes(prop, 20);
    if (!with_sig || (nilf & 4)) w.put(0x80);
    else w.bytes(sig, 65);
    uint32_t pl = w.n;
    // move the payload so the list header (1 or 2 bytes) directly precedes it at m[0]
    uint32_t hl = pl < 56 ? 1u : 2u;
    uint8_t* dst = m + hl;
    for (uint32_t k = 0; k < pl; k++) dst[k] = m[3 + k];
    if (hl == 1) {
        m[0] = (uint8_t)(0xc0 + pl);
    } else {
        m[0] = 0xf8;
        m[1] = (uint8_t)pl;
    }
    return hl + pl;
}

__global__ __launch_bounds__(256) void k_header_hash(const uint8_t* __restrict__ sid32,
                                                     const uint8_t* __restrict__ root32,
                                                     const uint8_t* __restrict__ per32,
                                                     const uint8_t* __restrict__ prop20,
                                                     const uint8_t* __restrict__ sig65,
                                                     const uint8_t* __restrict__ nil_flags, uint32_t n,
                                                     uint8_t* pre, uint8_t* unsigned32, uint8_t* hash32) {
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint8_t nf = nil_flags ? nil_flags[i] : 0;
    const uint8_t* sid = sid32 + (size_t)i * 32;
    const uint8_t* root = root32 + (size_t)i * 32;
    const uint8_t* per = per32 + (size_t)i * 32;
    const uint8_t* prop = prop20 + (size_t)i * 20;
    const uint8_t* sig = sig65 + (size_t)i * 65;
    uint8_t* m = pre + (size_t)i * 2 * HDR_PRE;
    uint32_t l0 = header_rlp(m, sid, root, per, prop, sig, nf, false);
    keccak_aligned(unsigned32 + (size_t)i * 32, m, l0);
    if (hash32) {
        uint8_t* m1 = m + HDR_PRE;
        uint32_t l1 = header_rlp(m1, sid, root, per, prop, sig, nf, true);
        keccak_aligned(hash32 + (size_t)i * 32, m1, l1);
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

size_t header_scratch_bytes(uint32_t n) { return (size_t)n * (2 * HDR_PRE + 32 + 20); }

// d_scratch: header_scratch_bytes(n), 8-byte aligned
hipError_t launch_header_verify(const uint8_t* d_sid32, const uint8_t* d_root32, const uint8_t* d_per32,
                                const uint8_t* d_prop20, const uint8_t* d_sig65, const uint8_t* d_nil, uint32_t n,
                                const uint4* gtab, uint8_t* d_scratch, uint8_t* d_hash32, uint8_t* d_signer20,
                                uint8_t* d_status, hipStream_t st) {
    if (n == 0) return hipSuccess;
    uint8_t* pre = d_scratch;
    uint8_t* uh = pre + (size_t)n * 2 * HDR_PRE;
    uint8_t* rec = uh + (size_t)n * 32;
    dim3 g((n + 255) / 256);
    hipLaunchKernelGGL(k_header_hash, g, dim3(256), 0, st, d_sid32, d_root32, d_per32, d_prop20, d_sig65, d_nil, n,
                       pre, uh, d_hash32);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = launch_ecrecover(uh, d_sig65, n, gtab, nullptr, rec, d_status, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_header_compare, g, dim3(256), 0, st, rec, d_prop20, d_nil, n, d_status, d_signer20);
    return hipGetLastError();
}

}  // namespace gsv

GSV_OPCOUNT_READER(collation)

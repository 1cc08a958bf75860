// Batched Keccak-256 over variable-length messages (crypto.Keccak256, crypto/crypto.go:43-49;
// sponge crypto/sha3/sha3.go:98-157, rate 136, dsbyte 0x01).  One message per lane; each lane
// absorbs its own 136-byte blocks.  Used for transaction sighashes (RLP preimages) and as the
// generic batch hash entry point.
#include "gsv_internal.h"
#include "keccak_dev.cuh"

namespace gsv {

// Absorb one rate block (17 little-endian 64-bit words) of the message at p, `avail` bytes of it
// valid (136: a full block), into the state; `fin`: the last block, which also takes the padding
// (0x01 after the message, 0x80 in byte 135: sha3.go:98-157, dsbyte 0x01).  Messages sit at any byte
// offset (RLP strings packed back to back), so the block is read as up to 35 aligned dwords from p
// rounded down to 4 and realigned with v_alignbyte_b32 — 35 loads instead of 136 byte loads.  Each
// word is XORed into the state as soon as it is assembled (no 17-word block held in registers).
GSV_DI void absorb_words(uint64_t a[25], const uint32_t d[35], uint32_t sh, uint32_t avail, bool fin) {
#pragma unroll
    for (int k = 0; k < 17; k++) {
        uint32_t lo = __builtin_amdgcn_alignbyte(d[2 * k + 1], d[2 * k], sh);
        uint32_t hi = __builtin_amdgcn_alignbyte(d[2 * k + 2], d[2 * k + 1], sh);
        uint64_t v = (uint64_t)lo | ((uint64_t)hi << 32);
        int32_t valid = (int32_t)avail - 8 * k;
        if (valid < 8) v = valid <= 0 ? 0 : v & ((1ull << (8 * valid)) - 1);
        if (fin && (avail >> 3) == (uint32_t)k) v ^= 0x01ull << (8 * (avail & 7u));
        if (fin && k == 16) v ^= 0x8000000000000000ULL;
        a[k] ^= v;
    }
}
// From HBM: a dword is read only if it holds a valid byte (so never past the page of the last one).
GSV_DI void absorb_block(uint64_t a[25], const uint8_t* p, uint32_t avail, bool fin) {
    uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t* q = (const uint32_t*)(p - sh);  // pointer arithmetic: stays a global (not flat) load
    uint32_t need = sh + avail;  // bytes from q
    uint32_t d[35];
#pragma unroll
    for (int j = 0; j < 35; j++) d[j] = (4u * j < need) ? q[j] : 0u;
    absorb_words(a, d, sh, avail, fin);
}
// From the workgroup's LDS copy of its messages (k_keccak256 staging): s32 is the copy itself and b the
// block's byte offset in it (no integer round trip of the pointer, which would make the reads flat
// loads); the dwords are read unconditionally (the copy is padded past its end).
GSV_DI void absorb_block_lds(uint64_t a[25], const uint32_t* s32, uint32_t b, uint32_t avail, bool fin) {
    const uint32_t* q = s32 + (b >> 2);
    uint32_t d[35];
#pragma unroll
    for (int j = 0; j < 35; j++) d[j] = q[j];
    absorb_words(a, d, b & 3u, avail, fin);
}

// 1: a workgroup whose 256 messages span at most KECCAK_STAGE_BYTES copies that span into LDS with
// coalesced 16-byte loads first, and each lane then assembles its blocks from LDS.  Read straight from
// HBM, every dword load of a wave touches 64 different cache lines (one per lane's message): the
// memory pipeline, not the permutation, set the kernel's pace (0.29 of the instruction
// floor, 55 % of wave time issue-stalled).  0: always the direct loads (A/B).  Larger spans (long
// messages) take the direct path.
#ifndef GSV_KECCAK_STAGE
#define GSV_KECCAK_STAGE 1
#endif
constexpr uint32_t KECCAK_STAGE_BYTES = 36 * 1024;  // + pad: four workgroups per CU (160 KB LDS)
constexpr uint32_t KECCAK_STAGE_PAD = 160;          // load_block_lds reads up to 143 bytes past a block start

// Messages are taken in block-count order within each workgroup (keccak_dev.cuh wg_bucket_order:
// 3.21 -> 3.58 G hashes/s on tx-sized messages, profiles/r02/ab_keccak_bucket.txt).
__global__ __launch_bounds__(256) void k_keccak256(const uint8_t* __restrict__ data,
                                                   const uint64_t* __restrict__ off, uint32_t n,
                                                   uint8_t* __restrict__ out32) {
    uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x;
#if GSV_KECCAK_STAGE
    __shared__ uint4 s_msg[(KECCAK_STAGE_BYTES + KECCAK_STAGE_PAD) / 16];
    // the workgroup's messages [first, last) are one contiguous byte span (message i = [off[i], off[i+1]))
    const uint32_t first = blockIdx.x * blockDim.x, last = min(n, first + blockDim.x);
    const uint8_t* lo16 = data + off[first] - ((uintptr_t)(data + off[first]) & 15u);
    const uint64_t span = (uint64_t)(data + off[last] - lo16 + 15) & ~(uint64_t)15;
    // a 16-byte aligned chunk holding a message byte never crosses a page, so the rounding is safe
    const bool staged = span <= KECCAK_STAGE_BYTES;  // uniform across the workgroup
    if (staged) {
        const uint32_t nv = (uint32_t)(span >> 4);
        const uint4* src = (const uint4*)lo16;
        for (uint32_t v = threadIdx.x; v < nv; v += blockDim.x) s_msg[v] = src[v];
    }
#endif
    uint32_t i = wg_bucket_order(i0, i0 < n, i0 < n ? (off[i0 + 1] - off[i0]) / 136u : 0);  // barriers
    if (i >= n) return;
    const uint8_t* p = data + off[i];
    uint64_t len = off[i + 1] - off[i];
    uint64_t a[25];
#pragma unroll
    for (int k = 0; k < 25; k++) a[k] = 0;
#if GSV_KECCAK_STAGE
    const uint32_t* s32 = (const uint32_t*)s_msg;
    uint32_t ps = (uint32_t)(p - lo16);  // the message's byte offset in the LDS copy (when staged)
#else
    const bool staged = false;
    const uint32_t* s32 = nullptr;
    uint32_t ps = 0;
#endif
    // one block loop for both sources (a uniform branch per block) and the final padded block: one
    // copy of the permutation
    while (true) {
        const bool fin = len < 136;
        const uint32_t avail = fin ? (uint32_t)len : 136u;
        if (staged) absorb_block_lds(a, s32, ps, avail, fin);
        else absorb_block(a, p, avail, fin);
        keccakf(a);
        if (fin) break;
        p += 136;
        ps += 136;
        len -= 136;
    }
    uint8_t* o = out32 + (size_t)i * 32;
    if (((uintptr_t)out32 & 15u) == 0) {  // uniform: two 16-byte stores
        uint4* o4 = (uint4*)o;
        o4[0] = make_uint4((uint32_t)a[0], (uint32_t)(a[0] >> 32), (uint32_t)a[1], (uint32_t)(a[1] >> 32));
        o4[1] = make_uint4((uint32_t)a[2], (uint32_t)(a[2] >> 32), (uint32_t)a[3], (uint32_t)(a[3] >> 32));
        return;
    }
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int b = 0; b < 8; b++) o[8 * k + b] = (uint8_t)(a[k] >> (8 * b));
}

hipError_t launch_keccak256(const uint8_t* data, const uint64_t* off, uint32_t n, uint8_t* out32,
                            hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_keccak256, dim3((n + 255) / 256), dim3(256), 0, st, data, off, n, out32);
    return hipGetLastError();
}

}  // namespace gsv

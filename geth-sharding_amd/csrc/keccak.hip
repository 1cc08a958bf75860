// Batched Keccak-256 over variable-length messages (crypto.Keccak256, crypto/crypto.go:43-49;
// sponge crypto/sha3/sha3.go:98-157, rate 136, dsbyte 0x01).  One message per lane; each lane
// absorbs its own 136-byte blocks.  Used for transaction sighashes (RLP preimages) and as the
// generic batch hash entry point.
#include <stdlib.h>
#include "gsv_internal.h"
#include "keccak_dev.cuh"

namespace gsv {

// One rate block (17 little-endian 64-bit words) of the message at p, `avail` bytes of it valid
// (>= 136: a full block).  Messages sit at any byte offset (RLP strings packed back to back), so the
// block is read as up to 35 aligned dwords from p rounded down to 4 and realigned with
// v_alignbyte_b32 — 35 loads instead of 136 byte loads.  A dword is read only if it holds a valid
// byte (so never past the page of the last one); bytes past `avail` are masked to zero.
GSV_DI void load_block(uint64_t w[17], const uint8_t* p, uint32_t avail) {
    const uint32_t* q = (const uint32_t*)((uintptr_t)p & ~(uintptr_t)3);
    uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
    uint32_t take = avail < 136u ? avail : 136u;
    uint32_t need = sh + take;  // bytes from q
    uint32_t d[35];
#pragma unroll
    for (int j = 0; j < 35; j++) d[j] = (4u * j < need) ? q[j] : 0u;
#pragma unroll
    for (int k = 0; k < 17; k++) {
        uint32_t lo = __builtin_amdgcn_alignbyte(d[2 * k + 1], d[2 * k], sh);
        uint32_t hi = __builtin_amdgcn_alignbyte(d[2 * k + 2], d[2 * k + 1], sh);
        uint64_t v = (uint64_t)lo | ((uint64_t)hi << 32);
        int32_t valid = (int32_t)take - 8 * k;
        if (valid < 8) v = valid <= 0 ? 0 : v & ((1ull << (8 * valid)) - 1);
        w[k] = v;
    }
}

// The final (partial) block, `avail` < 136 bytes.  load_block's per-dword predicates differ between
// lanes here, so each of its 35 loads becomes a branch of its own around a one-dword load.  When at
// least 16 bytes of the batch follow the message (every message but the last few), each 16-byte group
// that holds a valid byte is read whole instead — one dwordx4; the bytes read past the message belong to
// the next ones and are masked to zero as in load_block.  Half the kernel's vector-memory instructions
// and ~40 % less TA busy time; 5.53-5.57 -> 5.65-5.70 G permutations/s at 400 k tx-sized messages and
// 6.86-7.04 -> 7.10-7.21 at 1.6 M (r06, profiles/r06/ab/keccak_tail_loader.txt).  106 registers (four
// waves per SIMD) measured equal to 96 forced with 24 B of spill (five waves).
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

GSV_DI void load_block_tail(uint64_t w[17], const uint8_t* p, uint32_t avail) {
    const uint32_t* q = (const uint32_t*)((uintptr_t)p & ~(uintptr_t)3);
    uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
    uint32_t need = sh + avail;  // bytes from q, <= 138
    uint32_t d[36];
#pragma unroll
    for (int g = 0; g < 9; g++) {
        u32x4a4 v = {0u, 0u, 0u, 0u};
        if (16u * g < need) v = *(const u32x4a4*)(q + 4 * g);
        d[4 * g] = v.x;
        d[4 * g + 1] = v.y;
        d[4 * g + 2] = v.z;
        d[4 * g + 3] = v.w;
    }
#pragma unroll
    for (int k = 0; k < 17; k++) {
        uint32_t lo = __builtin_amdgcn_alignbyte(d[2 * k + 1], d[2 * k], sh);
        uint32_t hi = __builtin_amdgcn_alignbyte(d[2 * k + 2], d[2 * k + 1], sh);
        uint64_t v = (uint64_t)lo | ((uint64_t)hi << 32);
        int32_t valid = (int32_t)avail - 8 * k;
        if (valid < 8) v = valid <= 0 ? 0 : v & ((1ull << (8 * valid)) - 1);
        w[k] = v;
    }
}

// digest = the first 32 bytes of the state; out32 16-byte aligned (uniform): two dwordx4 stores
GSV_DI void store_hash(uint8_t* __restrict__ out32, uint32_t i, const uint64_t a[25]) {
    uint8_t* o = out32 + (size_t)i * 32;
    if (((uintptr_t)out32 & 15u) == 0) {
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

// Messages are taken in block-count order within each workgroup (keccak_dev.cuh wg_bucket_order:
// 3.21 -> 3.58 G hashes/s on tx-sized messages, profiles/r02/ab_keccak_bucket.txt).
// Measured and not kept (r05): staging each workgroup's contiguous message span in LDS with coalesced
// 16-byte loads and assembling the blocks from LDS — 5.04 vs 5.25 G permutations/s at 400 k messages,
// 6.54 / 6.60 vs 6.53 / 6.58 at 1.6 / 6.4 M (profiles/r05/ab/keccak_scale_*.txt): the per-lane dword
// loads were not what limits the kernel; the permutation's instruction mix is.
// Measured and not kept (r06): two messages per lane with each next rate block staged in LDS by
// global_load_lds_dwordx4 while the current one is permuted (121 registers, 36 KB of LDS per workgroup)
// — 4.94-4.95 vs 5.69 G permutations/s at 400 k messages, 6.43-6.48 vs 7.13-7.21 at 1.6 M
// (profiles/r06/ab/keccak_staged_lds.txt): hiding a lane's own load latency does not pay either.
__global__ __launch_bounds__(256) void k_keccak256(const uint8_t* __restrict__ data,
                                                   const uint64_t* __restrict__ off, uint32_t n,
                                                   uint8_t* __restrict__ out32) {
    uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t i = wg_bucket_order(i0, i0 < n, i0 < n ? (off[i0 + 1] - off[i0]) / 136u : 0);
    if (i >= n) return;
    const uint8_t* p = data + off[i];
    uint64_t len = off[i + 1] - off[i];
    uint64_t a[25], w[17];
#pragma unroll
    for (int k = 0; k < 25; k++) a[k] = 0;
    while (len >= 136) {
        load_block(w, p, 136);
#pragma unroll
        for (int k = 0; k < 17; k++) a[k] ^= w[k];
        keccakf(a);
        p += 136;
        len -= 136;
    }
    // final block: remaining len bytes, then 0x01 at len, 0x80 at 135
    uint32_t rem = (uint32_t)len;
    // one loader per wave: the whole-group reads unless a lane's message ends within 16 bytes of the batch
    if (__builtin_amdgcn_ballot_w64(off[n] - off[i + 1] < 16) == 0)
        load_block_tail(w, p, rem);
    else
        load_block(w, p, rem);
#pragma unroll
    for (int k = 0; k < 17; k++) {
        uint64_t x = w[k];
        if ((uint32_t)(rem >> 3) == (uint32_t)k) x ^= 0x01ull << (8 * (rem & 7u));
        if (k == 16) x ^= 0x8000000000000000ULL;
        a[k] ^= x;
    }
    keccakf_digest(a);
    store_hash(out32, i, a);
}

hipError_t launch_keccak256(const uint8_t* data, const uint64_t* off, uint32_t n, uint8_t* out32,
                            hipStream_t st) {
    if (n == 0) return hipSuccess;
    // 256-thread workgroups: 0.096-0.098 ms per 400 k tx strings against 0.100 (128) and 0.109 (64)
    // (r05, profiles/r05/ab/keccak_block_depth)
    hipLaunchKernelGGL(k_keccak256, dim3((n + 255) / 256), dim3(256), 0, st, data, off, n, out32);
    return hipGetLastError();
}

}  // namespace gsv

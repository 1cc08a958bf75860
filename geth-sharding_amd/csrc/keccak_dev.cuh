// Keccak-f[1600] and Keccak-256 (pre-FIPS padding 0x01 ... 0x80, rate 136) on gfx950 VALU.
// One message per lane; the 25 x 64-bit state lives in 50 VGPRs.  64-bit rotates lower to
// v_alignbit_b32 pairs, theta's 5-way XORs and chi's a ^ (~b & c) to v_bitop3_b32.
// Restates crypto/sha3/keccakf.go:39 (permutation), :10 (round constants) and
// crypto/sha3/sha3.go:98-157 + hashes.go:16 (sponge, rate 136, dsbyte 0x01).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GSV_DI __device__ __forceinline__

namespace gsv {

__device__ constexpr uint64_t KECCAK_RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};

template <int R>
GSV_DI uint64_t rotl64(uint64_t x) {
    if constexpr (R == 0) return x;
    else return (x << R) | (x >> (64 - R));
}

GSV_DI uint64_t xor5(uint64_t a, uint64_t b, uint64_t c, uint64_t d, uint64_t e) {
    return a ^ b ^ c ^ d ^ e;
}

// One full permutation, rounds fully unrolled in-place (lane index x + 5y).
GSV_DI void keccakf(uint64_t a[25]) {
#pragma unroll 1
    for (int round = 0; round < 24; round++) {
        uint64_t c0 = xor5(a[0], a[5], a[10], a[15], a[20]);
        uint64_t c1 = xor5(a[1], a[6], a[11], a[16], a[21]);
        uint64_t c2 = xor5(a[2], a[7], a[12], a[17], a[22]);
        uint64_t c3 = xor5(a[3], a[8], a[13], a[18], a[23]);
        uint64_t c4 = xor5(a[4], a[9], a[14], a[19], a[24]);
        uint64_t d0 = c4 ^ rotl64<1>(c1);
        uint64_t d1 = c0 ^ rotl64<1>(c2);
        uint64_t d2 = c1 ^ rotl64<1>(c3);
        uint64_t d3 = c2 ^ rotl64<1>(c4);
        uint64_t d4 = c3 ^ rotl64<1>(c0);
        // theta + rho + pi: b[y][2x+3y] = rot(a[x][y] ^ d[x], r[x][y])
        uint64_t b0 = a[0] ^ d0;
        uint64_t b10 = rotl64<1>(a[1] ^ d1);
        uint64_t b20 = rotl64<62>(a[2] ^ d2);
        uint64_t b5 = rotl64<28>(a[3] ^ d3);
        uint64_t b15 = rotl64<27>(a[4] ^ d4);
        uint64_t b16 = rotl64<36>(a[5] ^ d0);
        uint64_t b1 = rotl64<44>(a[6] ^ d1);
        uint64_t b11 = rotl64<6>(a[7] ^ d2);
        uint64_t b21 = rotl64<55>(a[8] ^ d3);
        uint64_t b6 = rotl64<20>(a[9] ^ d4);
        uint64_t b7 = rotl64<3>(a[10] ^ d0);
        uint64_t b17 = rotl64<10>(a[11] ^ d1);
        uint64_t b2 = rotl64<43>(a[12] ^ d2);
        uint64_t b12 = rotl64<25>(a[13] ^ d3);
        uint64_t b22 = rotl64<39>(a[14] ^ d4);
        uint64_t b23 = rotl64<41>(a[15] ^ d0);
        uint64_t b8 = rotl64<45>(a[16] ^ d1);
        uint64_t b18 = rotl64<15>(a[17] ^ d2);
        uint64_t b3 = rotl64<21>(a[18] ^ d3);
        uint64_t b13 = rotl64<8>(a[19] ^ d4);
        uint64_t b14 = rotl64<18>(a[20] ^ d0);
        uint64_t b24 = rotl64<2>(a[21] ^ d1);
        uint64_t b9 = rotl64<61>(a[22] ^ d2);
        uint64_t b19 = rotl64<56>(a[23] ^ d3);
        uint64_t b4 = rotl64<14>(a[24] ^ d4);
        // chi
        a[0] = b0 ^ (~b1 & b2);
        a[1] = b1 ^ (~b2 & b3);
        a[2] = b2 ^ (~b3 & b4);
        a[3] = b3 ^ (~b4 & b0);
        a[4] = b4 ^ (~b0 & b1);
        a[5] = b5 ^ (~b6 & b7);
        a[6] = b6 ^ (~b7 & b8);
        a[7] = b7 ^ (~b8 & b9);
        a[8] = b8 ^ (~b9 & b5);
        a[9] = b9 ^ (~b5 & b6);
        a[10] = b10 ^ (~b11 & b12);
        a[11] = b11 ^ (~b12 & b13);
        a[12] = b12 ^ (~b13 & b14);
        a[13] = b13 ^ (~b14 & b10);
        a[14] = b14 ^ (~b10 & b11);
        a[15] = b15 ^ (~b16 & b17);
        a[16] = b16 ^ (~b17 & b18);
        a[17] = b17 ^ (~b18 & b19);
        a[18] = b18 ^ (~b19 & b15);
        a[19] = b19 ^ (~b15 & b16);
        a[20] = b20 ^ (~b21 & b22);
        a[21] = b21 ^ (~b22 & b23);
        a[22] = b22 ^ (~b23 & b24);
        a[23] = b23 ^ (~b24 & b20);
        a[24] = b24 ^ (~b20 & b21);
        // iota
        a[0] ^= KECCAK_RC[round];
    }
}

// Keccak-256 of the 64-byte string X||Y given as big-endian 256-bit limb arrays
// (address derivation: crypto.Keccak256(pub[1:]) in core/types/transaction_signing.go:244).
GSV_DI void keccak256_xy(uint32_t h[8], const uint32_t x[8], const uint32_t y[8]) {
    uint64_t a[25];
#pragma unroll
    for (int i = 0; i < 25; i++) a[i] = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        a[j] = (uint64_t)__builtin_bswap32(x[7 - 2 * j]) |
               ((uint64_t)__builtin_bswap32(x[6 - 2 * j]) << 32);
        a[4 + j] = (uint64_t)__builtin_bswap32(y[7 - 2 * j]) |
                   ((uint64_t)__builtin_bswap32(y[6 - 2 * j]) << 32);
    }
    a[8] = 0x01;
    a[16] = 0x8000000000000000ULL;
    keccakf(a);
#pragma unroll
    for (int j = 0; j < 4; j++) {
        h[2 * j] = (uint32_t)a[j];
        h[2 * j + 1] = (uint32_t)(a[j] >> 32);
    }
}

}  // namespace gsv

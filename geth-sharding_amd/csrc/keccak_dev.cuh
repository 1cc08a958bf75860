// Keccak-f[1600] and Keccak-256 (pre-FIPS padding 0x01 ... 0x80, rate 136) on gfx950 VALU.
// One message per lane; the 25 x 64-bit state lives in 50 VGPRs as 32-bit halves.  64-bit rotates
// are explicit v_alignbit_b32 pairs, theta's 5-way XORs and chi's a ^ (~b & c) explicit v_bitop3_b32
// (the compiler's own lowering of the uint64 form was 64-bit shifts + v_bfi + v_xor: ~20% more issue).
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

// v_bitop3_b32 truth tables (index = S0<<2 | S1<<1 | S2): S0^S1^S2, and chi's S0 ^ (~S1 & S2)
#ifndef GSV_BITOP3_CHI
#define GSV_BITOP3_CHI 0xD2
#endif
constexpr uint32_t BITOP3_XOR3 = 0x96;

GSV_DI uint32_t kxor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, BITOP3_XOR3); }
GSV_DI uint32_t kchi(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, GSV_BITOP3_CHI); }

// 64-bit rotate-left by R of (hi:lo): two v_alignbit_b32 (rotates by 0/32 are register renames)
template <int R>
GSV_DI void krot(uint32_t& olo, uint32_t& ohi, uint32_t lo, uint32_t hi) {
    if constexpr (R == 0) {
        olo = lo;
        ohi = hi;
    } else if constexpr (R < 32) {
        ohi = __builtin_amdgcn_alignbit(hi, lo, 32 - R);
        olo = __builtin_amdgcn_alignbit(lo, hi, 32 - R);
    } else if constexpr (R == 32) {
        olo = hi;
        ohi = lo;
    } else {
        ohi = __builtin_amdgcn_alignbit(lo, hi, 64 - R);
        olo = __builtin_amdgcn_alignbit(hi, lo, 64 - R);
    }
}

// rho offsets r[x + 5y] (crypto/sha3/keccakf.go) and pi destinations: b[y + 5((2x + 3y) mod 5)]
__device__ constexpr int KECCAK_RHO[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                                           25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};

template <int I>
GSV_DI void theta_rho_pi(uint32_t bl[25], uint32_t bh[25], const uint32_t al[25], const uint32_t ah[25],
                         const uint32_t dl[5], const uint32_t dh[5]) {
    constexpr int x = I % 5, y = I / 5;
    constexpr int dst = y + 5 * ((2 * x + 3 * y) % 5);
    krot<KECCAK_RHO[I]>(bl[dst], bh[dst], al[I] ^ dl[x], ah[I] ^ dh[x]);
    if constexpr (I + 1 < 25) theta_rho_pi<I + 1>(bl, bh, al, ah, dl, dh);
}

// One full permutation over the state split into 32-bit halves (lane index x + 5y).  Per round:
// theta's column parities as 20 three-way v_bitop3, rho as 48 v_alignbit, chi as 50 v_bitop3.
GSV_DI void keccakf_split(uint32_t al[25], uint32_t ah[25]) {
#pragma unroll 1
    for (int round = 0; round < 24; round++) {
        uint32_t cl[5], ch[5], dl[5], dh[5];
#pragma unroll
        for (int x = 0; x < 5; x++) {
            cl[x] = kxor3(kxor3(al[x], al[x + 5], al[x + 10]), al[x + 15], al[x + 20]);
            ch[x] = kxor3(kxor3(ah[x], ah[x + 5], ah[x + 10]), ah[x + 15], ah[x + 20]);
        }
#pragma unroll
        for (int x = 0; x < 5; x++) {
            uint32_t rl, rh;
            krot<1>(rl, rh, cl[(x + 1) % 5], ch[(x + 1) % 5]);
            dl[x] = cl[(x + 4) % 5] ^ rl;
            dh[x] = ch[(x + 4) % 5] ^ rh;
        }
        uint32_t bl[25], bh[25];
        theta_rho_pi<0>(bl, bh, al, ah, dl, dh);
#pragma unroll
        for (int y = 0; y < 25; y += 5) {
#pragma unroll
            for (int x = 0; x < 5; x++) {
                al[y + x] = kchi(bl[y + x], bl[y + (x + 1) % 5], bl[y + (x + 2) % 5]);
                ah[y + x] = kchi(bh[y + x], bh[y + (x + 1) % 5], bh[y + (x + 2) % 5]);
            }
        }
        al[0] ^= (uint32_t)KECCAK_RC[round];
        ah[0] ^= (uint32_t)(KECCAK_RC[round] >> 32);
    }
}

GSV_DI void keccakf(uint64_t a[25]) {
    uint32_t al[25], ah[25];
#pragma unroll
    for (int k = 0; k < 25; k++) {
        al[k] = (uint32_t)a[k];
        ah[k] = (uint32_t)(a[k] >> 32);
    }
    keccakf_split(al, ah);
#pragma unroll
    for (int k = 0; k < 25; k++) a[k] = (uint64_t)al[k] | ((uint64_t)ah[k] << 32);
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

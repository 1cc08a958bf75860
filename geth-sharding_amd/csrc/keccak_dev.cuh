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
constexpr uint32_t BITOP3_XOR3 = 0x96;
constexpr uint32_t BITOP3_CHI = 0xD2;

GSV_DI uint32_t kxor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, BITOP3_XOR3); }
GSV_DI uint32_t kchi(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, BITOP3_CHI); }

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

// theta's D[x] = C[x - 1] ^ rot(C[x + 1], 1) is applied as ONE three-input XOR per word,
// A ^ C[x - 1] ^ rot(C[x + 1], 1) (r05): 50 v_bitop3 instead of 10 v_xor for D plus 50 v_xor (through
// r04), i.e. the round at the 180-instruction floor (profiles/r05/ab/keccak_theta3.txt).
template <int I>
GSV_DI void theta_rho_pi(uint32_t bl[25], uint32_t bh[25], const uint32_t al[25], const uint32_t ah[25],
                         const uint32_t dl[5], const uint32_t dh[5], const uint32_t cl[5], const uint32_t ch[5]) {
    constexpr int x = I % 5, y = I / 5;
    constexpr int dst = y + 5 * ((2 * x + 3 * y) % 5);
    // dl / dh hold rot(C[x + 1], 1)
    krot<KECCAK_RHO[I]>(bl[dst], bh[dst], kxor3(al[I], cl[(x + 4) % 5], dl[x]), kxor3(ah[I], ch[(x + 4) % 5], dh[x]));
    if constexpr (I + 1 < 25) theta_rho_pi<I + 1>(bl, bh, al, ah, dl, dh, cl, ch);
}

// One full permutation over the state split into 32-bit halves (lane index x + 5y).  Per round:
// theta's column parities as 20 three-way v_bitop3, rot(C, 1) as 10 v_alignbit, theta's application as
// 50 three-way v_bitop3, rho as 48 v_alignbit, chi as 50 v_bitop3, iota 2.  One round per loop
// iteration (two measured equal, r05: profiles/r05/ab/chunk_levels5_unroll2.txt).
template <int ROUNDS>
GSV_DI void keccakf_rounds(uint32_t al[25], uint32_t ah[25]) {
#pragma unroll 1
    for (int round = 0; round < ROUNDS; round++) {
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
            dl[x] = rl;
            dh[x] = rh;
        }
        uint32_t bl[25], bh[25];
        theta_rho_pi<0>(bl, bh, al, ah, dl, dh, cl, ch);
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

GSV_DI void keccakf_split(uint32_t al[25], uint32_t ah[25]) { keccakf_rounds<24>(al, ah); }

// The permutation whose output is only read as a Keccak-256 digest (state words 0..3, the sponge's
// last squeeze): 23 full rounds, then the last round computes just those four words.  Row 0 after
// pi is rho(theta(A)) of the diagonal x = y (B[k] = rot(A'[6k], r[6k])), and chi of words 0..3 reads
// B[0..4]; theta still needs all five column parities.  20 + 10 + 10 + 8 + 8 + 2 = 58 instructions
// instead of 180: 4,198 per digest permutation instead of 4,320 (-2.8 %).  Words 4..24 of the
// state are left unspecified.
GSV_DI void keccakf_split_digest(uint32_t al[25], uint32_t ah[25]) {
    keccakf_rounds<23>(al, ah);
    uint32_t cl[5], ch[5], dl[5], dh[5];
#pragma unroll
    for (int x = 0; x < 5; x++) {
        cl[x] = kxor3(kxor3(al[x], al[x + 5], al[x + 10]), al[x + 15], al[x + 20]);
        ch[x] = kxor3(kxor3(ah[x], ah[x + 5], ah[x + 10]), ah[x + 15], ah[x + 20]);
    }
#pragma unroll
    for (int x = 0; x < 5; x++) krot<1>(dl[x], dh[x], cl[(x + 1) % 5], ch[(x + 1) % 5]);
    uint32_t bl[5], bh[5];
    krot<KECCAK_RHO[0]>(bl[0], bh[0], kxor3(al[0], cl[4], dl[0]), kxor3(ah[0], ch[4], dh[0]));
    krot<KECCAK_RHO[6]>(bl[1], bh[1], kxor3(al[6], cl[0], dl[1]), kxor3(ah[6], ch[0], dh[1]));
    krot<KECCAK_RHO[12]>(bl[2], bh[2], kxor3(al[12], cl[1], dl[2]), kxor3(ah[12], ch[1], dh[2]));
    krot<KECCAK_RHO[18]>(bl[3], bh[3], kxor3(al[18], cl[2], dl[3]), kxor3(ah[18], ch[2], dh[3]));
    krot<KECCAK_RHO[24]>(bl[4], bh[4], kxor3(al[24], cl[3], dl[4]), kxor3(ah[24], ch[3], dh[4]));
#pragma unroll
    for (int x = 0; x < 4; x++) {
        al[x] = kchi(bl[x], bl[(x + 1) % 5], bl[(x + 2) % 5]);
        ah[x] = kchi(bh[x], bh[(x + 1) % 5], bh[(x + 2) % 5]);
    }
    al[0] ^= (uint32_t)KECCAK_RC[23];
    ah[0] ^= (uint32_t)(KECCAK_RC[23] >> 32);
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

// keccakf for a digest: only a[0..3] are defined afterwards
GSV_DI void keccakf_digest(uint64_t a[25]) {
    uint32_t al[25], ah[25];
#pragma unroll
    for (int k = 0; k < 25; k++) {
        al[k] = (uint32_t)a[k];
        ah[k] = (uint32_t)(a[k] >> 32);
    }
    keccakf_split_digest(al, ah);
#pragma unroll
    for (int k = 0; k < 4; k++) a[k] = (uint64_t)al[k] | ((uint64_t)ah[k] << 32);
}

// ---------------------------------------------------------------- group-cooperative Keccak-f
// Keccak-f[1600] by a 32-lane group (a half wave): lane i < 25 holds A[i] (x = i % 5, y = i / 5)
// as (lo, hi); lanes 25..31 mirror lane 24 and are never read.  Column parities, the theta D
// term, pi and chi's neighbours move between lanes with ds_bpermute (__shfl): 18 per round, so
// one permutation's latency is ~3x shorter than one lane's 190-instruction rounds.  For the
// latency-bound top of a trie, where one node at a time is on the critical path.
__device__ constexpr int KECCAK_RHO_C[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                                             25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};
GSV_DI uint32_t gshfl(uint32_t v, int src) { return (uint32_t)__shfl((int)v, src, 32); }

GSV_DI void keccakf_coop(uint32_t& lo, uint32_t& hi, int i) {
    const int x = i % 5, y = i / 5;
    const int c1 = (i + 5) % 25, c2 = (i + 10) % 25, c3 = (i + 15) % 25, c4 = (i + 20) % 25;
    const int xm = (x + 4) % 5, xp = (x + 1) % 5;
    // pi: B[y + 5((2x + 3y) mod 5)] = rot(A[x + 5y]): lane (x, y) receives from (3(y - 3x) mod 5, x)
    const int src = (3 * (((y - 3 * x) % 5 + 5) % 5)) % 5 + 5 * x;
    const int n1 = (x + 1) % 5 + 5 * y, n2 = (x + 2) % 5 + 5 * y;
    const int r = KECCAK_RHO_C[i];
    const bool swap = (r & 32) != 0;
    const uint32_t sh = 32u - (uint32_t)(r & 31);  // alignbit amount (r & 31 == 0 -> no rotate)
    const bool rot = (r & 31) != 0;
#pragma unroll 1
    for (int round = 0; round < 24; round++) {
        uint32_t cl = kxor3(kxor3(lo, gshfl(lo, c1), gshfl(lo, c2)), gshfl(lo, c3), gshfl(lo, c4));
        uint32_t ch = kxor3(kxor3(hi, gshfl(hi, c1), gshfl(hi, c2)), gshfl(hi, c3), gshfl(hi, c4));
        uint32_t ml = gshfl(cl, xm), mh = gshfl(ch, xm), pl = gshfl(cl, xp), ph = gshfl(ch, xp);
        uint32_t rl, rh;
        krot<1>(rl, rh, pl, ph);
        uint32_t al = lo ^ ml ^ rl, ah = hi ^ mh ^ rh;
        // rho: rotate by r (r >= 32: swap halves, then by r - 32)
        uint32_t tl = swap ? ah : al, th = swap ? al : ah;
        uint32_t ol = rot ? __builtin_amdgcn_alignbit(tl, th, sh) : tl;
        uint32_t oh = rot ? __builtin_amdgcn_alignbit(th, tl, sh) : th;
        uint32_t bl = gshfl(ol, src), bh = gshfl(oh, src);
        uint32_t b1l = gshfl(bl, n1), b1h = gshfl(bh, n1), b2l = gshfl(bl, n2), b2h = gshfl(bh, n2);
        lo = kchi(bl, b1l, b2l);
        hi = kchi(bh, b1h, b2h);
        if (i == 0) {
            lo ^= (uint32_t)KECCAK_RC[round];
            hi ^= (uint32_t)(KECCAK_RC[round] >> 32);
        }
    }
}

// Keccak-256 of len bytes at m (8-byte aligned; LDS or global) by a 32-lane group (gl = lane in
// group); every lane of the group returns the digest words.
GSV_DI void keccak256_coop(uint32_t h[8], const uint8_t* m, uint32_t len, int gl) {
    const int i = gl < 25 ? gl : 24;
    uint32_t lo = 0, hi = 0;
    const uint64_t* q = (const uint64_t*)m;
    uint32_t nb = len / 136 + 1;
    for (uint32_t b = 0; b < nb; b++) {
        if (gl < 17) {
            uint64_t w;
            if (b + 1 < nb) {
                w = q[17 * b + gl];
            } else {
                int32_t avail = (int32_t)(len - 136 * b) - 8 * gl;
                w = avail >= 8 ? q[17 * b + gl] : avail > 0 ? q[17 * b + gl] & ((1ull << (8 * avail)) - 1ull) : 0ull;
                uint32_t rem = len - 136 * b;
                if ((rem >> 3) == (uint32_t)gl) w ^= 0x01ull << (8 * (rem & 7u));
                if (gl == 16) w ^= 0x8000000000000000ULL;
            }
            lo ^= (uint32_t)w;
            hi ^= (uint32_t)(w >> 32);
        }
        keccakf_coop(lo, hi, i);
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        h[2 * k] = gshfl(lo, k);
        h[2 * k + 1] = gshfl(hi, k);
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

// Lane-to-item order for a 256-thread workgroup whose lanes each absorb a variable number of rate
// blocks: a wave runs as many permutations as its longest message, so with tx-sized messages (one or
// two blocks) half a wave would idle through the second one.  Every thread passes its item's block
// count (`valid` false past the end); the items are bucketed by count (LDS counters and a prefix
// over the buckets) and the function returns the item this thread takes in that order, or ~0u.
// Results are written to each item's own slot, so they do not depend on the order.  All 256
// threads of the workgroup must call it (it has barriers).
constexpr uint32_t WG_BUCKETS = 10;  // 0..8 blocks, 9 = no item
GSV_DI uint32_t wg_bucket_order(uint32_t item, bool valid, uint64_t blocks) {
    __shared__ uint32_t s_cnt[WG_BUCKETS], s_base[WG_BUCKETS], s_idx[256];
    uint32_t t = threadIdx.x;
    if (t < WG_BUCKETS) s_cnt[t] = 0;
    __syncthreads();
    uint32_t key = !valid ? WG_BUCKETS - 1 : blocks < WG_BUCKETS - 2 ? (uint32_t)blocks : WG_BUCKETS - 2;
    uint32_t pos = atomicAdd(&s_cnt[key], 1u);
    __syncthreads();
    if (t == 0) {
        uint32_t acc = 0;
        for (uint32_t b = 0; b < WG_BUCKETS; b++) {
            s_base[b] = acc;
            acc += s_cnt[b];
        }
    }
    __syncthreads();
    s_idx[s_base[key] + pos] = valid ? item : ~0u;
    __syncthreads();
    return s_idx[t];
}

}  // namespace gsv

// secp256k1 device arithmetic for gfx950 — one signature per lane.
//
// Field elements mod p = 2^256 - 2^32 - 977 and scalars mod the group order n are 8 x 32-bit
// little-endian limbs held in VGPRs, always FULLY reduced (< modulus) between operations so
// that equality / parity tests are plain limb compares.  Products are 8x8 schoolbook
// product-scanning columns in inline asm (mul_asm.cuh: v_mad_u64_u32 with carry-out + addc);
// additions/reductions are __builtin_addc chains (v_add_co_u32 / v_addc_co_u32);
// reduction folds the high half with the sparse constant 2^256 mod p = 0x1000003D1
// (mod n: the 129-bit 2^256 - n).
//
// This restates the MATH of libsecp256k1's field/scalar/group layers (field_10x26_impl.h,
// scalar_8x32_impl.h, group_impl.h in crypto/secp256k1/libsecp256k1/src) for a SIMD machine;
// the algorithms (limb width, reduction, addition chains, coordinate formulas) are our own.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GSV_DI __device__ __forceinline__

#include "mul_asm.cuh"
#include "opcount.cuh"

namespace gsv {

struct fe { uint32_t v[8]; };
struct sc { uint32_t v[8]; };

// ------------------------------------------------------------------ generic limb helpers
GSV_DI uint32_t lo32(uint64_t x) { return (uint32_t)x; }
GSV_DI uint32_t hi32(uint64_t x) { return (uint32_t)(x >> 32); }
// carry-chain primitives: lower to v_add_co_u32 / v_addc_co_u32 / v_sub(b)_co_u32 chains
GSV_DI uint32_t addc(uint32_t a, uint32_t b, uint32_t& c) {
    uint32_t co;
    uint32_t r = __builtin_addc(a, b, c, &co);
    c = co;
    return r;
}
GSV_DI uint32_t subb(uint32_t a, uint32_t b, uint32_t& br) {
    uint32_t bo;
    uint32_t r = __builtin_subc(a, b, br, &bo);
    br = bo;
    return r;
}

// ------------------------------------------------------------------ field mod p
// p limbs (little endian)
__device__ constexpr uint32_t FP[8] = {0xFFFFFC2Fu, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                       0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};

// r = x if x < p else x - p, for x < 2^256 (uses x - p == x + 0x1000003D1 mod 2^256)
GSV_DI void fe_cond_sub_p(uint32_t r[8], const uint32_t x[8], uint32_t extra_carry) {
    uint32_t y[8], c = 0;
    y[0] = addc(x[0], 0x3D1u, c);
    y[1] = addc(x[1], 1u, c);
#pragma unroll
    for (int i = 2; i < 8; i++) y[i] = addc(x[i], 0u, c);
    uint32_t ge = c | extra_carry;  // x >= p  (or x had a 2^256 bit)
#pragma unroll
    for (int i = 0; i < 8; i++) r[i] = ge ? y[i] : x[i];
}

// reduce a 512-bit product mod p: T = H*2^256 + L == L + H*977 + H*2^32
GSV_DI void fe_reduce(fe& r, const uint32_t t[16]) {
    uint32_t pl[8], ph[8], s[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t p = (uint64_t)t[8 + i] * 977u;
        pl[i] = lo32(p);
        ph[i] = hi32(p);
    }
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = addc(t[i], pl[i], c);
    uint32_t s8 = c;
    c = 0;
#pragma unroll
    for (int i = 1; i < 8; i++) s[i] = addc(s[i], ph[i - 1], c);
    s8 = s8 + ph[7] + c;  // < 2^11
    c = 0;
#pragma unroll
    for (int i = 1; i < 8; i++) s[i] = addc(s[i], t[7 + i], c);
    uint32_t top_lo = addc(s8, t[15], c);  // top = c:top_lo < 2^33
    uint32_t top_hi = c;
    // s += top * (2^32 + 977): f = top * 977 < 2^43
    uint64_t f = (uint64_t)top_lo * 977u + (top_hi ? (977ull << 32) : 0ull);
    c = 0;
    s[0] = addc(s[0], lo32(f), c);
    s[1] = addc(s[1], hi32(f), c);
#pragma unroll
    for (int i = 2; i < 8; i++) s[i] = addc(s[i], 0u, c);
    uint32_t c2 = 0;
    s[1] = addc(s[1], top_lo, c2);
    s[2] = addc(s[2], top_hi, c2);
#pragma unroll
    for (int i = 3; i < 8; i++) s[i] = addc(s[i], 0u, c2);
    // a carry means s + 2^256 with s tiny: fold 2^256 == 0x1000003D1 once more (no further carry)
    uint32_t carry = c | c2;
    uint32_t c3 = 0;
    s[0] = addc(s[0], carry ? 0x3D1u : 0u, c3);
    s[1] = addc(s[1], carry, c3);
#pragma unroll
    for (int i = 2; i < 8; i++) s[i] = addc(s[i], 0u, c3);
    fe_cond_sub_p(r.v, s, 0);
}

// whole-product asm statements (mul_8x8_fx / sqr_8_fx, dedicated squaring)
GSV_DI void fe_mul(fe& r, const fe& a, const fe& b) {
    GSV_OPC(OPC_FE_MUL);
    uint32_t t[16];
    mul_8x8_fx(t, a.v, b.v);
    fe_reduce(r, t);
}
GSV_DI void fe_sqr(fe& r, const fe& a) {
    GSV_OPC(OPC_FE_SQR);
    uint32_t t[16];
    sqr_8_fx(t, a.v);
    fe_reduce(r, t);
}
GSV_DI void fe_sqr_n(fe& r, const fe& a, int n) {
    r = a;
#pragma unroll 1
    for (int i = 0; i < n; i++) fe_sqr(r, r);
}

GSV_DI void fe_add(fe& r, const fe& a, const fe& b) {
    uint32_t s[8], c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = addc(a.v[i], b.v[i], c);
    fe_cond_sub_p(r.v, s, c);
}

GSV_DI void fe_sub(fe& r, const fe& a, const fe& b) {
    uint32_t d[8], br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d[i] = subb(a.v[i], b.v[i], br);
    // if borrow: add p  (== subtract 0x1000003D1 mod 2^256)
    uint32_t m = 0u - br;
    uint32_t b2 = 0;
    r.v[0] = subb(d[0], m & 0x3D1u, b2);
    r.v[1] = subb(d[1], m & 1u, b2);
#pragma unroll
    for (int i = 2; i < 8; i++) r.v[i] = subb(d[i], 0u, b2);
}

GSV_DI bool fe_is_zero(const fe& a) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) o |= a.v[i];
    return o == 0;
}
GSV_DI bool fe_eq(const fe& a, const fe& b) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) o |= a.v[i] ^ b.v[i];
    return o == 0;
}
GSV_DI void fe_neg(fe& r, const fe& a) {
    fe z;
#pragma unroll
    for (int i = 0; i < 8; i++) z.v[i] = 0;
    fe_sub(r, z, a);
}
GSV_DI void fe_set_u32(fe& r, uint32_t x) {
    r.v[0] = x;
#pragma unroll
    for (int i = 1; i < 8; i++) r.v[i] = 0;
}
GSV_DI void fe_cmov(fe& r, const fe& a, bool flag) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = flag ? a.v[i] : r.v[i];
}

// x^(2^k - 1) ladder pieces shared by inversion and sqrt (block lengths 1,2,3,6,9,11,22,44,88,
// 176,220,223 of ones)
GSV_DI void fe_pow_x223(fe& x223, fe& x22, fe& x2, const fe& a) {
    fe x3, x6, x9, x11, x44, x88, x176, x220, t;
    fe_sqr(x2, a);
    fe_mul(x2, x2, a);
    fe_sqr(x3, x2);
    fe_mul(x3, x3, a);
    fe_sqr_n(t, x3, 3);
    fe_mul(x6, t, x3);
    fe_sqr_n(t, x6, 3);
    fe_mul(x9, t, x3);
    fe_sqr_n(t, x9, 2);
    fe_mul(x11, t, x2);
    fe_sqr_n(t, x11, 11);
    fe_mul(x22, t, x11);
    fe_sqr_n(t, x22, 22);
    fe_mul(x44, t, x22);
    fe_sqr_n(t, x44, 44);
    fe_mul(x88, t, x44);
    fe_sqr_n(t, x88, 88);
    fe_mul(x176, t, x88);
    fe_sqr_n(t, x176, 44);
    fe_mul(x220, t, x44);
    fe_sqr_n(t, x220, 3);
    fe_mul(x223, t, x3);
}

// a^(p-2):  p-2 = [223 ones] 0 [22 ones] 0000 1 0 11 0 1
GSV_DI void fe_inv(fe& r, const fe& a) {
    fe x223, x22, x2, t;
    fe_pow_x223(x223, x22, x2, a);
    fe_sqr_n(t, x223, 23);
    fe_mul(t, t, x22);
    fe_sqr_n(t, t, 5);
    fe_mul(t, t, a);
    fe_sqr_n(t, t, 3);
    fe_mul(t, t, x2);
    fe_sqr_n(t, t, 2);
    fe_mul(r, t, a);
}

// candidate sqrt a^((p+1)/4): (p+1)/4 = [223 ones] 0 [22 ones] 0000 11 00.
// Returns true iff r^2 == a (libsecp256k1 field_impl.h:38 secp256k1_fe_sqrt contract).
GSV_DI bool fe_sqrt(fe& r, const fe& a) {
    fe x223, x22, x2, t;
    fe_pow_x223(x223, x22, x2, a);
    fe_sqr_n(t, x223, 23);
    fe_mul(t, t, x22);
    fe_sqr_n(t, t, 6);
    fe_mul(t, t, x2);
    fe_sqr_n(r, t, 2);
    fe_sqr(t, r);
    return fe_eq(t, a);
}

// big-endian 32 bytes <-> limbs
GSV_DI void limbs_from_be(uint32_t v[8], const uint8_t* b) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint8_t* p = b + 28 - 4 * i;
        v[i] = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
    }
}
GSV_DI void limbs_from_be_words(uint32_t v[8], const uint32_t w[8]) {
    // w = 8 little-endian-loaded words of a big-endian 32-byte string
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = __builtin_bswap32(w[7 - i]);
}
GSV_DI void limbs_to_be(uint8_t* b, const uint32_t v[8]) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint8_t* p = b + 28 - 4 * i;
        p[0] = (uint8_t)(v[i] >> 24);
        p[1] = (uint8_t)(v[i] >> 16);
        p[2] = (uint8_t)(v[i] >> 8);
        p[3] = (uint8_t)v[i];
    }
}

// x < m ? (limb compare, m constant)
GSV_DI bool limbs_lt(const uint32_t x[8], const uint32_t m[8]) {
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) (void)subb(x[i], m[i], br);
    return br != 0;
}

// ------------------------------------------------------------------ scalars mod n
__device__ constexpr uint32_t SN[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                                       0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
// 2^256 - n (129 bits)
__device__ constexpr uint32_t SNC[5] = {0x2FC9BEBFu, 0x402DA173u, 0x50B75FC4u, 0x45512319u, 1u};

// r = x mod n for x < 2^256 + small carry (at most one subtraction needed for x < 2n)
GSV_DI void sc_cond_sub_n(uint32_t r[8], const uint32_t x[8], uint32_t extra_carry) {
    uint32_t y[8], c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) y[i] = addc(x[i], i < 5 ? SNC[i] : 0u, c);
    uint32_t ge = c | extra_carry;
#pragma unroll
    for (int i = 0; i < 8; i++) r[i] = ge ? y[i] : x[i];
}

// 2^256 == SNC (mod n), SNC = SNC' + 2^128 with SNC' = SNC[0..3].  Reduce a 512-bit product
// by three folds hi * SNC -> lo (the hi part shrinks 256 -> 130 -> 35 -> 0 bits).
GSV_DI void sc_reduce(sc& r, const uint32_t t[16]) {
    const uint32_t C4[4] = {SNC[0], SNC[1], SNC[2], SNC[3]};
    // stage 1: m = L + H*SNC' + H*2^128  (< 2^386, 13 limbs)
    uint32_t p[12], m[13], c = 0;
    mul_8x4_fx(p, t + 8, C4);
#pragma unroll
    for (int i = 0; i < 8; i++) m[i] = addc(t[i], p[i], c);
#pragma unroll
    for (int i = 8; i < 12; i++) m[i] = addc(p[i], 0u, c);
    m[12] = c;
    c = 0;
#pragma unroll
    for (int i = 4; i < 12; i++) m[i] = addc(m[i], t[4 + i], c);
    m[12] += c;
    // stage 2: m2 = m[0..7] + m[8..12]*SNC' + m[8..12]*2^128  (< 2^291, 10 limbs)
    uint32_t p2[9], m2[10];
    mul_5x4_fx(p2, m + 8, C4);
    c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) m2[i] = addc(m[i], p2[i], c);
    m2[8] = addc(p2[8], 0u, c);
    m2[9] = c;
    c = 0;
#pragma unroll
    for (int i = 4; i < 9; i++) m2[i] = addc(m2[i], m[4 + i], c);
    m2[9] += c;
    // stage 3: m3 = m2[0..7] + m2[8..9]*SNC' + m2[8..9]*2^128  (< 2^256 + 2^166, carry limb 0/1)
    uint32_t p3[6], m3[8];
    mul_2x4_fx(p3, m2 + 8, C4);
    c = 0;
#pragma unroll
    for (int i = 0; i < 6; i++) m3[i] = addc(m2[i], p3[i], c);
    m3[6] = addc(m2[6], 0u, c);
    m3[7] = addc(m2[7], 0u, c);
    uint32_t c2 = 0;
    m3[4] = addc(m3[4], m2[8], c2);
    m3[5] = addc(m3[5], m2[9], c2);
    m3[6] = addc(m3[6], 0u, c2);
    m3[7] = addc(m3[7], 0u, c2);
    // value = m3 + (c + c2) * 2^256 < 2^256 + 2^166 < 2n: one conditional subtraction
    sc_cond_sub_n(r.v, m3, c | c2);
}

GSV_DI void sc_mul(sc& r, const sc& a, const sc& b) {
    GSV_OPC(OPC_SC_MUL);
    uint32_t t[16];
    mul_8x8_fx(t, a.v, b.v);
    sc_reduce(r, t);
}
GSV_DI void sc_sqr(sc& r, const sc& a) {
    GSV_OPC(OPC_SC_SQR);
    uint32_t t[16];
    sqr_8_fx(t, a.v);
    sc_reduce(r, t);
}
GSV_DI bool sc_is_zero(const sc& a) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) o |= a.v[i];
    return o == 0;
}
GSV_DI void sc_neg(sc& r, const sc& a) {
    // n - a, 0 -> 0
    bool z = sc_is_zero(a);
    int64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        int64_t t = (int64_t)SN[i] - a.v[i] + br;
        r.v[i] = z ? 0u : (uint32_t)t;
        br = t >> 32;
    }
}
GSV_DI void sc_add(sc& r, const sc& a, const sc& b) {
    uint32_t s[8], c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = addc(a.v[i], b.v[i], c);
    sc_cond_sub_n(r.v, s, c);
}

// a^(n-2): n-2 = [127 ones] 0 || 0xBAAEDCE6AF48A03BBFD25E8CD036413F.  The run of ones uses an
// addition chain (x^(2^k-1) blocks), the low 128 bits plain square-and-multiply on the public
// exponent (uniform branches, no table, no scratch).
GSV_DI void sc_sqr_n(sc& r, const sc& a, int n) {
    r = a;
#pragma unroll 1
    for (int i = 0; i < n; i++) sc_sqr(r, r);
}
GSV_DI void sc_inv(sc& r, const sc& a) {
    sc x2, x3, x6, x12, x24, x48, x96, t;
    sc_sqr(x2, a);
    sc_mul(x2, x2, a);
    sc_sqr(x3, x2);
    sc_mul(x3, x3, a);
    sc_sqr_n(t, x3, 3);
    sc_mul(x6, t, x3);
    sc_sqr_n(t, x6, 6);
    sc_mul(x12, t, x6);
    sc_sqr_n(t, x12, 12);
    sc_mul(x24, t, x12);
    sc_sqr_n(t, x24, 24);
    sc_mul(x48, t, x24);
    sc_sqr_n(t, x48, 48);
    sc_mul(x96, t, x48);
    sc_sqr_n(t, x96, 24);
    sc_mul(t, t, x24);      // x120
    sc_sqr_n(t, t, 6);
    sc_mul(t, t, x6);       // x126
    sc_sqr(t, t);
    sc_mul(t, t, a);        // x127
    sc_sqr(t, t);           // the 0 bit (bit 128)
    const uint32_t E0 = 0xD036413Fu, E1 = 0xBFD25E8Cu, E2 = 0xAF48A03Bu, E3 = 0xBAAEDCE6u;
#pragma unroll 1
    for (int b = 127; b >= 0; b--) {
        sc_sqr(t, t);
        uint32_t w = (b >= 96) ? E3 : (b >= 64) ? E2 : (b >= 32) ? E1 : E0;
        if ((w >> (b & 31)) & 1u) sc_mul(t, t, a);
    }
    r = t;
}

// word k of a small array with a runtime (wave-uniform) index, via selects (no scratch)
template <int N>
GSV_DI uint32_t sel_word(const uint32_t (&w)[N], uint32_t k) {
    uint32_t r = w[0];
#pragma unroll
    for (int i = 1; i < N; i++) r = (k == (uint32_t)i) ? w[i] : r;
    return r;
}

// ------------------------------------------------------------------ group: Jacobian, a = 0
struct gej { fe x, y, z; };
struct ge { fe x, y; };

// dbl-2009-l: 2M + 5S.  Input must not be infinity; Y == 0 cannot occur on secp256k1
// (no point of order 2).
GSV_DI void gej_dbl(gej& r, const gej& p) {
    fe A, B, C, D, E, F, t;
    fe_sqr(A, p.x);
    fe_sqr(B, p.y);
    fe_sqr(C, B);
    fe_add(t, p.x, B);
    fe_sqr(t, t);
    fe_sub(t, t, A);
    fe_sub(t, t, C);
    fe_add(D, t, t);
    fe_add(E, A, A);
    fe_add(E, E, A);
    fe_sqr(F, E);
    fe z3;
    fe_mul(z3, p.y, p.z);
    fe_add(r.z, z3, z3);
    fe_sub(t, F, D);
    fe_sub(r.x, t, D);
    fe_sub(t, D, r.x);
    fe_mul(t, E, t);
    fe_add(C, C, C);
    fe_add(C, C, C);
    fe_add(C, C, C);
    fe_sub(r.y, t, C);
}

typedef uint32_t gsv_v8 __attribute__((ext_vector_type(8)));
typedef uint32_t gsv_v32 __attribute__((ext_vector_type(32)));
// Rare path of the mixed add (p == q): the doubling, out of line so the hot loops stay small in
// I-cache.  Values travel in VGPR vectors (an aggregate or a pointer argument would pin the
// caller's accumulator to scratch memory for the whole loop).
__device__ __noinline__ gsv_v32 gej_dbl_ool(gsv_v8 x, gsv_v8 y, gsv_v8 z) {
    gej p, d;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        p.x.v[i] = x[i];
        p.y.v[i] = y[i];
        p.z.v[i] = z[i];
    }
    gej_dbl(d, p);
    gsv_v32 o;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        o[i] = d.x.v[i];
        o[8 + i] = d.y.v[i];
        o[16 + i] = d.z.v[i];
        o[24 + i] = 0;
    }
    return o;
}
GSV_DI void gej_add_ge_exceptional(gej& r, bool& inf, const gej& p, const fe& rr) {
    if (fe_is_zero(rr)) {
        gsv_v8 x, y, z;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            x[i] = p.x.v[i];
            y[i] = p.y.v[i];
            z[i] = p.z.v[i];
        }
        gsv_v32 o = gej_dbl_ool(x, y, z);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            r.x.v[i] = o[i];
            r.y.v[i] = o[8 + i];
            r.z.v[i] = o[16 + i];
        }
    } else {
        inf = true;
        r = p;
    }
}

// mixed add r = p + q, q affine. madd-2007-bl: 7M + 4S.
// inf: in/out flag for p; handles p == inf, p == q (doubling), p == -q (infinity).
GSV_DI void gej_add_ge(gej& r, bool& inf, const gej& p, const ge& q) {
    fe z1z1, u2, s2, h, hh, i4, j, rr, v, t;
    fe_sqr(z1z1, p.z);
    fe_mul(u2, q.x, z1z1);
    fe_mul(s2, q.y, p.z);
    fe_mul(s2, s2, z1z1);
    fe_sub(h, u2, p.x);
    fe_sub(rr, s2, p.y);
    bool exc = fe_is_zero(h) && !inf;
    if (__builtin_expect(exc, 0)) {
        gej_add_ge_exceptional(r, inf, p, rr);
        return;
    }
    fe_sqr(hh, h);
    fe_add(i4, hh, hh);
    fe_add(i4, i4, i4);
    fe_mul(j, h, i4);
    fe_add(rr, rr, rr);
    fe_mul(v, p.x, i4);
    gej o;
    fe_sqr(t, rr);
    fe_sub(t, t, j);
    fe_sub(t, t, v);
    fe_sub(o.x, t, v);
    fe_sub(t, v, o.x);
    fe_mul(t, rr, t);
    fe_mul(v, p.y, j);
    fe_add(v, v, v);
    fe_sub(o.y, t, v);
    fe_add(t, p.z, h);
    fe_sqr(t, t);
    fe_sub(t, t, z1z1);
    fe_sub(o.z, t, hh);
    // p == inf -> result is q
    if (inf) {
        o.x = q.x;
        o.y = q.y;
        fe_set_u32(o.z, 1);
    }
    inf = false;
    r = o;
}

// general add r = p + q (both Jacobian), add-2007-bl: 11M + 5S; handles all exceptions.
GSV_DI void gej_add(gej& r, bool& rinf, const gej& p, bool pinf, const gej& q, bool qinf) {
    if (pinf) { r = q; rinf = qinf; return; }
    if (qinf) { r = p; rinf = false; return; }
    fe z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t;
    fe_sqr(z1z1, p.z);
    fe_sqr(z2z2, q.z);
    fe_mul(u1, p.x, z2z2);
    fe_mul(u2, q.x, z1z1);
    fe_mul(s1, p.y, q.z);
    fe_mul(s1, s1, z2z2);
    fe_mul(s2, q.y, p.z);
    fe_mul(s2, s2, z1z1);
    fe_sub(h, u2, u1);
    fe_sub(rr, s2, s1);
    if (fe_is_zero(h)) {
        if (fe_is_zero(rr)) {
            gej_dbl(r, p);
            rinf = false;
        } else {
            rinf = true;
            r = p;
        }
        return;
    }
    fe_add(i, h, h);
    fe_sqr(i, i);
    fe_mul(j, h, i);
    fe_add(rr, rr, rr);
    fe_mul(v, u1, i);
    gej o;
    fe_sqr(t, rr);
    fe_sub(t, t, j);
    fe_sub(t, t, v);
    fe_sub(o.x, t, v);
    fe_sub(t, v, o.x);
    fe_mul(t, rr, t);
    fe_mul(s1, s1, j);
    fe_add(s1, s1, s1);
    fe_sub(o.y, t, s1);
    fe_add(t, p.z, q.z);
    fe_sqr(t, t);
    fe_sub(t, t, z1z1);
    fe_sub(t, t, z2z2);
    fe_mul(o.z, t, h);
    r = o;
    rinf = false;
}

}  // namespace gsv

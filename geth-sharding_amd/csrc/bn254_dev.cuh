// BN254 device arithmetic for gfx950 — the pairing check of crypto/bn256 (cloudflare).
//
// F_p elements are 8 x 32-bit little-endian limbs in VGPRs, in the reference's Montgomery form
// (R = 2^256, crypto/bn256/cloudflare/gfp.go) and always canonical (< p), so every value the
// kernels compute is bit-identical to the reference's gfP words (and to oracle/bn256_oracle.c).
// Products are product-scanning Montgomery multiplications (mul_asm.cuh mont_mul_8_asm:
// v_mad_u64_u32 column accumulators, modulus words in SGPRs).
//
// Tower and curve formulas restate crypto/bn256/cloudflare/{gfp2,gfp6,gfp12,twist,optate}.go
// operation for operation (file:line at each function); MI355X-specific choices (limb width,
// reduction, code layout) are ours.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GSV_DI __device__ __forceinline__

#include "modinv30.cuh"
#include "mul_asm.cuh"

namespace gsv {
namespace bn {

// ---------------------------------------------------------------- constants (constants.go)
__device__ constexpr uint32_t BN_P[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                         0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
constexpr uint32_t BN_N0 = 0xe4866389u;  // -p^-1 mod 2^32 (low word of np)
__device__ constexpr uint32_t BN_R2[8] = {0x538afa89u, 0xf32cfc5bu, 0xd44501fbu, 0xb5e71911u,
                                          0x0a417ff6u, 0x47ab1effu, 0xcab8351fu, 0x06d89f71u};
__device__ constexpr uint32_t BN_ONE[8] = {0xc58f0d9du, 0xd35d438du, 0xf5c70b3du, 0x0a78eb28u,
                                           0x7879462cu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
__device__ constexpr uint32_t BN_THREE[8] = {0x50ad28d7u, 0x7a17caa9u, 0xe15521b9u, 0x1f6ac17au,
                                             0x696bd284u, 0x334bea4eu, 0xce179d8eu, 0x2a1f6744u};
__device__ constexpr uint32_t BN_PM2[8] = {0xd87cfd45u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                           0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
__device__ constexpr uint32_t BN_ORDER[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                                             0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
__device__ constexpr uint32_t XI_P1_6_X[8] = {0x4c492d72u, 0xa222ae23u, 0x565de15bu, 0xd00f02a4u,
                                              0x53dfc926u, 0xdc2ff3a2u, 0xb3899551u, 0x10a75716u};
__device__ constexpr uint32_t XI_P1_6_Y[8] = {0x33144907u, 0xaf9ba696u, 0x87afb78au, 0xca6b1d73u,
                                              0xf08a2087u, 0x11bded5eu, 0x1a1f3a7cu, 0x02f34d75u};
__device__ constexpr uint32_t XI_P1_3_X[8] = {0xa0aa4757u, 0x6e849f1eu, 0x89f89141u, 0xaa1c7b6du,
                                              0xfae0ca3au, 0xb6e713cdu, 0x4e82ebc3u, 0x26694fbbu};
__device__ constexpr uint32_t XI_P1_3_Y[8] = {0x4563ab30u, 0xb5773b10u, 0xa9aa6454u, 0x347f91c8u,
                                              0x242e0991u, 0x7a007127u, 0x118214ecu, 0x1956bcd8u};
__device__ constexpr uint32_t XI_P1_2_X[8] = {0x5ffe77c7u, 0xa1d77ce4u, 0x7826d1dbu, 0x07affd11u,
                                              0xbb7edc6bu, 0x6d16bd27u, 0x85defeccu, 0x2c872002u};
__device__ constexpr uint32_t XI_P1_2_Y[8] = {0x2936b629u, 0xe4bbdd0cu, 0xe133bacbu, 0xbb30f162u,
                                              0xf9645366u, 0x31a9d1b6u, 0xa500f8ddu, 0x253570beu};
__device__ constexpr uint32_t XI_PSQ1_3[8] = {0x13e80b9cu, 0x3350c88eu, 0xdb5e56b9u, 0x7dce557cu,
                                              0xb615564au, 0x6001b4b8u, 0x020217e0u, 0x2682e617u};
__device__ constexpr uint32_t XI_2PSQ2_3[8] = {0xd782e155u, 0x71930c11u, 0xffbe3323u, 0xa6bb947cu,
                                               0xd4741444u, 0xaa303344u, 0x26594943u, 0x2c3b3f0du};
__device__ constexpr uint32_t XI_PSQ1_6[8] = {0x00fa1bf2u, 0xca8d8005u, 0x68b39769u, 0xf0c5d614u,
                                              0xad0d4418u, 0x0e201271u, 0xbad856e6u, 0x04290f65u};
__device__ constexpr uint32_t XI_2P2_3_X[8] = {0x4bd8c949u, 0x5dddfd15u, 0xa4445b60u, 0x62cb29a5u,
                                               0x0c7dd2b9u, 0x37bc870au, 0x3171f0fdu, 0x24830a9du};
__device__ constexpr uint32_t XI_2P2_3_Y[8] = {0x843abe92u, 0x7361d77fu, 0x273411fbu, 0xa5bb2bd3u,
                                               0x4b3e2399u, 0x9c941f31u, 0xbb9fd3ecu, 0x15df9cddu};
__device__ constexpr uint32_t TWIST_B_X[8] = {0xd1dcff67u, 0x38e7ecccu, 0x93ce0d3eu, 0x65f0b37du,
                                              0x22ac00aau, 0xd749d0ddu, 0x4a688d4du, 0x0141b9ceu};
__device__ constexpr uint32_t TWIST_B_Y[8] = {0x77b802a8u, 0x3bf938e3u, 0x3633535du, 0x020b1b27u,
                                              0x49755260u, 0x26b7edf0u, 0x4384a86du, 0x2514c632u};
constexpr uint64_t BN_U = 4965661367192848881ULL;  // constants.go:17
// sixuPlus2NAF (optate.go:114-118) digits 0..63 as two bit masks (digit 64 is the leading 1)
constexpr uint64_t NAF_POS = 0xa1818041c0864428ULL;  // bit i set where digit i == +1
constexpr uint64_t NAF_NEG = 0x0408100802100880ULL;  // bit i set where digit i == -1

struct fp { uint32_t v[8]; };
struct fp2 { fp x, y; };          // x*i + y
struct fp6 { fp2 x, y, z; };      // x*tau^2 + y*tau + z
struct fp12 { fp6 x, y; };        // x*omega + y
struct g1a { fp x, y; };          // affine G1 point (Montgomery)
struct g2a { fp2 x, y; };         // affine G2 point
struct g2j { fp2 x, y, z, t; };   // twistPoint (Jacobian, t = z^2 where maintained)

// ---------------------------------------------------------------- F_p (gfp_generic.go)
GSV_DI uint32_t add_c(uint32_t a, uint32_t b, uint32_t& c) {
    uint32_t co;
    uint32_t r = __builtin_addc(a, b, c, &co);
    c = co;
    return r;
}
GSV_DI uint32_t sub_b(uint32_t a, uint32_t b, uint32_t& br) {
    uint32_t bo;
    uint32_t r = __builtin_subc(a, b, br, &bo);
    br = bo;
    return r;
}
GSV_DI void fp_const(fp& r, const uint32_t c[8]) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = c[i];
}
GSV_DI void fp_zero(fp& r) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = 0;
}
// r = x - p if x >= p (x < 2^256 plus `hi` carry) else x   (gfpCarry)
GSV_DI void fp_reduce_once(fp& r, const uint32_t x[8], uint32_t hi) {
    uint32_t d[8], br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d[i] = sub_b(x[i], BN_P[i], br);
    bool take = hi || !br;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = take ? d[i] : x[i];
}
GSV_DI void fp_add(fp& r, const fp& a, const fp& b) {
    uint32_t s[8], c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = add_c(a.v[i], b.v[i], c);
    fp_reduce_once(r, s, c);
}
GSV_DI void fp_sub(fp& r, const fp& a, const fp& b) {
    uint32_t d[8], br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d[i] = sub_b(a.v[i], b.v[i], br);
    uint32_t m = 0u - br, c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = add_c(d[i], BN_P[i] & m, c);
}
GSV_DI bool fp_is_zero(const fp& a) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) o |= a.v[i];
    return o == 0;
}
GSV_DI bool fp_eq(const fp& a, const fp& b) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) o |= a.v[i] ^ b.v[i];
    return o == 0;
}
GSV_DI void fp_neg(fp& r, const fp& a) {  // p - a, 0 -> 0
    bool z = fp_is_zero(a);
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint32_t d = sub_b(BN_P[i], a.v[i], br);
        r.v[i] = z ? 0u : d;
    }
}
GSV_DI void fp_mul(fp& r, const fp& a, const fp& b) {
    GSV_OPC(gsv::OPC_BN_MUL);
    uint32_t t[8];
    uint32_t hi = mont_mul_8_asm(t, a.v, b.v, BN_P, BN_N0);
    fp_reduce_once(r, t, hi);
}
GSV_DI bool fp_geq_p(const uint32_t x[8]) {
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) (void)sub_b(x[i], BN_P[i], br);
    return br == 0;
}

// ---------------------------------------------------------------- code layout
// A Miller loop or final exponentiation fully inlined is ~10^5 instructions: too big for the
// CU instruction cache and for the compiler.  The F_p product is therefore an out-of-line leaf
// function taking and returning VGPR vectors (no memory traffic), and the F_p^6 / F_p^12 /
// curve routines are out-of-line functions over per-lane (scratch) pointers, called at a
// granularity where the 96-word loads/stores are negligible next to the arithmetic.
typedef uint32_t v8 __attribute__((ext_vector_type(8)));
typedef uint32_t v16 __attribute__((ext_vector_type(16)));
#define BN_NI __device__ __noinline__

GSV_DI v8 tov(const fp& a) {
    v8 r;
#pragma unroll
    for (int i = 0; i < 8; i++) r[i] = a.v[i];
    return r;
}
GSV_DI fp fromv(v8 a) {
    fp r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = a[i];
    return r;
}
GSV_DI v16 cat(const fp& x, const fp& y) {
    v16 r;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        r[i] = x.v[i];
        r[8 + i] = y.v[i];
    }
    return r;
}

static BN_NI v8 fp_mul_v(v8 a, v8 b) {
    fp x = fromv(a), y = fromv(b), r;
    fp_mul(r, x, y);
    return tov(r);
}
GSV_DI void fp_mul_c(fp& r, const fp& a, const fp& b) { r = fromv(fp_mul_v(tov(a), tov(b))); }
GSV_DI void fp_sqr_c(fp& r, const fp& a) { fp_mul_c(r, a, a); }
// Inverse of a Montgomery residue aR: safegcd (modinv30.cuh, ~8k issue slots) gives (aR)^-1 =
// a^-1 R^-1, and one Montgomery product by R^3 mod p turns it into a^-1 R — the same canonical
// residue as the reference's a^(p-2) (gfp.go:31-49), whose 254 squarings + 127 products it replaces.
__device__ constexpr uint32_t BN_R3[8] = {0xda1530dfu, 0xb1cd6dafu, 0xa7283db6u, 0x62f210e6u,
                                          0x0ada0afbu, 0xef7f0b0cu, 0x2d592544u, 0x20fd6e90u};
GSV_DI void fp_inv(fp& r, const fp& a) {
    fp t, r3;
    modinv30_words(t.v, a.v, MI30_BN);
    fp_const(r3, BN_R3);
    fp_mul_c(r, t, r3);
}

// ---------------------------------------------------------------- F_p^2 (gfp2.go)
GSV_DI void fp2_zero(fp2& e) { fp_zero(e.x); fp_zero(e.y); }
GSV_DI void fp2_one(fp2& e) { fp_zero(e.x); fp_const(e.y, BN_ONE); }
GSV_DI bool fp2_is_zero(const fp2& e) { return fp_is_zero(e.x) && fp_is_zero(e.y); }
GSV_DI bool fp2_eq(const fp2& a, const fp2& b) { return fp_eq(a.x, b.x) && fp_eq(a.y, b.y); }
GSV_DI void fp2_const(fp2& e, const uint32_t x[8], const uint32_t y[8]) { fp_const(e.x, x); fp_const(e.y, y); }
GSV_DI void fp2_conj(fp2& e, const fp2& a) { e.y = a.y; fp_neg(e.x, a.x); }
GSV_DI void fp2_neg(fp2& e, const fp2& a) { fp_neg(e.x, a.x); fp_neg(e.y, a.y); }
GSV_DI void fp2_add(fp2& e, const fp2& a, const fp2& b) { fp_add(e.x, a.x, b.x); fp_add(e.y, a.y, b.y); }
GSV_DI void fp2_sub(fp2& e, const fp2& a, const fp2& b) { fp_sub(e.x, a.x, b.x); fp_sub(e.y, a.y, b.y); }

// F_p^2 products are inlined compositions of the out-of-line F_p product (fp_mul_v: 28 VGPRs, no
// callee-saved registers, so a call spills nothing); an out-of-line F_p^2 product needed ~100
// VGPRs and saved/restored 32 callee-saved registers through scratch on every call (A/B on
// MI355X: Miller loop 50.6 -> 48.8 ms, final exponentiation 21.1 -> 20.0 ms per 65,536 checks).
#define BN_FP2 GSV_DI
#define fp_mul fp_mul_c
// gfp2.go:83-98: x = ax*by + bx*ay, y = ay*by - ax*bx.  Karatsuba form (3 products):
// x = (ax+ay)(bx+by) - ax*bx - ay*by — the same canonical residues.
BN_FP2 v16 fp2_mul_v(v8 ax_, v8 ay_, v8 bx_, v8 by_) {
    fp ax = fromv(ax_), ay = fromv(ay_), bx = fromv(bx_), by = fromv(by_);
    fp t0, t1, s0, s1, x, y;
    fp_mul(t0, ax, bx);
    fp_mul(t1, ay, by);
    fp_add(s0, ax, ay);
    fp_add(s1, bx, by);
    fp_mul(x, s0, s1);
    fp_sub(x, x, t0);
    fp_sub(x, x, t1);
    fp_sub(y, t1, t0);
    return cat(x, y);
}
// gfp2.go:130-143: (x i + y)^2 = 2xy i + (y - x)(y + x)
BN_FP2 v16 fp2_sqr_v(v8 x_, v8 y_) {
    fp ax = fromv(x_), ay = fromv(y_), tx, ty;
    fp_sub(tx, ay, ax);
    fp_add(ty, ax, ay);
    fp_mul(ty, tx, ty);
    fp_mul(tx, ax, ay);
    fp_add(tx, tx, tx);
    return cat(tx, ty);
}
BN_FP2 v16 fp2_mul_fp_v(v8 ax_, v8 ay_, v8 b_) {
    fp ax = fromv(ax_), ay = fromv(ay_), b = fromv(b_), x, y;
    fp_mul(x, ax, b);
    fp_mul(y, ay, b);
    return cat(x, y);
}
#undef fp_mul
GSV_DI void fp2_from(fp2& e, v16 r) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
        e.x.v[i] = r[i];
        e.y.v[i] = r[8 + i];
    }
}
GSV_DI void fp2_mul(fp2& e, const fp2& a, const fp2& b) { fp2_from(e, fp2_mul_v(tov(a.x), tov(a.y), tov(b.x), tov(b.y))); }
GSV_DI void fp2_sqr(fp2& e, const fp2& a) { fp2_from(e, fp2_sqr_v(tov(a.x), tov(a.y))); }
GSV_DI void fp2_mul_fp(fp2& e, const fp2& a, const fp& b) { fp2_from(e, fp2_mul_fp_v(tov(a.x), tov(a.y), tov(b))); }
// gfp2.go:107-128: (x i + y)(i + 9) = (9x + y) i + (9y - x)
GSV_DI void fp2_mul_xi(fp2& e, const fp2& a) {
    fp tx, ty;
    fp_add(tx, a.x, a.x);
    fp_add(tx, tx, tx);
    fp_add(tx, tx, tx);
    fp_add(tx, tx, a.x);
    fp_add(tx, tx, a.y);
    fp_add(ty, a.y, a.y);
    fp_add(ty, ty, ty);
    fp_add(ty, ty, ty);
    fp_add(ty, ty, a.y);
    fp_sub(ty, ty, a.x);
    e.x = tx;
    e.y = ty;
}
// gfp2.go:145-156
GSV_DI void fp2_inv(fp2& e, const fp2& a) {
    fp t1, t2, inv;
    fp_sqr_c(t1, a.x);
    fp_sqr_c(t2, a.y);
    fp_add(t1, t1, t2);
    fp_inv(inv, t1);
    fp_neg(t1, a.x);
    fp_mul_c(e.x, t1, inv);
    fp_mul_c(e.y, a.y, inv);
}

// ---------------------------------------------------------------- F_p^6 (gfp6.go)
GSV_DI void fp6_zero(fp6& e) { fp2_zero(e.x); fp2_zero(e.y); fp2_zero(e.z); }
GSV_DI void fp6_one(fp6& e) { fp2_zero(e.x); fp2_zero(e.y); fp2_one(e.z); }
GSV_DI void fp6_neg(fp6& e, const fp6& a) { fp2_neg(e.x, a.x); fp2_neg(e.y, a.y); fp2_neg(e.z, a.z); }
GSV_DI void fp6_add(fp6& e, const fp6& a, const fp6& b) { fp2_add(e.x, a.x, b.x); fp2_add(e.y, a.y, b.y); fp2_add(e.z, a.z, b.z); }
GSV_DI void fp6_sub(fp6& e, const fp6& a, const fp6& b) { fp2_sub(e.x, a.x, b.x); fp2_sub(e.y, a.y, b.y); fp2_sub(e.z, a.z, b.z); }
// gfp6.go:54-62
GSV_DI void fp6_frob(fp6& e, const fp6& a) {
    fp2 c, k;
    fp2_conj(e.z, a.z);
    fp2_conj(c, a.x);
    fp2_const(k, XI_2P2_3_X, XI_2P2_3_Y);
    fp2_mul(e.x, c, k);
    fp2_conj(c, a.y);
    fp2_const(k, XI_P1_3_X, XI_P1_3_Y);
    fp2_mul(e.y, c, k);
}
// gfp6.go:65-73
GSV_DI void fp6_frob_p2(fp6& e, const fp6& a) {
    fp k;
    fp_const(k, XI_2PSQ2_3);
    fp2_mul_fp(e.x, a.x, k);
    fp_const(k, XI_PSQ1_3);
    fp2_mul_fp(e.y, a.y, k);
    e.z = a.z;
}
// gfp6.go:96-123 (Karatsuba).  The *_i forms are always inlined (the Miller loop keeps its whole
// state in VGPRs); the *_p forms are out-of-line wrappers for the colder callers.
GSV_DI void fp6_mul_i(fp6& e, const fp6& pa_, const fp6& pb_) {
    const fp6 a = pa_, b = pb_;
    fp2 v0, v1, v2, t0, t1, tz, ty, tx;
    fp2_mul(v0, a.z, b.z);
    fp2_mul(v1, a.y, b.y);
    fp2_mul(v2, a.x, b.x);
    fp2_add(t0, a.x, a.y);
    fp2_add(t1, b.x, b.y);
    fp2_mul(tz, t0, t1);
    fp2_sub(tz, tz, v1);
    fp2_sub(tz, tz, v2);
    fp2_mul_xi(tz, tz);
    fp2_add(tz, tz, v0);
    fp2_add(t0, a.y, a.z);
    fp2_add(t1, b.y, b.z);
    fp2_mul(ty, t0, t1);
    fp2_mul_xi(t0, v2);
    fp2_sub(ty, ty, v0);
    fp2_sub(ty, ty, v1);
    fp2_add(ty, ty, t0);
    fp2_add(t0, a.x, a.z);
    fp2_add(t1, b.x, b.z);
    fp2_mul(tx, t0, t1);
    fp2_sub(tx, tx, v0);
    fp2_add(tx, tx, v1);
    fp2_sub(tx, tx, v2);
    e.x = tx;
    e.y = ty;
    e.z = tz;
}
static BN_NI void fp6_mul_p(fp6* e, const fp6* pa, const fp6* pb) { fp6_mul_i(*e, *pa, *pb); }
GSV_DI void fp6_mul(fp6& e, const fp6& a, const fp6& b) { fp6_mul_p(&e, &a, &b); }
// e = a * (by tau + bz) (a line's sparse factor, x coefficient 0): 5 F_p^2 products instead of 6;
// the same field element as fp6_mul with b.x = 0, hence the same canonical words.
GSV_DI void fp6_mul_sparse_i(fp6& e, const fp6& pa_, const fp2& pby_, const fp2& pbz_) {
    const fp6 a = pa_;
    const fp2 by = pby_, bz = pbz_;
    fp2 v0, v1, t0, t1, tx, ty, tz;
    fp2_mul(v0, a.z, bz);
    fp2_mul(v1, a.y, by);
    fp2_mul(tz, a.x, by);  // tau^3 = xi
    fp2_mul_xi(tz, tz);
    fp2_add(tz, tz, v0);
    fp2_add(t0, a.y, a.z);
    fp2_add(t1, by, bz);
    fp2_mul(ty, t0, t1);
    fp2_sub(ty, ty, v0);
    fp2_sub(ty, ty, v1);
    fp2_mul(tx, a.x, bz);
    fp2_add(tx, tx, v1);
    e.x = tx;
    e.y = ty;
    e.z = tz;
}
static BN_NI void fp6_mul_sparse_p(fp6* e, const fp6* pa, const fp2* pby, const fp2* pbz) {
    fp6_mul_sparse_i(*e, *pa, *pby, *pbz);
}
GSV_DI void fp6_mul_fp2_i(fp6& e, const fp6& a_, const fp2& b_) {
    const fp6 a = a_;
    const fp2 b = b_;
    fp2_mul(e.x, a.x, b);
    fp2_mul(e.y, a.y, b);
    fp2_mul(e.z, a.z, b);
}
static BN_NI void fp6_mul_fp2_p(fp6* e, const fp6* a, const fp2* b) { fp6_mul_fp2_i(*e, *a, *b); }
GSV_DI void fp6_mul_fp2(fp6& e, const fp6& a, const fp2& b) { fp6_mul_fp2_p(&e, &a, &b); }
GSV_DI void fp6_mul_fp(fp6& e, const fp6& a, const fp& b) { fp2_mul_fp(e.x, a.x, b); fp2_mul_fp(e.y, a.y, b); fp2_mul_fp(e.z, a.z, b); }
// gfp6.go:140-149: tau (x tau^2 + y tau + z) = y tau^2 + z tau + x xi
GSV_DI void fp6_mul_tau(fp6& e, const fp6& a) {
    fp2 tz, ty;
    fp2_mul_xi(tz, a.x);
    ty = a.y;
    e.y = a.z;
    e.x = ty;
    e.z = tz;
}
// gfp6.go:151-170
static BN_NI void fp6_sqr_p(fp6* e, const fp6* pa) {
    const fp6 a = *pa;
    fp2 v0, v1, v2, c0, c1, c2, xiv2;
    fp2_sqr(v0, a.z);
    fp2_sqr(v1, a.y);
    fp2_sqr(v2, a.x);
    fp2_add(c0, a.x, a.y);
    fp2_sqr(c0, c0);
    fp2_sub(c0, c0, v1);
    fp2_sub(c0, c0, v2);
    fp2_mul_xi(c0, c0);
    fp2_add(c0, c0, v0);
    fp2_add(c1, a.y, a.z);
    fp2_sqr(c1, c1);
    fp2_sub(c1, c1, v0);
    fp2_sub(c1, c1, v1);
    fp2_mul_xi(xiv2, v2);
    fp2_add(c1, c1, xiv2);
    fp2_add(c2, a.x, a.z);
    fp2_sqr(c2, c2);
    fp2_sub(c2, c2, v0);
    fp2_add(c2, c2, v1);
    fp2_sub(c2, c2, v2);
    e->x = c2;
    e->y = c1;
    e->z = c0;
}
GSV_DI void fp6_sqr(fp6& e, const fp6& a) { fp6_sqr_p(&e, &a); }
// gfp6.go:172-213
GSV_DI void fp6_inv(fp6& e, const fp6& a) {
    fp2 t1, A, B, C, F;
    fp2_mul(t1, a.x, a.y);
    fp2_mul_xi(t1, t1);
    fp2_sqr(A, a.z);
    fp2_sub(A, A, t1);
    fp2_sqr(B, a.x);
    fp2_mul_xi(B, B);
    fp2_mul(t1, a.y, a.z);
    fp2_sub(B, B, t1);
    fp2_sqr(C, a.y);
    fp2_mul(t1, a.x, a.z);
    fp2_sub(C, C, t1);
    fp2_mul(F, C, a.y);
    fp2_mul_xi(F, F);
    fp2_mul(t1, A, a.z);
    fp2_add(F, F, t1);
    fp2_mul(t1, B, a.x);
    fp2_mul_xi(t1, t1);
    fp2_add(F, F, t1);
    fp2_inv(F, F);
    fp2_mul(e.x, C, F);
    fp2_mul(e.y, B, F);
    fp2_mul(e.z, A, F);
}

}  // namespace bn
}  // namespace gsv

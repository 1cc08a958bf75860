/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle (restatement) of the reference's BN254 pairing check,
 * as driven by the bn256Pairing precompile.  Never linked into the product library.
 *
 * Restates, operation for operation, the cloudflare implementation the reference builds on
 * amd64/arm64 (crypto/bn256/bn256_fast.go):
 *   crypto/bn256/cloudflare/constants.go        p, np, R^2, R^3, Frobenius constants
 *   crypto/bn256/cloudflare/gfp.go:10-81        gfP Montgomery form (R = 2^256), Unmarshal (reject >= p)
 *   crypto/bn256/cloudflare/gfp_generic.go      gfpAdd/Sub/Neg/Mul (Montgomery, canonical results)
 *   crypto/bn256/cloudflare/gfp2.go             F_p^2 = F_p[i]/(i^2+1), value x*i + y
 *   crypto/bn256/cloudflare/gfp6.go             F_p^6 = F_p^2[tau]/(tau^3 - xi), xi = i + 9
 *   crypto/bn256/cloudflare/gfp12.go            F_p^12 = F_p^6[omega]/(omega^2 - tau)
 *   crypto/bn256/cloudflare/curve.go:39-52      G1 IsOnCurve (y^2 = x^3 + 3)
 *   crypto/bn256/cloudflare/twist.go:47-63      G2 IsOnCurve + Order*Q == infinity (subgroup check)
 *   crypto/bn256/cloudflare/twist.go:73-186     twist Add (add-2007-bl), Double (dbl-2009-l), Mul
 *   crypto/bn256/cloudflare/optate.go:3-210     line functions, mulLine, NAF(6u+2) Miller loop
 *   crypto/bn256/cloudflare/optate.go:212-261   final exponentiation
 *   crypto/bn256/cloudflare/bn256.go:120-164    G1.Unmarshal, :256-306 G2.Unmarshal, :313-327 PairingCheck
 *   core/vm/contracts.go:333-360                precompile input layout / errBadPairingInput
 *
 * Every F_p result is canonical (fully reduced Montgomery residue), so these values are
 * bit-identical to the reference's at every step, not only in the final verdict.
 */
#include <stdint.h>
#include <string.h>

#include "gsv_oracle.h"

typedef unsigned __int128 u128;

typedef struct { uint64_t v[4]; } fp;
typedef struct { fp x, y; } fp2;          /* x*i + y */
typedef struct { fp2 x, y, z; } fp6;      /* x*tau^2 + y*tau + z */
typedef struct { fp6 x, y; } fp12;        /* x*omega + y */
typedef struct { fp x, y, z, t; } g1p;    /* Jacobian, t = z^2 when valid (curve.go:9-11) */
typedef struct { fp2 x, y, z, t; } g2p;   /* twist.go:9-13 */

/* ---------------------------------------------------------------- constants (constants.go) */
static const uint64_t P[4] = {0x3c208c16d87cfd47ULL, 0x97816a916871ca8dULL, 0xb85045b68181585dULL,
                              0x30644e72e131a029ULL};
static const uint64_t NP0 = 0x87d20782e4866389ULL; /* low word of np = -p^-1 mod 2^256 */
static const fp R2 = {{0xf32cfc5b538afa89ULL, 0xb5e71911d44501fbULL, 0x47ab1eff0a417ff6ULL,
                       0x06d89f71cab8351fULL}};
static const fp R3 = {{0xb1cd6dafda1530dfULL, 0x62f210e6a7283db6ULL, 0xef7f0b0c0ada0afbULL,
                       0x20fd6e902d592544ULL}};
static const fp RN1 = {{0xed84884a014afa37ULL, 0xeb2022850278edf8ULL, 0xcf63e9cfb74492d9ULL,
                        0x2e67157159e5c639ULL}};
static const fp2 XI_P1_6 = {{{0xa222ae234c492d72ULL, 0xd00f02a4565de15bULL, 0xdc2ff3a253dfc926ULL,
                              0x10a75716b3899551ULL}},
                            {{0xaf9ba69633144907ULL, 0xca6b1d7387afb78aULL, 0x11bded5ef08a2087ULL,
                              0x02f34d751a1f3a7cULL}}};
static const fp2 XI_P1_3 = {{{0x6e849f1ea0aa4757ULL, 0xaa1c7b6d89f89141ULL, 0xb6e713cdfae0ca3aULL,
                              0x26694fbb4e82ebc3ULL}},
                            {{0xb5773b104563ab30ULL, 0x347f91c8a9aa6454ULL, 0x7a007127242e0991ULL,
                              0x1956bcd8118214ecULL}}};
static const fp2 XI_P1_2 = {{{0xa1d77ce45ffe77c7ULL, 0x07affd117826d1dbULL, 0x6d16bd27bb7edc6bULL,
                              0x2c87200285defeccULL}},
                            {{0xe4bbdd0c2936b629ULL, 0xbb30f162e133bacbULL, 0x31a9d1b6f9645366ULL,
                              0x253570bea500f8ddULL}}};
static const fp XI_PSQ1_3 = {{0x3350c88e13e80b9cULL, 0x7dce557cdb5e56b9ULL, 0x6001b4b8b615564aULL,
                              0x2682e617020217e0ULL}};
static const fp XI_2PSQ2_3 = {{0x71930c11d782e155ULL, 0xa6bb947cffbe3323ULL, 0xaa303344d4741444ULL,
                               0x2c3b3f0d26594943ULL}};
static const fp XI_PSQ1_6 = {{0xca8d800500fa1bf2ULL, 0xf0c5d61468b39769ULL, 0x0e201271ad0d4418ULL,
                              0x04290f65bad856e6ULL}};
static const fp2 XI_2P2_3 = {{{0x5dddfd154bd8c949ULL, 0x62cb29a5a4445b60ULL, 0x37bc870a0c7dd2b9ULL,
                               0x24830a9d3171f0fdULL}},
                             {{0x7361d77f843abe92ULL, 0xa5bb2bd3273411fbULL, 0x9c941f314b3e2399ULL,
                               0x15df9cddbb9fd3ecULL}}};
/* twist.go:15-18 twistB = 3/xi (Montgomery) */
static const fp2 TWIST_B = {{{0x38e7ecccd1dcff67ULL, 0x65f0b37d93ce0d3eULL, 0xd749d0dd22ac00aaULL,
                              0x0141b9ce4a688d4dULL}},
                            {{0x3bf938e377b802a8ULL, 0x020b1b273633535dULL, 0x26b7edf049755260ULL,
                              0x2514c6324384a86dULL}}};
/* Order (constants.go:20) little-endian words */
static const uint64_t ORDER[4] = {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL,
                                  0x30644e72e131a029ULL};
/* u (constants.go:17) */
static const uint64_t BN_U = 4965661367192848881ULL;
/* sixuPlus2NAF (optate.go:114-118) */
static const int8_t NAF[65] = {0, 0, 0, 1, 0, 1, 0, -1, 0, 0, 1, -1, 0, 0, 1, 0,
                               0, 1, 1, 0, -1, 0, 0, 1, 0, -1, 0, 0, 0, 0, 1, 1,
                               1, 0, 0, -1, 0, 0, 1, 0, 0, 0, 0, 0, -1, 0, 0, 1,
                               1, 0, 0, -1, 0, 0, 0, 1, 1, 0, -1, 0, 0, 1, 0, 1, 1};

/* ---------------------------------------------------------------- F_p (gfp_generic.go) */
static int fp_geq_p(const uint64_t a[4]) {
    for (int i = 3; i >= 0; i--) {
        if (a[i] > P[i]) return 1;
        if (a[i] < P[i]) return 0;
    }
    return 1;
}
static void fp_sub_p(uint64_t a[4]) {
    u128 br = 0;
    for (int i = 0; i < 4; i++) {
        u128 d = (u128)a[i] - P[i] - br;
        a[i] = (uint64_t)d;
        br = (d >> 64) ? 1 : 0;
    }
}
/* gfpCarry: subtract p when the (head:a) value is >= p */
static void fp_carry(fp *a, uint64_t head) {
    if (head || fp_geq_p(a->v)) fp_sub_p(a->v);
}
static void fp_add(fp *c, const fp *a, const fp *b) {
    u128 s = 0;
    fp r;
    for (int i = 0; i < 4; i++) {
        s = (u128)a->v[i] + b->v[i] + (uint64_t)(s >> 64);
        r.v[i] = (uint64_t)s;
    }
    fp_carry(&r, (uint64_t)(s >> 64));
    *c = r;
}
static void fp_neg(fp *c, const fp *a) { /* p - a, then reduce (neg(0) = 0) */
    fp r;
    u128 br = 0;
    for (int i = 0; i < 4; i++) {
        u128 d = (u128)P[i] - a->v[i] - br;
        r.v[i] = (uint64_t)d;
        br = (d >> 64) ? 1 : 0;
    }
    fp_carry(&r, 0);
    *c = r;
}
static void fp_sub(fp *c, const fp *a, const fp *b) { /* a + (p - b), reduce */
    fp t;
    u128 br = 0;
    for (int i = 0; i < 4; i++) {
        u128 d = (u128)P[i] - b->v[i] - br;
        t.v[i] = (uint64_t)d;
        br = (d >> 64) ? 1 : 0;
    }
    fp_add(c, a, &t);
}
/* F_p multiplication counter (algorithmic work per check, reported by bench.py) */
static __thread uint64_t g_fp_muls;
uint64_t oracle_bn256_fp_mul_count(int reset) {
    uint64_t v = g_fp_muls;
    if (reset) g_fp_muls = 0;
    return v;
}
/* Montgomery product a*b*2^-256 mod p (gfpMul), CIOS form, canonical output */
static void fp_mul(fp *c, const fp *a, const fp *b) {
    g_fp_muls++;
    uint64_t t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; i++) {
        u128 acc;
        uint64_t carry = 0;
        for (int j = 0; j < 4; j++) {
            acc = (u128)a->v[j] * b->v[i] + t[j] + carry;
            t[j] = (uint64_t)acc;
            carry = (uint64_t)(acc >> 64);
        }
        acc = (u128)t[4] + carry;
        t[4] = (uint64_t)acc;
        t[5] = (uint64_t)(acc >> 64);
        uint64_t m = t[0] * NP0;
        acc = (u128)m * P[0] + t[0];
        carry = (uint64_t)(acc >> 64);
        for (int j = 1; j < 4; j++) {
            acc = (u128)m * P[j] + t[j] + carry;
            t[j - 1] = (uint64_t)acc;
            carry = (uint64_t)(acc >> 64);
        }
        acc = (u128)t[4] + carry;
        t[3] = (uint64_t)acc;
        t[4] = t[5] + (uint64_t)(acc >> 64);
    }
    fp r = {{t[0], t[1], t[2], t[3]}};
    fp_carry(&r, t[4]);
    *c = r;
}
static int fp_eq(const fp *a, const fp *b) { return memcmp(a, b, sizeof(fp)) == 0; }
static int fp_is_zero(const fp *a) { return (a->v[0] | a->v[1] | a->v[2] | a->v[3]) == 0; }
static void fp_set_int(fp *r, uint64_t x) { /* newGFp(x) (gfp.go:10-20) */
    fp t = {{x, 0, 0, 0}};
    fp_mul(r, &t, &R2);
}
/* gfP.Invert (gfp.go:31-49): a^(p-2) by square-and-multiply over the fixed exponent bits */
static void fp_inv(fp *e, const fp *f) {
    static const uint64_t bits[4] = {0x3c208c16d87cfd45ULL, 0x97816a916871ca8dULL, 0xb85045b68181585dULL,
                                     0x30644e72e131a029ULL};
    fp sum = RN1, power = *f;
    for (int w = 0; w < 4; w++)
        for (int b = 0; b < 64; b++) {
            if ((bits[w] >> b) & 1) fp_mul(&sum, &sum, &power);
            fp_mul(&power, &power, &power);
        }
    fp_mul(e, &sum, &R3);
}
/* gfP.Unmarshal (gfp.go:61-78): big-endian 32 bytes, reject >= p. Returns 0 ok. */
static int fp_unmarshal(fp *e, const uint8_t *in) {
    for (int w = 0; w < 4; w++) {
        uint64_t x = 0;
        for (int b = 0; b < 8; b++) x = (x << 8) | in[8 * w + b];
        e->v[3 - w] = x;
    }
    return fp_geq_p(e->v) ? -1 : 0;
}
static void fp_marshal(uint8_t *out, const fp *e) {
    for (int w = 0; w < 4; w++)
        for (int b = 0; b < 8; b++) out[8 * w + b] = (uint8_t)(e->v[3 - w] >> (56 - 8 * b));
}
static void fp_mont_encode(fp *c, const fp *a) { fp_mul(c, a, &R2); }
static void fp_mont_decode(fp *c, const fp *a) {
    fp one = {{1, 0, 0, 0}};
    fp_mul(c, a, &one);
}

/* ---------------------------------------------------------------- F_p^2 (gfp2.go) */
static void fp2_zero(fp2 *e) { memset(e, 0, sizeof(*e)); }
static void fp2_one(fp2 *e) {
    memset(&e->x, 0, sizeof(fp));
    fp_set_int(&e->y, 1);
}
static int fp2_is_zero(const fp2 *e) { return fp_is_zero(&e->x) && fp_is_zero(&e->y); }
static int fp2_is_one(const fp2 *e) {
    fp one;
    fp_set_int(&one, 1);
    return fp_is_zero(&e->x) && fp_eq(&e->y, &one);
}
static int fp2_eq(const fp2 *a, const fp2 *b) { return fp_eq(&a->x, &b->x) && fp_eq(&a->y, &b->y); }
static void fp2_conj(fp2 *e, const fp2 *a) {
    e->y = a->y;
    fp_neg(&e->x, &a->x);
}
static void fp2_neg(fp2 *e, const fp2 *a) {
    fp_neg(&e->x, &a->x);
    fp_neg(&e->y, &a->y);
}
static void fp2_add(fp2 *e, const fp2 *a, const fp2 *b) {
    fp_add(&e->x, &a->x, &b->x);
    fp_add(&e->y, &a->y, &b->y);
}
static void fp2_sub(fp2 *e, const fp2 *a, const fp2 *b) {
    fp_sub(&e->x, &a->x, &b->x);
    fp_sub(&e->y, &a->y, &b->y);
}
static void fp2_mul(fp2 *e, const fp2 *a, const fp2 *b) { /* gfp2.go:83-98 */
    fp tx, t, ty;
    fp_mul(&tx, &a->x, &b->y);
    fp_mul(&t, &b->x, &a->y);
    fp_add(&tx, &tx, &t);
    fp_mul(&ty, &a->y, &b->y);
    fp_mul(&t, &a->x, &b->x);
    fp_sub(&ty, &ty, &t);
    e->x = tx;
    e->y = ty;
}
static void fp2_mul_scalar(fp2 *e, const fp2 *a, const fp *b) {
    fp_mul(&e->x, &a->x, b);
    fp_mul(&e->y, &a->y, b);
}
static void fp2_mul_xi(fp2 *e, const fp2 *a) { /* gfp2.go:107-128: (9x+y)i + (9y-x) */
    fp tx, ty;
    fp_add(&tx, &a->x, &a->x);
    fp_add(&tx, &tx, &tx);
    fp_add(&tx, &tx, &tx);
    fp_add(&tx, &tx, &a->x);
    fp_add(&tx, &tx, &a->y);
    fp_add(&ty, &a->y, &a->y);
    fp_add(&ty, &ty, &ty);
    fp_add(&ty, &ty, &ty);
    fp_add(&ty, &ty, &a->y);
    fp_sub(&ty, &ty, &a->x);
    e->x = tx;
    e->y = ty;
}
static void fp2_sqr(fp2 *e, const fp2 *a) { /* gfp2.go:130-143 */
    fp tx, ty;
    fp_sub(&tx, &a->y, &a->x);
    fp_add(&ty, &a->x, &a->y);
    fp_mul(&ty, &tx, &ty);
    fp_mul(&tx, &a->x, &a->y);
    fp_add(&tx, &tx, &tx);
    e->x = tx;
    e->y = ty;
}
static void fp2_inv(fp2 *e, const fp2 *a) { /* gfp2.go:145-156 */
    fp t1, t2, inv;
    fp_mul(&t1, &a->x, &a->x);
    fp_mul(&t2, &a->y, &a->y);
    fp_add(&t1, &t1, &t2);
    fp_inv(&inv, &t1);
    fp_neg(&t1, &a->x);
    fp2 r;
    fp_mul(&r.x, &t1, &inv);
    fp_mul(&r.y, &a->y, &inv);
    *e = r;
}

/* ---------------------------------------------------------------- F_p^6 (gfp6.go) */
static void fp6_zero(fp6 *e) { memset(e, 0, sizeof(*e)); }
static void fp6_one(fp6 *e) {
    fp2_zero(&e->x);
    fp2_zero(&e->y);
    fp2_one(&e->z);
}
static int fp6_is_zero(const fp6 *e) { return fp2_is_zero(&e->x) && fp2_is_zero(&e->y) && fp2_is_zero(&e->z); }
static int fp6_is_one(const fp6 *e) { return fp2_is_zero(&e->x) && fp2_is_zero(&e->y) && fp2_is_one(&e->z); }
static void fp6_neg(fp6 *e, const fp6 *a) {
    fp2_neg(&e->x, &a->x);
    fp2_neg(&e->y, &a->y);
    fp2_neg(&e->z, &a->z);
}
static void fp6_add(fp6 *e, const fp6 *a, const fp6 *b) {
    fp2_add(&e->x, &a->x, &b->x);
    fp2_add(&e->y, &a->y, &b->y);
    fp2_add(&e->z, &a->z, &b->z);
}
static void fp6_sub(fp6 *e, const fp6 *a, const fp6 *b) {
    fp2_sub(&e->x, &a->x, &b->x);
    fp2_sub(&e->y, &a->y, &b->y);
    fp2_sub(&e->z, &a->z, &b->z);
}
static void fp6_frob(fp6 *e, const fp6 *a) { /* gfp6.go:54-62 */
    fp6 r;
    fp2_conj(&r.x, &a->x);
    fp2_conj(&r.y, &a->y);
    fp2_conj(&r.z, &a->z);
    fp2_mul(&r.x, &r.x, &XI_2P2_3);
    fp2_mul(&r.y, &r.y, &XI_P1_3);
    *e = r;
}
static void fp6_frob_p2(fp6 *e, const fp6 *a) { /* gfp6.go:65-73 */
    fp6 r;
    fp2_mul_scalar(&r.x, &a->x, &XI_2PSQ2_3);
    fp2_mul_scalar(&r.y, &a->y, &XI_PSQ1_3);
    r.z = a->z;
    *e = r;
}
static void fp6_mul(fp6 *e, const fp6 *a, const fp6 *b) { /* gfp6.go:96-123 */
    fp2 v0, v1, v2, t0, t1, tz, ty, tx;
    fp2_mul(&v0, &a->z, &b->z);
    fp2_mul(&v1, &a->y, &b->y);
    fp2_mul(&v2, &a->x, &b->x);
    fp2_add(&t0, &a->x, &a->y);
    fp2_add(&t1, &b->x, &b->y);
    fp2_mul(&tz, &t0, &t1);
    fp2_sub(&tz, &tz, &v1);
    fp2_sub(&tz, &tz, &v2);
    fp2_mul_xi(&tz, &tz);
    fp2_add(&tz, &tz, &v0);
    fp2_add(&t0, &a->y, &a->z);
    fp2_add(&t1, &b->y, &b->z);
    fp2_mul(&ty, &t0, &t1);
    fp2_mul_xi(&t0, &v2);
    fp2_sub(&ty, &ty, &v0);
    fp2_sub(&ty, &ty, &v1);
    fp2_add(&ty, &ty, &t0);
    fp2_add(&t0, &a->x, &a->z);
    fp2_add(&t1, &b->x, &b->z);
    fp2_mul(&tx, &t0, &t1);
    fp2_sub(&tx, &tx, &v0);
    fp2_add(&tx, &tx, &v1);
    fp2_sub(&tx, &tx, &v2);
    e->x = tx;
    e->y = ty;
    e->z = tz;
}
static void fp6_mul_scalar(fp6 *e, const fp6 *a, const fp2 *b) {
    fp2_mul(&e->x, &a->x, b);
    fp2_mul(&e->y, &a->y, b);
    fp2_mul(&e->z, &a->z, b);
}
static void fp6_mul_gfp(fp6 *e, const fp6 *a, const fp *b) {
    fp2_mul_scalar(&e->x, &a->x, b);
    fp2_mul_scalar(&e->y, &a->y, b);
    fp2_mul_scalar(&e->z, &a->z, b);
}
static void fp6_mul_tau(fp6 *e, const fp6 *a) { /* gfp6.go:140-149: tau(x t^2 + y t + z) = y t^2 + z t + x xi */
    fp2 tz, ty;
    fp2_mul_xi(&tz, &a->x);
    ty = a->y;
    e->y = a->z;
    e->x = ty;
    e->z = tz;
}
static void fp6_sqr(fp6 *e, const fp6 *a) { /* gfp6.go:151-170 */
    fp2 v0, v1, v2, c0, c1, c2, xiv2;
    fp2_sqr(&v0, &a->z);
    fp2_sqr(&v1, &a->y);
    fp2_sqr(&v2, &a->x);
    fp2_add(&c0, &a->x, &a->y);
    fp2_sqr(&c0, &c0);
    fp2_sub(&c0, &c0, &v1);
    fp2_sub(&c0, &c0, &v2);
    fp2_mul_xi(&c0, &c0);
    fp2_add(&c0, &c0, &v0);
    fp2_add(&c1, &a->y, &a->z);
    fp2_sqr(&c1, &c1);
    fp2_sub(&c1, &c1, &v0);
    fp2_sub(&c1, &c1, &v1);
    fp2_mul_xi(&xiv2, &v2);
    fp2_add(&c1, &c1, &xiv2);
    fp2_add(&c2, &a->x, &a->z);
    fp2_sqr(&c2, &c2);
    fp2_sub(&c2, &c2, &v0);
    fp2_add(&c2, &c2, &v1);
    fp2_sub(&c2, &c2, &v2);
    e->x = c2;
    e->y = c1;
    e->z = c0;
}
static void fp6_inv(fp6 *e, const fp6 *a) { /* gfp6.go:172-213 */
    fp2 t1, A, B, C, F;
    fp2_mul(&t1, &a->x, &a->y);
    fp2_mul_xi(&t1, &t1);
    fp2_sqr(&A, &a->z);
    fp2_sub(&A, &A, &t1);
    fp2_sqr(&B, &a->x);
    fp2_mul_xi(&B, &B);
    fp2_mul(&t1, &a->y, &a->z);
    fp2_sub(&B, &B, &t1);
    fp2_sqr(&C, &a->y);
    fp2_mul(&t1, &a->x, &a->z);
    fp2_sub(&C, &C, &t1);
    fp2_mul(&F, &C, &a->y);
    fp2_mul_xi(&F, &F);
    fp2_mul(&t1, &A, &a->z);
    fp2_add(&F, &F, &t1);
    fp2_mul(&t1, &B, &a->x);
    fp2_mul_xi(&t1, &t1);
    fp2_add(&F, &F, &t1);
    fp2_inv(&F, &F);
    fp2_mul(&e->x, &C, &F);
    fp2_mul(&e->y, &B, &F);
    fp2_mul(&e->z, &A, &F);
}

/* ---------------------------------------------------------------- F_p^12 (gfp12.go) */
static void fp12_one(fp12 *e) {
    fp6_zero(&e->x);
    fp6_one(&e->y);
}
static int fp12_is_one(const fp12 *e) { return fp6_is_zero(&e->x) && fp6_is_one(&e->y); }
static void fp12_conj(fp12 *e, const fp12 *a) {
    fp6_neg(&e->x, &a->x);
    e->y = a->y;
}
static void fp12_frob(fp12 *e, const fp12 *a) { /* gfp12.go:60-66 */
    fp12 r;
    fp6_frob(&r.x, &a->x);
    fp6_frob(&r.y, &a->y);
    fp6_mul_scalar(&r.x, &r.x, &XI_P1_6);
    *e = r;
}
static void fp12_frob_p2(fp12 *e, const fp12 *a) { /* gfp12.go:68-74 */
    fp12 r;
    fp6_frob_p2(&r.x, &a->x);
    fp6_mul_gfp(&r.x, &r.x, &XI_PSQ1_6);
    fp6_frob_p2(&r.y, &a->y);
    *e = r;
}
static void fp12_mul(fp12 *e, const fp12 *a, const fp12 *b) { /* gfp12.go:94-106 */
    fp6 tx, t, ty;
    fp6_mul(&tx, &a->x, &b->y);
    fp6_mul(&t, &b->x, &a->y);
    fp6_add(&tx, &tx, &t);
    fp6_mul(&ty, &a->y, &b->y);
    fp6_mul(&t, &a->x, &b->x);
    fp6_mul_tau(&t, &t);
    e->x = tx;
    fp6_add(&e->y, &ty, &t);
}
static void fp12_sqr(fp12 *e, const fp12 *a) { /* gfp12.go:129-143 */
    fp6 v0, t, ty;
    fp6_mul(&v0, &a->x, &a->y);
    fp6_mul_tau(&t, &a->x);
    fp6_add(&t, &a->y, &t);
    fp6_add(&ty, &a->x, &a->y);
    fp6_mul(&ty, &ty, &t);
    fp6_sub(&ty, &ty, &v0);
    fp6_mul_tau(&t, &v0);
    fp6_sub(&ty, &ty, &t);
    fp6_add(&e->x, &v0, &v0);
    e->y = ty;
}
static void fp12_inv(fp12 *e, const fp12 *a) { /* gfp12.go:145-160 */
    fp6 t1, t2;
    fp6_sqr(&t1, &a->x);
    fp6_sqr(&t2, &a->y);
    fp6_mul_tau(&t1, &t1);
    fp6_sub(&t1, &t2, &t1);
    fp6_inv(&t2, &t1);
    fp12 r;
    fp6_neg(&r.x, &a->x);
    r.y = a->y;
    fp6_mul(&r.x, &r.x, &t2);
    fp6_mul(&r.y, &r.y, &t2);
    *e = r;
}
static void fp12_exp_u(fp12 *c, const fp12 *a) { /* gfp12.go:113-127 with power = u */
    fp12 sum, t;
    fp12_one(&sum);
    for (int i = 63 - __builtin_clzll(BN_U); i >= 0; i--) {
        fp12_sqr(&t, &sum);
        if ((BN_U >> i) & 1) fp12_mul(&sum, &t, a);
        else sum = t;
    }
    *c = sum;
}

/* ---------------------------------------------------------------- G1 (curve.go) */
static void g1_make_affine(g1p *c) { /* curve.go:197-219 */
    fp one;
    fp_set_int(&one, 1);
    if (fp_eq(&c->z, &one)) return;
    if (fp_is_zero(&c->z)) {
        memset(&c->x, 0, sizeof(fp));
        c->y = one;
        memset(&c->t, 0, sizeof(fp));
        return;
    }
    fp zinv, t, zinv2;
    fp_inv(&zinv, &c->z);
    fp_mul(&t, &c->y, &zinv);
    fp_mul(&zinv2, &zinv, &zinv);
    fp_mul(&c->x, &c->x, &zinv2);
    fp_mul(&c->y, &t, &zinv2);
    c->z = one;
    c->t = one;
}
static int g1_on_curve(g1p *c) { /* curve.go:39-52 */
    g1_make_affine(c);
    if (fp_is_zero(&c->z)) return 1;
    fp y2, x3, b;
    fp_set_int(&b, 3);
    fp_mul(&y2, &c->y, &c->y);
    fp_mul(&x3, &c->x, &c->x);
    fp_mul(&x3, &x3, &c->x);
    fp_add(&x3, &x3, &b);
    return fp_eq(&y2, &x3);
}
static void g1_double(g1p *c, const g1p *a) { /* curve.go:143-172 dbl-2009-l */
    fp A, B, C, t, t2, d, e, f;
    fp_mul(&A, &a->x, &a->x);
    fp_mul(&B, &a->y, &a->y);
    fp_mul(&C, &B, &B);
    fp_add(&t, &a->x, &B);
    fp_mul(&t2, &t, &t);
    fp_sub(&t, &t2, &A);
    fp_sub(&t2, &t, &C);
    fp_add(&d, &t2, &t2);
    fp_add(&t, &A, &A);
    fp_add(&e, &t, &A);
    fp_mul(&f, &e, &e);
    g1p r;
    fp_add(&t, &d, &d);
    fp_sub(&r.x, &f, &t);
    fp_add(&t, &C, &C);
    fp_add(&t2, &t, &t);
    fp_add(&t, &t2, &t2);
    fp_sub(&r.y, &d, &r.x);
    fp_mul(&t2, &e, &r.y);
    fp_sub(&r.y, &t2, &t);
    fp_mul(&t, &a->y, &a->z);
    fp_add(&r.z, &t, &t);
    r.t = a->t;
    *c = r;
}
static void g1_add(g1p *c, const g1p *a, const g1p *b) { /* curve.go:63-141 add-2007-bl */
    if (fp_is_zero(&a->z)) { *c = *b; return; }
    if (fp_is_zero(&b->z)) { *c = *a; return; }
    fp z12, z22, u1, u2, t, s1, s2, h, i, j, r, v, t4, t6;
    fp_mul(&z12, &a->z, &a->z);
    fp_mul(&z22, &b->z, &b->z);
    fp_mul(&u1, &a->x, &z22);
    fp_mul(&u2, &b->x, &z12);
    fp_mul(&t, &b->z, &z22);
    fp_mul(&s1, &a->y, &t);
    fp_mul(&t, &a->z, &z12);
    fp_mul(&s2, &b->y, &t);
    fp_sub(&h, &u2, &u1);
    int xeq = fp_is_zero(&h);
    fp_add(&t, &h, &h);
    fp_mul(&i, &t, &t);
    fp_mul(&j, &h, &i);
    fp_sub(&t, &s2, &s1);
    int yeq = fp_is_zero(&t);
    if (xeq && yeq) { g1_double(c, a); return; }
    fp_add(&r, &t, &t);
    fp_mul(&v, &u1, &i);
    g1p o;
    fp_mul(&t4, &r, &r);
    fp_add(&t, &v, &v);
    fp_sub(&t6, &t4, &j);
    fp_sub(&o.x, &t6, &t);
    fp_sub(&t, &v, &o.x);
    fp_mul(&t4, &s1, &j);
    fp_add(&t6, &t4, &t4);
    fp_mul(&t4, &r, &t);
    fp_sub(&o.y, &t4, &t6);
    fp_add(&t, &a->z, &b->z);
    fp_mul(&t4, &t, &t);
    fp_sub(&t, &t4, &z12);
    fp_sub(&t4, &t, &z22);
    fp_mul(&o.z, &t4, &h);
    o.t = a->t;
    *c = o;
}
/* plain double-and-add; same group element as curvePoint.Mul's lattice method (curve.go:174-195) */
static void g1_mul(g1p *c, const g1p *a, const uint8_t k32[32]) {
    g1p sum;
    memset(&sum, 0, sizeof(sum));
    fp_set_int(&sum.y, 1);
    for (int i = 0; i < 256; i++) {
        g1p t;
        g1_double(&t, &sum);
        if ((k32[i >> 3] >> (7 - (i & 7))) & 1) g1_add(&sum, &t, a);
        else sum = t;
    }
    *c = sum;
}

/* ---------------------------------------------------------------- G2 (twist.go) */
static void g2_set_inf(g2p *c) {
    fp2_zero(&c->x);
    fp2_one(&c->y);
    fp2_zero(&c->z);
    fp2_zero(&c->t);
}
static void g2_make_affine(g2p *c) { /* twist.go:178-196 */
    if (fp2_is_one(&c->z)) return;
    if (fp2_is_zero(&c->z)) {
        fp2_zero(&c->x);
        fp2_one(&c->y);
        fp2_zero(&c->t);
        return;
    }
    fp2 zinv, t, zinv2;
    fp2_inv(&zinv, &c->z);
    fp2_mul(&t, &c->y, &zinv);
    fp2_sqr(&zinv2, &zinv);
    fp2_mul(&c->y, &t, &zinv2);
    fp2_mul(&t, &c->x, &zinv2);
    c->x = t;
    fp2_one(&c->z);
    fp2_one(&c->t);
}
static void g2_double(g2p *c, const g2p *a) { /* twist.go:136-162 */
    fp2 A, B, C, t, t2, d, e, f;
    fp2_sqr(&A, &a->x);
    fp2_sqr(&B, &a->y);
    fp2_sqr(&C, &B);
    fp2_add(&t, &a->x, &B);
    fp2_sqr(&t2, &t);
    fp2_sub(&t, &t2, &A);
    fp2_sub(&t2, &t, &C);
    fp2_add(&d, &t2, &t2);
    fp2_add(&t, &A, &A);
    fp2_add(&e, &t, &A);
    fp2_sqr(&f, &e);
    g2p r;
    fp2_add(&t, &d, &d);
    fp2_sub(&r.x, &f, &t);
    fp2_add(&t, &C, &C);
    fp2_add(&t2, &t, &t);
    fp2_add(&t, &t2, &t2);
    fp2_sub(&r.y, &d, &r.x);
    fp2_mul(&t2, &e, &r.y);
    fp2_sub(&r.y, &t2, &t);
    fp2_mul(&t, &a->y, &a->z);
    fp2_add(&r.z, &t, &t);
    r.t = a->t;
    *c = r;
}
static void g2_add(g2p *c, const g2p *a, const g2p *b) { /* twist.go:73-134 */
    if (fp2_is_zero(&a->z)) { *c = *b; return; }
    if (fp2_is_zero(&b->z)) { *c = *a; return; }
    fp2 z12, z22, u1, u2, t, s1, s2, h, i, j, r, v, t4, t6;
    fp2_sqr(&z12, &a->z);
    fp2_sqr(&z22, &b->z);
    fp2_mul(&u1, &a->x, &z22);
    fp2_mul(&u2, &b->x, &z12);
    fp2_mul(&t, &b->z, &z22);
    fp2_mul(&s1, &a->y, &t);
    fp2_mul(&t, &a->z, &z12);
    fp2_mul(&s2, &b->y, &t);
    fp2_sub(&h, &u2, &u1);
    int xeq = fp2_is_zero(&h);
    fp2_add(&t, &h, &h);
    fp2_sqr(&i, &t);
    fp2_mul(&j, &h, &i);
    fp2_sub(&t, &s2, &s1);
    int yeq = fp2_is_zero(&t);
    if (xeq && yeq) { g2_double(c, a); return; }
    fp2_add(&r, &t, &t);
    fp2_mul(&v, &u1, &i);
    g2p o;
    fp2_sqr(&t4, &r);
    fp2_add(&t, &v, &v);
    fp2_sub(&t6, &t4, &j);
    fp2_sub(&o.x, &t6, &t);
    fp2_sub(&t, &v, &o.x);
    fp2_mul(&t4, &s1, &j);
    fp2_add(&t6, &t4, &t4);
    fp2_mul(&t4, &r, &t);
    fp2_sub(&o.y, &t4, &t6);
    fp2_add(&t, &a->z, &b->z);
    fp2_sqr(&t4, &t);
    fp2_sub(&t, &t4, &z12);
    fp2_sub(&t4, &t, &z22);
    fp2_mul(&o.z, &t4, &h);
    o.t = a->t;
    *c = o;
}
/* twist.go:164-176: for i = bitlen .. 0 (one extra leading doubling of the zero point) */
static void g2_mul_words(g2p *c, const g2p *a, const uint64_t k[4]) {
    g2p sum, t;
    memset(&sum, 0, sizeof(sum)); /* zero value: z = 0 -> infinity */
    int bl = 0;
    for (int i = 255; i >= 0; i--)
        if ((k[i >> 6] >> (i & 63)) & 1) { bl = i + 1; break; }
    for (int i = bl; i >= 0; i--) {
        g2_double(&t, &sum);
        int bit = i < 256 ? (int)((k[i >> 6] >> (i & 63)) & 1) : 0;
        if (bit) g2_add(&sum, &t, a);
        else sum = t;
    }
    *c = sum;
}
static int g2_on_curve(g2p *c) { /* twist.go:47-63 */
    g2_make_affine(c);
    if (fp2_is_zero(&c->z)) return 1;
    fp2 y2, x3;
    fp2_sqr(&y2, &c->y);
    fp2_sqr(&x3, &c->x);
    fp2_mul(&x3, &x3, &c->x);
    fp2_add(&x3, &x3, &TWIST_B);
    if (!fp2_eq(&y2, &x3)) return 0;
    g2p cn;
    g2_mul_words(&cn, c, ORDER);
    return fp2_is_zero(&cn.z);
}

/* ---------------------------------------------------------------- Miller loop (optate.go) */
static void line_add(fp2 *a, fp2 *b, fp2 *c, g2p *rout, const g2p *r, const g2p *p, const g1p *q,
                     const fp2 *r2) { /* optate.go:3-50 */
    fp2 B, D, H, I, E, J, L1, V, t, t2;
    fp2_mul(&B, &p->x, &r->t);
    fp2_add(&D, &p->y, &r->z);
    fp2_sqr(&D, &D);
    fp2_sub(&D, &D, r2);
    fp2_sub(&D, &D, &r->t);
    fp2_mul(&D, &D, &r->t);
    fp2_sub(&H, &B, &r->x);
    fp2_sqr(&I, &H);
    fp2_add(&E, &I, &I);
    fp2_add(&E, &E, &E);
    fp2_mul(&J, &H, &E);
    fp2_sub(&L1, &D, &r->y);
    fp2_sub(&L1, &L1, &r->y);
    fp2_mul(&V, &r->x, &E);
    g2p o;
    fp2_sqr(&o.x, &L1);
    fp2_sub(&o.x, &o.x, &J);
    fp2_sub(&o.x, &o.x, &V);
    fp2_sub(&o.x, &o.x, &V);
    fp2_add(&o.z, &r->z, &H);
    fp2_sqr(&o.z, &o.z);
    fp2_sub(&o.z, &o.z, &r->t);
    fp2_sub(&o.z, &o.z, &I);
    fp2_sub(&t, &V, &o.x);
    fp2_mul(&t, &t, &L1);
    fp2_mul(&t2, &r->y, &J);
    fp2_add(&t2, &t2, &t2);
    fp2_sub(&o.y, &t, &t2);
    fp2_sqr(&o.t, &o.z);
    fp2_add(&t, &p->y, &o.z);
    fp2_sqr(&t, &t);
    fp2_sub(&t, &t, r2);
    fp2_sub(&t, &t, &o.t);
    fp2_mul(&t2, &L1, &p->x);
    fp2_add(&t2, &t2, &t2);
    fp2_sub(a, &t2, &t);
    fp2_mul_scalar(c, &o.z, &q->y);
    fp2_add(c, c, c);
    fp2_neg(b, &L1);
    fp2_mul_scalar(b, b, &q->x);
    fp2_add(b, b, b);
    *rout = o;
}
static void line_double(fp2 *a, fp2 *b, fp2 *c, g2p *rout, const g2p *r, const g1p *q) { /* optate.go:52-92 */
    fp2 A, B, C, D, E, G, t;
    fp2_sqr(&A, &r->x);
    fp2_sqr(&B, &r->y);
    fp2_sqr(&C, &B);
    fp2_add(&D, &r->x, &B);
    fp2_sqr(&D, &D);
    fp2_sub(&D, &D, &A);
    fp2_sub(&D, &D, &C);
    fp2_add(&D, &D, &D);
    fp2_add(&E, &A, &A);
    fp2_add(&E, &E, &A);
    fp2_sqr(&G, &E);
    g2p o;
    fp2_sub(&o.x, &G, &D);
    fp2_sub(&o.x, &o.x, &D);
    fp2_add(&o.z, &r->y, &r->z);
    fp2_sqr(&o.z, &o.z);
    fp2_sub(&o.z, &o.z, &B);
    fp2_sub(&o.z, &o.z, &r->t);
    fp2_sub(&o.y, &D, &o.x);
    fp2_mul(&o.y, &o.y, &E);
    fp2_add(&t, &C, &C);
    fp2_add(&t, &t, &t);
    fp2_add(&t, &t, &t);
    fp2_sub(&o.y, &o.y, &t);
    fp2_sqr(&o.t, &o.z);
    fp2_mul(&t, &E, &r->t);
    fp2_add(&t, &t, &t);
    fp2_neg(b, &t);
    fp2_mul_scalar(b, b, &q->x);
    fp2_add(a, &r->x, &E);
    fp2_sqr(a, a);
    fp2_sub(a, a, &A);
    fp2_sub(a, a, &G);
    fp2_add(&t, &B, &B);
    fp2_add(&t, &t, &t);
    fp2_sub(a, a, &t);
    fp2_mul(c, &o.z, &r->t);
    fp2_add(c, c, c);
    fp2_mul_scalar(c, c, &q->y);
    *rout = o;
}
static void mul_line(fp12 *ret, const fp2 *a, const fp2 *b, const fp2 *c) { /* optate.go:94-112 */
    fp6 a2, t3, t2;
    fp2 t;
    fp2_zero(&a2.x);
    a2.y = *a;
    a2.z = *b;
    fp6_mul(&a2, &a2, &ret->x);
    fp6_mul_scalar(&t3, &ret->y, c);
    fp2_add(&t, b, c);
    fp2_zero(&t2.x);
    t2.y = *a;
    t2.z = t;
    fp6_add(&ret->x, &ret->x, &ret->y);
    ret->y = t3;
    fp6_mul(&ret->x, &ret->x, &t2);
    fp6_sub(&ret->x, &ret->x, &a2);
    fp6_sub(&ret->x, &ret->x, &ret->y);
    fp6_mul_tau(&a2, &a2);
    fp6_add(&ret->y, &ret->y, &a2);
}
/* miller(q, p) with q, p already affine (bn256.go:313-327 passes Unmarshal'ed affine points) */
static void miller(fp12 *ret, const g2p *q, const g1p *p) { /* optate.go:122-210 */
    fp12_one(ret);
    g2p A = *q, minusA, r;
    g1p B = *p;
    g2_make_affine(&A);
    g1_make_affine(&B);
    minusA.x = A.x;
    fp2_neg(&minusA.y, &A.y);
    minusA.z = A.z;
    fp2_zero(&minusA.t);
    r = A;
    fp2 r2, a, b, c;
    fp2_sqr(&r2, &A.y);
    for (int i = 64; i > 0; i--) {
        g2p nr;
        line_double(&a, &b, &c, &nr, &r, &B);
        if (i != 64) fp12_sqr(ret, ret);
        mul_line(ret, &a, &b, &c);
        r = nr;
        if (NAF[i - 1] == 1) line_add(&a, &b, &c, &nr, &r, &A, &B, &r2);
        else if (NAF[i - 1] == -1) line_add(&a, &b, &c, &nr, &r, &minusA, &B, &r2);
        else continue;
        mul_line(ret, &a, &b, &c);
        r = nr;
    }
    g2p q1, mq2, nr;
    fp2_conj(&q1.x, &A.x);
    fp2_mul(&q1.x, &q1.x, &XI_P1_3);
    fp2_conj(&q1.y, &A.y);
    fp2_mul(&q1.y, &q1.y, &XI_P1_2);
    fp2_one(&q1.z);
    fp2_one(&q1.t);
    fp2_mul_scalar(&mq2.x, &A.x, &XI_PSQ1_3);
    mq2.y = A.y;
    fp2_one(&mq2.z);
    fp2_one(&mq2.t);
    fp2_sqr(&r2, &q1.y);
    line_add(&a, &b, &c, &nr, &r, &q1, &B, &r2);
    mul_line(ret, &a, &b, &c);
    r = nr;
    fp2_sqr(&r2, &mq2.y);
    line_add(&a, &b, &c, &nr, &r, &mq2, &B, &r2);
    mul_line(ret, &a, &b, &c);
}
static void final_exp(fp12 *out, const fp12 *in) { /* optate.go:212-261 */
    fp12 t1, inv, t2, fp, fp2_, fp3, fu, fu2, fu3, y0, y1, y2, y3, y4, y5, y6, fu2p, fu3p, t0;
    fp6_neg(&t1.x, &in->x);
    t1.y = in->y;
    fp12_inv(&inv, in);
    fp12_mul(&t1, &t1, &inv);
    fp12_frob_p2(&t2, &t1);
    fp12_mul(&t1, &t1, &t2);
    fp12_frob(&fp, &t1);
    fp12_frob_p2(&fp2_, &t1);
    fp12_frob(&fp3, &fp2_);
    fp12_exp_u(&fu, &t1);
    fp12_exp_u(&fu2, &fu);
    fp12_exp_u(&fu3, &fu2);
    fp12_frob(&y3, &fu);
    fp12_frob(&fu2p, &fu2);
    fp12_frob(&fu3p, &fu3);
    fp12_frob_p2(&y2, &fu2);
    fp12_mul(&y0, &fp, &fp2_);
    fp12_mul(&y0, &y0, &fp3);
    fp12_conj(&y1, &t1);
    fp12_conj(&y5, &fu2);
    fp12_conj(&y3, &y3);
    fp12_mul(&y4, &fu, &fu2p);
    fp12_conj(&y4, &y4);
    fp12_mul(&y6, &fu3, &fu3p);
    fp12_conj(&y6, &y6);
    fp12_sqr(&t0, &y6);
    fp12_mul(&t0, &t0, &y4);
    fp12_mul(&t0, &t0, &y5);
    fp12_mul(&t1, &y3, &y5);
    fp12_mul(&t1, &t1, &t0);
    fp12_mul(&t0, &t0, &y2);
    fp12_sqr(&t1, &t1);
    fp12_mul(&t1, &t1, &t0);
    fp12_sqr(&t1, &t1);
    fp12_mul(&t0, &t1, &y1);
    fp12_mul(&t1, &t1, &y0);
    fp12_sqr(&t0, &t0);
    fp12_mul(&t0, &t0, &t1);
    *out = t0;
}

/* ---------------------------------------------------------------- decoding (bn256.go) */
/* G1.Unmarshal (bn256.go:120-164): 0 ok, -1 error */
static int g1_unmarshal(g1p *e, const uint8_t *m) {
    memset(e, 0, sizeof(*e));
    if (fp_unmarshal(&e->x, m) || fp_unmarshal(&e->y, m + 32)) return -1;
    fp_mont_encode(&e->x, &e->x);
    fp_mont_encode(&e->y, &e->y);
    if (fp_is_zero(&e->x) && fp_is_zero(&e->y)) {
        fp_set_int(&e->y, 1);
        memset(&e->z, 0, sizeof(fp));
        memset(&e->t, 0, sizeof(fp));
    } else {
        fp_set_int(&e->z, 1);
        fp_set_int(&e->t, 1);
        if (!g1_on_curve(e)) return -1;
    }
    return 0;
}
/* G2.Unmarshal (bn256.go:256-306): x.x (imaginary), x.y, y.x, y.y */
static int g2_unmarshal(g2p *e, const uint8_t *m) {
    memset(e, 0, sizeof(*e));
    if (fp_unmarshal(&e->x.x, m) || fp_unmarshal(&e->x.y, m + 32) || fp_unmarshal(&e->y.x, m + 64) ||
        fp_unmarshal(&e->y.y, m + 96))
        return -1;
    fp_mont_encode(&e->x.x, &e->x.x);
    fp_mont_encode(&e->x.y, &e->x.y);
    fp_mont_encode(&e->y.x, &e->y.x);
    fp_mont_encode(&e->y.y, &e->y.y);
    if (fp2_is_zero(&e->x) && fp2_is_zero(&e->y)) {
        g2_set_inf(e);
    } else {
        fp2_one(&e->z);
        fp2_one(&e->t);
        if (!g2_on_curve(e)) return -1;
    }
    return 0;
}
static void g1_marshal(uint8_t out[64], g1p *e) { /* bn256.go:96-116 */
    g1_make_affine(e);
    memset(out, 0, 64);
    if (fp_is_zero(&e->z)) return;
    fp t;
    fp_mont_decode(&t, &e->x);
    fp_marshal(out, &t);
    fp_mont_decode(&t, &e->y);
    fp_marshal(out + 32, &t);
}
static void g2_marshal(uint8_t out[128], g2p *e) { /* bn256.go:226-252 */
    g2_make_affine(e);
    memset(out, 0, 128);
    if (fp2_is_zero(&e->z)) return;
    fp t;
    fp_mont_decode(&t, &e->x.x);
    fp_marshal(out, &t);
    fp_mont_decode(&t, &e->x.y);
    fp_marshal(out + 32, &t);
    fp_mont_decode(&t, &e->y.x);
    fp_marshal(out + 64, &t);
    fp_mont_decode(&t, &e->y.y);
    fp_marshal(out + 96, &t);
}

/* ---------------------------------------------------------------- exported */
/* bn256Pairing.Run (core/vm/contracts.go:333-360) + PairingCheck (bn256.go:313-327):
 * returns 1 (true32Byte), 0 (false32Byte) or -1 (error: bad size / malformed point). */
int oracle_bn256_pairing_check(const uint8_t *in, size_t len) {
    if (len % 192) return -1;
    fp12 acc;
    fp12_one(&acc);
    for (size_t i = 0; i < len; i += 192) {
        g1p a;
        g2p b;
        if (g1_unmarshal(&a, in + i)) return -1;
        if (g2_unmarshal(&b, in + i + 64)) return -1;
        if (fp_is_zero(&a.z) || fp2_is_zero(&b.z)) continue;
        fp12 m;
        miller(&m, &b, &a);
        fp12_mul(&acc, &acc, &m);
    }
    fp12 r;
    final_exp(&r, &acc);
    return fp12_is_one(&r) ? 1 : 0;
}

/* debugging/cross-check helpers: F_p^12 values as 12 x 4 little-endian Montgomery words
 * in the order x.x.x, x.x.y, x.y.x, x.y.y, x.z.x, x.z.y, y.x.x, ... (384 bytes) */
static void fp12_store(uint8_t *out, const fp12 *e) { memcpy(out, e, sizeof(fp12)); }
int oracle_bn256_miller(const uint8_t in192[192], uint8_t out384[384]) {
    g1p a;
    g2p b;
    if (g1_unmarshal(&a, in192) || g2_unmarshal(&b, in192 + 64)) return -1;
    fp12 m;
    if (fp_is_zero(&a.z) || fp2_is_zero(&b.z)) fp12_one(&m);
    else miller(&m, &b, &a);
    fp12_store(out384, &m);
    return 0;
}
int oracle_bn256_final_exp(const uint8_t in384[384], uint8_t out384[384]) {
    fp12 a, r;
    memcpy(&a, in384, sizeof(fp12));
    final_exp(&r, &a);
    fp12_store(out384, &r);
    return fp12_is_one(&r);
}
/* G1 / G2 scalar multiplication in the precompile encoding (test-data generation).
 * in == NULL uses the generator (curve.go:16-21, twist.go:20-32). Returns -1 on bad input. */
int oracle_bn256_g1_mul(uint8_t out64[64], const uint8_t *in64, const uint8_t k32[32]) {
    g1p a;
    if (in64) {
        if (g1_unmarshal(&a, in64)) return -1;
    } else {
        fp_set_int(&a.x, 1);
        fp_set_int(&a.y, 2);
        fp_set_int(&a.z, 1);
        fp_set_int(&a.t, 1);
    }
    g1p r;
    g1_mul(&r, &a, k32);
    g1_marshal(out64, &r);
    return 0;
}
int oracle_bn256_g2_mul(uint8_t out128[128], const uint8_t *in128, const uint8_t k32[32]) {
    static const g2p GEN = {
        {{{0xafb4737da84c6140ULL, 0x6043dd5a5802d8c4ULL, 0x09e950fc52a02f86ULL, 0x14fef0833aea7b6bULL}},
         {{0x8e83b5d102bc2026ULL, 0xdceb1935497b0172ULL, 0xfbb8264797811adfULL, 0x19573841af96503bULL}}},
        {{{0x64095b56c71856eeULL, 0xdc57f922327d3cbbULL, 0x55f935be33351076ULL, 0x0da4a0e693fd6482ULL}},
         {{0x619dfa9d886be9f6ULL, 0xfe7fd297f59e9b78ULL, 0xff9e1a62231b7dfeULL, 0x28fd7eebae9e4206ULL}}},
        {{{0}}, {{0}}},
        {{{0}}, {{0}}}};
    g2p a;
    if (in128) {
        if (g2_unmarshal(&a, in128)) return -1;
    } else {
        a = GEN;
        fp2_one(&a.z);
        fp2_one(&a.t);
    }
    uint64_t k[4];
    for (int w = 0; w < 4; w++) {
        uint64_t x = 0;
        for (int b = 0; b < 8; b++) x = (x << 8) | k32[8 * w + b];
        k[3 - w] = x;
    }
    g2p r;
    g2_mul_words(&r, &a, k);
    g2_marshal(out128, &r);
    return 0;
}
/* G2 decode + checks alone: 0 ok (incl. infinity), -1 bad (range / off-twist / not in G2) */
int oracle_bn256_g2_check(const uint8_t in128[128]) {
    g2p b;
    return g2_unmarshal(&b, in128);
}

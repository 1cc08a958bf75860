/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle (restatement) for the collation-validation hot path.
 * See gsv_oracle.h.  Plain, obviously-correct C: 4x64-bit limbs with __int128, textbook
 * Jacobian group law, recursive Merkle-Patricia trie.  Speed is not a goal; only
 * tests/, __graft_entry__.smoke() and bench.py (cpu_baseline "port") call it.
 */
#include "gsv_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ===================================================================================
 * Keccak-256  (crypto/sha3/keccakf.go:10 round constants, :39 keccakF1600;
 *              crypto/sha3/sha3.go:98-157 absorb/padAndPermute; hashes.go:16 rate 136,
 *              dsbyte 0x01 = pre-FIPS Keccak padding)
 * =================================================================================== */
static const uint64_t KRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static const int KROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                             25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

static inline uint64_t rol64(uint64_t x, int r) { return r ? (x << r) | (x >> (64 - r)) : x; }

void oracle_keccakf1600(uint64_t a[25]) {
    for (int round = 0; round < 24; round++) {
        uint64_t c[5], d[5], b[25];
        for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
        for (int x = 0; x < 5; x++) d[x] = c[(x + 4) % 5] ^ rol64(c[(x + 1) % 5], 1);
        for (int i = 0; i < 25; i++) a[i] ^= d[i % 5];
        /* rho + pi: B[y][2x+3y] = rot(A[x][y], r[x][y]) with lane index x + 5y */
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++) {
                int src = x + 5 * y;
                int dx = y, dy = (2 * x + 3 * y) % 5;
                b[dx + 5 * dy] = rol64(a[src], KROT[src]);
            }
        for (int y = 0; y < 5; y++)
            for (int x = 0; x < 5; x++)
                a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
        a[0] ^= KRC[round];
    }
}

static inline uint64_t le64(const uint8_t *p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
    return v;
}

void oracle_keccak256(const uint8_t *in, size_t len, uint8_t out[32]) {
    uint64_t st[25] = {0};
    const size_t rate = 136;
    while (len >= rate) {
        for (int i = 0; i < 17; i++) st[i] ^= le64(in + 8 * i);
        oracle_keccakf1600(st);
        in += rate;
        len -= rate;
    }
    uint8_t blk[136] = {0};
    memcpy(blk, in, len);
    blk[len] ^= 0x01;
    blk[rate - 1] ^= 0x80;
    for (int i = 0; i < 17; i++) st[i] ^= le64(blk + 8 * i);
    oracle_keccakf1600(st);
    for (int i = 0; i < 32; i++) out[i] = (uint8_t)(st[i / 8] >> (8 * (i % 8)));
}

/* Generic sponge (rate bytes, domain byte) — used only to pin the permutation against the
 * reference's SHA3-256 KATs (crypto/sha3/testdata/keccakKats.json.deflate, dsbyte 0x06). */
void oracle_keccak_sponge(const uint8_t *in, size_t len, int rate, uint8_t dsbyte, uint8_t *out,
                          size_t outlen) {
    uint64_t st[25] = {0};
    uint8_t blk[200];
    while (len >= (size_t)rate) {
        memset(blk, 0, sizeof blk);
        memcpy(blk, in, rate);
        for (int i = 0; i < rate / 8; i++) st[i] ^= le64(blk + 8 * i);
        oracle_keccakf1600(st);
        in += rate;
        len -= rate;
    }
    memset(blk, 0, sizeof blk);
    memcpy(blk, in, len);
    blk[len] ^= dsbyte;
    blk[rate - 1] ^= 0x80;
    for (int i = 0; i < rate / 8; i++) st[i] ^= le64(blk + 8 * i);
    oracle_keccakf1600(st);
    for (size_t i = 0; i < outlen; i++) out[i] = (uint8_t)(st[i / 8] >> (8 * (i % 8)));
}

void oracle_keccak256_batch(const uint8_t *data, const uint64_t *off, long n, uint8_t *out32) {
    for (long i = 0; i < n; i++) oracle_keccak256(data + off[i], off[i + 1] - off[i], out32 + 32 * i);
}

/* ===================================================================================
 * 256-bit modular arithmetic for secp256k1 (p and the group order n).
 * Values are 4x64 little-endian limbs.  Both moduli have the form 2^256 - c, so a
 * 512-bit product reduces by repeatedly folding hi*2^256 -> hi*c.
 * =================================================================================== */
typedef struct { uint64_t v[4]; } u256;

static const u256 SECP_P = {{0xFFFFFFFEFFFFFC2FULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL,
                             0xFFFFFFFFFFFFFFFFULL}};
static const u256 SECP_N = {{0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL,
                             0xFFFFFFFFFFFFFFFFULL}};
static const uint64_t C_P[3] = {0x1000003D1ULL, 0, 0};
static const uint64_t C_N[3] = {0x402DA1732FC9BEBFULL, 0x4551231950B75FC4ULL, 1};

static int u256_cmp(const u256 *a, const u256 *b) {
    for (int i = 3; i >= 0; i--) {
        if (a->v[i] < b->v[i]) return -1;
        if (a->v[i] > b->v[i]) return 1;
    }
    return 0;
}
static int u256_is_zero(const u256 *a) { return !(a->v[0] | a->v[1] | a->v[2] | a->v[3]); }
static uint64_t u256_add(u256 *r, const u256 *a, const u256 *b) {
    u128 c = 0;
    for (int i = 0; i < 4; i++) {
        c += (u128)a->v[i] + b->v[i];
        r->v[i] = (uint64_t)c;
        c >>= 64;
    }
    return (uint64_t)c;
}
static uint64_t u256_sub(u256 *r, const u256 *a, const u256 *b) {
    uint64_t borrow = 0;
    for (int i = 0; i < 4; i++) {
        u128 t = (u128)a->v[i] - b->v[i] - borrow;
        r->v[i] = (uint64_t)t;
        borrow = (uint64_t)(t >> 64) & 1;
    }
    return borrow;
}
static void u256_from_be(u256 *r, const uint8_t *b) {
    for (int i = 0; i < 4; i++) {
        uint64_t w = 0;
        for (int j = 0; j < 8; j++) w = (w << 8) | b[(3 - i) * 8 + j];
        r->v[i] = w;
    }
}
static void u256_to_be(uint8_t *b, const u256 *a) {
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++) b[(3 - i) * 8 + j] = (uint8_t)(a->v[i] >> (56 - 8 * j));
}

/* t (8 limbs) mod m where m = 2^256 - c */
static void reduce512(u256 *r, const uint64_t t_in[8], const uint64_t c[3], const u256 *m) {
    uint64_t t[8];
    memcpy(t, t_in, sizeof t);
    for (;;) {
        int hi_nz = (t[4] | t[5] | t[6] | t[7]) != 0;
        if (!hi_nz) break;
        uint64_t nt[8] = {t[0], t[1], t[2], t[3], 0, 0, 0, 0};
        for (int i = 0; i < 4; i++) {
            u128 carry = 0;
            for (int j = 0; j < 3; j++) {
                if (i + j >= 8) break;
                carry += (u128)t[4 + i] * c[j] + nt[i + j];
                nt[i + j] = (uint64_t)carry;
                carry >>= 64;
            }
            for (int k = i + 3; k < 8 && carry; k++) {
                carry += nt[k];
                nt[k] = (uint64_t)carry;
                carry >>= 64;
            }
        }
        memcpy(t, nt, sizeof t);
    }
    u256 x = {{t[0], t[1], t[2], t[3]}};
    while (u256_cmp(&x, m) >= 0) u256_sub(&x, &x, m);
    *r = x;
}

static void mod_mul(u256 *r, const u256 *a, const u256 *b, const uint64_t c[3], const u256 *m) {
    uint64_t t[8] = {0};
    for (int i = 0; i < 4; i++) {
        u128 carry = 0;
        for (int j = 0; j < 4; j++) {
            carry += (u128)a->v[i] * b->v[j] + t[i + j];
            t[i + j] = (uint64_t)carry;
            carry >>= 64;
        }
        t[i + 4] = (uint64_t)carry;
    }
    reduce512(r, t, c, m);
}
static void mod_add(u256 *r, const u256 *a, const u256 *b, const u256 *m) {
    uint64_t c = u256_add(r, a, b);
    if (c || u256_cmp(r, m) >= 0) u256_sub(r, r, m);
}
static void mod_sub(u256 *r, const u256 *a, const u256 *b, const u256 *m) {
    if (u256_sub(r, a, b)) u256_add(r, r, m);
}
static void mod_pow(u256 *r, const u256 *a, const u256 *e, const uint64_t c[3], const u256 *m) {
    u256 acc = {{1, 0, 0, 0}};
    for (int i = 255; i >= 0; i--) {
        mod_mul(&acc, &acc, &acc, c, m);
        if ((e->v[i / 64] >> (i % 64)) & 1) mod_mul(&acc, &acc, a, c, m);
    }
    *r = acc;
}

#define FMUL(r, a, b) mod_mul((r), (a), (b), C_P, &SECP_P)
#define FADD(r, a, b) mod_add((r), (a), (b), &SECP_P)
#define FSUB(r, a, b) mod_sub((r), (a), (b), &SECP_P)
#define SMUL(r, a, b) mod_mul((r), (a), (b), C_N, &SECP_N)

static void f_inv(u256 *r, const u256 *a) {
    u256 e = SECP_P;
    e.v[0] -= 2;
    mod_pow(r, a, &e, C_P, &SECP_P);
}
static void s_inv(u256 *r, const u256 *a) {
    u256 e = SECP_N;
    e.v[0] -= 2;
    mod_pow(r, a, &e, C_N, &SECP_N);
}
/* sqrt for p = 3 mod 4: a^((p+1)/4); returns 1 iff a is a square
 * (libsecp256k1/src/field_impl.h:38 secp256k1_fe_sqrt semantics) */
static int f_sqrt(u256 *r, const u256 *a) {
    u256 e = SECP_P, chk;
    u256 one = {{1, 0, 0, 0}};
    u256_add(&e, &e, &one); /* p+1 fits: p+1 < 2^256 */
    for (int i = 0; i < 4; i++) e.v[i] = (e.v[i] >> 2) | (i < 3 ? e.v[i + 1] << 62 : 0);
    mod_pow(r, a, &e, C_P, &SECP_P);
    FMUL(&chk, r, r);
    return u256_cmp(&chk, a) == 0;
}

/* ---- group law: Jacobian coordinates on y^2 = x^3 + 7 ---- */
typedef struct { u256 x, y, z; int inf; } gej;

static void gej_double(gej *r, const gej *a) {
    if (a->inf || u256_is_zero(&a->y)) { r->inf = 1; return; }
    u256 yy, s, m, t, x3, y3, z3, yyyy;
    FMUL(&yy, &a->y, &a->y);
    FMUL(&s, &a->x, &yy);
    FADD(&s, &s, &s);
    FADD(&s, &s, &s);          /* S = 4 X Y^2 */
    FMUL(&m, &a->x, &a->x);
    FADD(&t, &m, &m);
    FADD(&m, &t, &m);          /* M = 3 X^2 */
    FMUL(&x3, &m, &m);
    FSUB(&x3, &x3, &s);
    FSUB(&x3, &x3, &s);        /* X3 = M^2 - 2S */
    FMUL(&yyyy, &yy, &yy);
    FADD(&yyyy, &yyyy, &yyyy);
    FADD(&yyyy, &yyyy, &yyyy);
    FADD(&yyyy, &yyyy, &yyyy); /* 8 Y^4 */
    FSUB(&t, &s, &x3);
    FMUL(&y3, &m, &t);
    FSUB(&y3, &y3, &yyyy);     /* Y3 = M (S - X3) - 8 Y^4 */
    FMUL(&z3, &a->y, &a->z);
    FADD(&z3, &z3, &z3);       /* Z3 = 2 Y Z */
    r->x = x3; r->y = y3; r->z = z3; r->inf = 0;
}

static void gej_add(gej *r, const gej *a, const gej *b) {
    if (a->inf) { *r = *b; return; }
    if (b->inf) { *r = *a; return; }
    u256 z1z1, z2z2, u1, u2, s1, s2, h, rr, hh, hhh, v, t, x3, y3, z3;
    FMUL(&z1z1, &a->z, &a->z);
    FMUL(&z2z2, &b->z, &b->z);
    FMUL(&u1, &a->x, &z2z2);
    FMUL(&u2, &b->x, &z1z1);
    FMUL(&s1, &a->y, &z2z2);
    FMUL(&s1, &s1, &b->z);
    FMUL(&s2, &b->y, &z1z1);
    FMUL(&s2, &s2, &a->z);
    FSUB(&h, &u2, &u1);
    FSUB(&rr, &s2, &s1);
    if (u256_is_zero(&h)) {
        if (u256_is_zero(&rr)) { gej_double(r, a); return; }
        r->inf = 1;
        return;
    }
    FMUL(&hh, &h, &h);
    FMUL(&hhh, &hh, &h);
    FMUL(&v, &u1, &hh);
    FMUL(&x3, &rr, &rr);
    FSUB(&x3, &x3, &hhh);
    FSUB(&x3, &x3, &v);
    FSUB(&x3, &x3, &v);
    FSUB(&t, &v, &x3);
    FMUL(&y3, &rr, &t);
    FMUL(&t, &s1, &hhh);
    FSUB(&y3, &y3, &t);
    FMUL(&z3, &a->z, &b->z);
    FMUL(&z3, &z3, &h);
    r->x = x3; r->y = y3; r->z = z3; r->inf = 0;
}

static void gej_mul(gej *r, const gej *p, const u256 *k) {
    gej acc;
    acc.inf = 1;
    for (int i = 255; i >= 0; i--) {
        gej_double(&acc, &acc);
        if ((k->v[i / 64] >> (i % 64)) & 1) gej_add(&acc, &acc, p);
    }
    *r = acc;
}

static const u256 GX = {{0x59F2815B16F81798ULL, 0x029BFCDB2DCE28D9ULL, 0x55A06295CE870B07ULL,
                         0x79BE667EF9DCBBACULL}};
static const u256 GY = {{0x9C47D08FFB10D4B8ULL, 0xFD17B448A6855419ULL, 0x5DA4FBFC0E1108A8ULL,
                         0x483ADA7726A3C465ULL}};

static void gej_to_affine(u256 *x, u256 *y, const gej *a) {
    u256 zi, zi2, zi3;
    f_inv(&zi, &a->z);
    FMUL(&zi2, &zi, &zi);
    FMUL(&zi3, &zi2, &zi);
    FMUL(x, &a->x, &zi2);
    FMUL(y, &a->y, &zi3);
}

/* ===================================================================================
 * ECDSA public-key recovery.
 *   crypto/secp256k1/ext.h:30-47 secp256k1_ext_ecdsa_recover
 *   libsecp256k1/src/modules/recovery/main_impl.h:38-58  parse_compact (r,s >= n -> fail)
 *   main_impl.h:170-191 secp256k1_ecdsa_recover (m = msg mod n)
 *   main_impl.h:87-121  secp256k1_ecdsa_sig_recover
 *   group_impl.h:216-236 ge_set_xo_var (y parity from recid & 1)
 *   secp256k1.c:165 / eckey_impl.h:36 serialize 0x04 || X || Y
 * Returns 1 ok, 0 recovery failed, -1 recid >= 4 (crypto/secp256k1/secp256.go:171-178).
 * =================================================================================== */
int oracle_ecrecover(uint8_t pub65[65], const uint8_t sig65[65], const uint8_t msg32[32]) {
    int recid = sig65[64];
    if (recid >= 4) return -1;
    u256 r, s, m, x, y, rhs, t, rn, u1, u2;
    u256_from_be(&r, sig65);
    u256_from_be(&s, sig65 + 32);
    if (u256_cmp(&r, &SECP_N) >= 0 || u256_cmp(&s, &SECP_N) >= 0) return 0;
    u256_from_be(&m, msg32);
    if (u256_cmp(&m, &SECP_N) >= 0) u256_sub(&m, &m, &SECP_N);
    if (u256_is_zero(&r) || u256_is_zero(&s)) return 0;
    x = r;
    if (recid & 2) {
        u256 pmn;
        u256_sub(&pmn, &SECP_P, &SECP_N);
        if (u256_cmp(&x, &pmn) >= 0) return 0;
        u256_add(&x, &x, &SECP_N);
    }
    FMUL(&t, &x, &x);
    FMUL(&rhs, &t, &x);
    u256 seven = {{7, 0, 0, 0}};
    FADD(&rhs, &rhs, &seven);
    if (!f_sqrt(&y, &rhs)) return 0;
    if ((int)(y.v[0] & 1) != (recid & 1)) { u256 zero = {{0}}; FSUB(&y, &zero, &y); }
    s_inv(&rn, &r);
    SMUL(&u1, &rn, &m);
    if (!u256_is_zero(&u1)) u256_sub(&u1, &SECP_N, &u1); /* u1 = -m/r */
    SMUL(&u2, &rn, &s);                                  /* u2 = s/r  */
    gej R = {x, y, {{1, 0, 0, 0}}, 0}, G = {GX, GY, {{1, 0, 0, 0}}, 0}, a, b, q;
    gej_mul(&a, &R, &u2);
    gej_mul(&b, &G, &u1);
    gej_add(&q, &a, &b);
    if (q.inf) return 0;
    u256 qx, qy;
    gej_to_affine(&qx, &qy, &q);
    pub65[0] = 4;
    u256_to_be(pub65 + 1, &qx);
    u256_to_be(pub65 + 33, &qy);
    return 1;
}

typedef struct {
    const uint8_t *msg, *sig;
    uint8_t *pub, *status;
    long lo, hi;
} rec_job;

static void *rec_worker(void *arg) {
    rec_job *j = (rec_job *)arg;
    for (long i = j->lo; i < j->hi; i++) {
        int rc = oracle_ecrecover(j->pub + 65 * i, j->sig + 65 * i, j->msg + 32 * i);
        if (rc != 1) memset(j->pub + 65 * i, 0, 65);
        j->status[i] = rc == 1 ? OR_OK : rc == -1 ? OR_INVALID_RECID : OR_RECOVER_FAILED;
    }
    return NULL;
}

void oracle_ecrecover_batch(const uint8_t *msg32, const uint8_t *sig65, long n, uint8_t *pub65,
                            uint8_t *status, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    rec_job jobs[256];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (rec_job){msg32, sig65, pub65, status, n * t / threads, n * (t + 1) / threads};
        pthread_create(&th[t], NULL, rec_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}

/* Key generation / signing: fixture generation only (signing is not on the path). */
int oracle_secp_pubkey(uint8_t pub65[65], const uint8_t seckey[32]) {
    u256 d;
    u256_from_be(&d, seckey);
    if (u256_is_zero(&d) || u256_cmp(&d, &SECP_N) >= 0) return 0;
    gej G = {GX, GY, {{1, 0, 0, 0}}, 0}, q;
    gej_mul(&q, &G, &d);
    u256 x, y;
    gej_to_affine(&x, &y, &q);
    pub65[0] = 4;
    u256_to_be(pub65 + 1, &x);
    u256_to_be(pub65 + 33, &y);
    return 1;
}

/* ECDSA with an explicit nonce k (nonce32 mod n, must be non-zero), low-s normalised,
 * recid per libsecp256k1 ecdsa_impl.h sig_sign semantics. */
int oracle_secp_sign(uint8_t sig65[65], const uint8_t msg32[32], const uint8_t seckey[32],
                     const uint8_t nonce32[32]) {
    u256 d, k, m, r, s, t, kinv, x, y;
    u256_from_be(&d, seckey);
    u256_from_be(&k, nonce32);
    u256_from_be(&m, msg32);
    if (u256_cmp(&m, &SECP_N) >= 0) u256_sub(&m, &m, &SECP_N);
    if (u256_cmp(&k, &SECP_N) >= 0) u256_sub(&k, &k, &SECP_N);
    if (u256_is_zero(&d) || u256_cmp(&d, &SECP_N) >= 0 || u256_is_zero(&k)) return 0;
    gej G = {GX, GY, {{1, 0, 0, 0}}, 0}, q;
    gej_mul(&q, &G, &k);
    gej_to_affine(&x, &y, &q);
    int recid = (int)(y.v[0] & 1);
    r = x;
    if (u256_cmp(&r, &SECP_N) >= 0) { u256_sub(&r, &r, &SECP_N); recid |= 2; }
    SMUL(&t, &r, &d);
    mod_add(&t, &t, &m, &SECP_N);
    s_inv(&kinv, &k);
    SMUL(&s, &kinv, &t);
    if (u256_is_zero(&r) || u256_is_zero(&s)) return 0;
    u256 halfn = SECP_N;
    for (int i = 0; i < 4; i++) halfn.v[i] = (halfn.v[i] >> 1) | (i < 3 ? halfn.v[i + 1] << 63 : 0);
    if (u256_cmp(&s, &halfn) > 0) { u256_sub(&s, &SECP_N, &s); recid ^= 1; }
    u256_to_be(sig65, &r);
    u256_to_be(sig65 + 32, &s);
    sig65[64] = (uint8_t)recid;
    return 1;
}

/* The GPU's synthetic signer (gsv_synth_sign, recover_dev.cuh derive32 / ecdsa_sign) restated for
 * the configs[1] fixture: msg, key, nonce = Keccak256(le64(seed) || le64(i) || "msg"/"key"/"nce") as
 * big-endian numbers, key and nonce reduced mod n (0 -> 1), low-s signature with its recid. */
static void synth_derive(uint8_t out[32], uint64_t seed, uint64_t i, const char *tag) {
    uint8_t in[19];
    for (int b = 0; b < 8; b++) {
        in[b] = (uint8_t)(seed >> (8 * b));
        in[8 + b] = (uint8_t)(i >> (8 * b));
    }
    memcpy(in + 16, tag, 3);
    oracle_keccak256(in, 19, out);
}
static void synth_mod_n(uint8_t v[32]) {
    u256 x;
    u256_from_be(&x, v);
    if (u256_cmp(&x, &SECP_N) >= 0) u256_sub(&x, &x, &SECP_N);
    if (u256_is_zero(&x)) x.v[0] = 1;
    u256_to_be(v, &x);
}
typedef struct { uint64_t seed; long lo, hi; uint8_t *msg, *sig; } synth_job;
static void *synth_worker(void *a) {
    synth_job *j = (synth_job *)a;
    for (long i = j->lo; i < j->hi; i++) {
        uint8_t d[32], k[32];
        synth_derive(j->msg + 32 * i, j->seed, (uint64_t)i, "msg");
        synth_derive(d, j->seed, (uint64_t)i, "key");
        synth_derive(k, j->seed, (uint64_t)i, "nce");
        synth_mod_n(d);
        synth_mod_n(k);
        oracle_secp_sign(j->sig + 65 * i, j->msg + 32 * i, d, k);
    }
    return NULL;
}
void oracle_synth_sign_many(uint64_t seed, long n, uint8_t *msg32, uint8_t *sig65, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    synth_job jobs[256];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (synth_job){seed, n * t / threads, n * (t + 1) / threads, msg32, sig65};
        pthread_create(&th[t], NULL, synth_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}

/* ===================================================================================
 * RLP (rlp/encode.go:390 writeUint, :429 writeBigInt, string/list headers) and a
 * strict decoder for txdata (core/types/transaction.go:55-70; rlp/decode.go canonical
 * rules: no leading-zero integers, single bytes < 0x80 not wrapped, minimal sizes).
 * =================================================================================== */
typedef struct { uint8_t *p; size_t n, cap; } buf_t;
static void buf_put(buf_t *b, const uint8_t *d, size_t n) {
    if (b->n + n > b->cap) {
        size_t nc = (b->cap ? b->cap * 2 : 256);
        while (nc < b->n + n) nc *= 2;
        b->p = (uint8_t *)realloc(b->p, nc);
        b->cap = nc;
    }
    memcpy(b->p + b->n, d, n);
    b->n += n;
}
static void rlp_header(buf_t *b, size_t len, uint8_t base) {
    uint8_t h[9];
    if (len < 56) { h[0] = (uint8_t)(base + len); buf_put(b, h, 1); return; }
    int nb = 0;
    for (size_t t = len; t; t >>= 8) nb++;
    h[0] = (uint8_t)(base + 55 + nb);
    for (int i = 0; i < nb; i++) h[1 + i] = (uint8_t)(len >> (8 * (nb - 1 - i)));
    buf_put(b, h, 1 + nb);
}
static void rlp_string(buf_t *b, const uint8_t *d, size_t n) {
    if (n == 1 && d[0] < 0x80) { buf_put(b, d, 1); return; }
    rlp_header(b, n, 0x80);
    buf_put(b, d, n);
}
/* big-endian integer bytes (possibly with leading zeros) -> minimal string */
static void rlp_uint_be(buf_t *b, const uint8_t *d, size_t n) {
    while (n && d[0] == 0) { d++; n--; }
    rlp_string(b, d, n);
}
static void rlp_u64(buf_t *b, uint64_t v) {
    uint8_t t[8];
    for (int i = 0; i < 8; i++) t[i] = (uint8_t)(v >> (56 - 8 * i));
    rlp_uint_be(b, t, 8);
}

typedef struct { const uint8_t *p; size_t n; int is_list; } rlp_item;

/* parse one item at p[0..len); returns consumed bytes or 0 on error */
static size_t rlp_next(const uint8_t *p, size_t len, rlp_item *it) {
    if (len == 0) return 0;
    uint8_t b0 = p[0];
    if (b0 < 0x80) { it->p = p; it->n = 1; it->is_list = 0; return 1; }
    if (b0 < 0xb8) {
        size_t n = b0 - 0x80;
        if (1 + n > len) return 0;
        if (n == 1 && p[1] < 0x80) return 0; /* non-canonical single byte */
        it->p = p + 1; it->n = n; it->is_list = 0; return 1 + n;
    }
    if (b0 < 0xc0) {
        size_t nb = b0 - 0xb7, n = 0;
        if (1 + nb > len || p[1] == 0) return 0;
        for (size_t i = 0; i < nb; i++) n = (n << 8) | p[1 + i];
        if (n < 56 || 1 + nb + n > len) return 0;
        it->p = p + 1 + nb; it->n = n; it->is_list = 0; return 1 + nb + n;
    }
    if (b0 < 0xf8) {
        size_t n = b0 - 0xc0;
        if (1 + n > len) return 0;
        it->p = p + 1; it->n = n; it->is_list = 1; return 1 + n;
    }
    size_t nb = b0 - 0xf7, n = 0;
    if (1 + nb > len || p[1] == 0) return 0;
    for (size_t i = 0; i < nb; i++) n = (n << 8) | p[1 + i];
    if (n < 56 || 1 + nb + n > len) return 0;
    it->p = p + 1 + nb; it->n = n; it->is_list = 1; return 1 + nb + n;
}

typedef struct {
    uint64_t nonce, gas;
    rlp_item price, to, value, data, v, r, s;
    int has_to;
} txdata_t;

static int rlp_uint_ok(const rlp_item *it, size_t maxlen) {
    if (it->is_list || it->n > maxlen) return 0;
    if (it->n > 0 && it->p[0] == 0) return 0; /* leading zero */
    return 1;
}
static uint64_t rlp_to_u64(const rlp_item *it) {
    uint64_t v = 0;
    for (size_t i = 0; i < it->n; i++) v = (v << 8) | it->p[i];
    return v;
}

/* core/types/transaction.go:55-70 txdata; rlp.DecodeBytes semantics for the list */
static int tx_decode(txdata_t *tx, const uint8_t *rlp, size_t len) {
    rlp_item outer, f[9];
    size_t used = rlp_next(rlp, len, &outer);
    if (!used || used != len || !outer.is_list) return 0;
    const uint8_t *p = outer.p;
    size_t rem = outer.n;
    for (int i = 0; i < 9; i++) {
        size_t u = rlp_next(p, rem, &f[i]);
        if (!u) return 0;
        p += u; rem -= u;
    }
    if (rem) return 0;
    if (!rlp_uint_ok(&f[0], 8) || !rlp_uint_ok(&f[2], 8)) return 0;
    if (!rlp_uint_ok(&f[1], 32 * 8) || !rlp_uint_ok(&f[4], 32 * 8)) return 0;
    if (!rlp_uint_ok(&f[6], 32 * 8) || !rlp_uint_ok(&f[7], 32 * 8) || !rlp_uint_ok(&f[8], 32 * 8))
        return 0;
    if (f[3].is_list || (f[3].n != 0 && f[3].n != 20)) return 0;
    if (f[5].is_list) return 0;
    tx->nonce = rlp_to_u64(&f[0]);
    tx->price = f[1];
    tx->gas = rlp_to_u64(&f[2]);
    tx->to = f[3];
    tx->has_to = f[3].n == 20;
    tx->value = f[4];
    tx->data = f[5];
    tx->v = f[6];
    tx->r = f[7];
    tx->s = f[8];
    return 1;
}

/* Crypto provider of the Sender path.  Default: this restatement.  The CPU baseline swaps in the
 * reference's own Keccak (ethash sha3.c) and libsecp256k1 recovery from oracle/_ref, so the timed
 * configs[0] path is the reference's crypto (>99% of Sender's time) behind this file's RLP. */
static or_keccak_fn g_keccak;
static or_recover_fn g_recover;
void oracle_set_crypto(or_keccak_fn k, or_recover_fn r) {
    g_keccak = k;
    g_recover = r;
}
static void sender_keccak(const uint8_t *in, size_t len, uint8_t out[32]) {
    if (g_keccak) g_keccak(out, in, len);
    else oracle_keccak256(in, len, out);
}
static int sender_recover(uint8_t pub[65], const uint8_t sig[65], const uint8_t h[32]) {
    return g_recover ? g_recover(pub, sig, h) : oracle_ecrecover(pub, sig, h);
}

/* signer_kind: 0 = EIP155Signer(chain_id), 1 = HomesteadSigner, 2 = FrontierSigner
 * EIP155Signer.Hash core/types/transaction_signing.go:155-165; FrontierSigner.Hash :207-216 */
static void tx_sighash(uint8_t out[32], const txdata_t *tx, const uint8_t *cid, size_t cidlen,
                       int eip155) {
    buf_t body = {0}, all = {0};
    rlp_u64(&body, tx->nonce);
    rlp_uint_be(&body, tx->price.p, tx->price.n);
    rlp_u64(&body, tx->gas);
    if (tx->has_to) rlp_string(&body, tx->to.p, 20);
    else rlp_header(&body, 0, 0x80);
    rlp_uint_be(&body, tx->value.p, tx->value.n);
    rlp_string(&body, tx->data.p, tx->data.n);
    if (eip155) {
        rlp_uint_be(&body, cid, cidlen);
        rlp_u64(&body, 0);
        rlp_u64(&body, 0);
    }
    rlp_header(&all, body.n, 0xc0);
    buf_put(&all, body.p, body.n);
    sender_keccak(all.p, all.n, out);
    free(body.p);
    free(all.p);
}

static size_t bitlen_be(const uint8_t *p, size_t n) {
    while (n && p[0] == 0) { p++; n--; }
    if (!n) return 0;
    size_t bits = 8 * (n - 1);
    for (uint8_t b = p[0]; b; b >>= 1) bits++;
    return bits;
}

/* recoverPlain core/types/transaction_signing.go:222-247 + ValidateSignatureValues
 * crypto/crypto.go:181-192 (r,s in [1,n); homestead: s <= n/2; v in {0,1}).  vb is the
 * already-adjusted V (27/28 based) as a non-negative big-endian integer. */
int oracle_recover_plain(uint8_t addr20[20], const uint8_t sighash[32], const uint8_t *r, size_t rlen,
                         const uint8_t *s, size_t slen, const uint8_t *vb, size_t vlen, int homestead) {
    if (bitlen_be(vb, vlen) > 8) return OR_INVALID_SIG;
    uint8_t vbyte = 0;
    for (size_t i = 0; i < vlen; i++) vbyte = vb[i]; /* low byte (value < 256 here) */
    uint8_t V = (uint8_t)(vbyte - 27);
    if (bitlen_be(r, rlen) > 256 || bitlen_be(s, slen) > 256) return OR_INVALID_SIG;
    uint8_t rb[32] = {0}, sb[32] = {0};
    while (rlen > 32) { r++; rlen--; }
    while (slen > 32) { s++; slen--; }
    memcpy(rb + 32 - rlen, r, rlen);
    memcpy(sb + 32 - slen, s, slen);
    u256 R, S, halfn = SECP_N;
    u256_from_be(&R, rb);
    u256_from_be(&S, sb);
    for (int i = 0; i < 4; i++) halfn.v[i] = (halfn.v[i] >> 1) | (i < 3 ? halfn.v[i + 1] << 63 : 0);
    if (u256_is_zero(&R) || u256_is_zero(&S)) return OR_INVALID_SIG;
    if (homestead && u256_cmp(&S, &halfn) > 0) return OR_INVALID_SIG;
    if (u256_cmp(&R, &SECP_N) >= 0 || u256_cmp(&S, &SECP_N) >= 0 || V > 1) return OR_INVALID_SIG;
    uint8_t sig[65], pub[65], h[32];
    memcpy(sig, rb, 32);
    memcpy(sig + 32, sb, 32);
    sig[64] = V;
    if (sender_recover(pub, sig, sighash) != 1) return OR_RECOVER_FAILED;
    sender_keccak(pub + 1, 64, h);
    memcpy(addr20, h + 12, 20);
    return OR_OK;
}

/* big-endian subtraction a - b (both <= 64 bytes); returns 0 if negative */
static int be_sub(uint8_t out[64], const uint8_t *a, size_t an, const uint8_t *b, size_t bn) {
    uint8_t A[64] = {0}, B[64] = {0};
    if (an > 64 || bn > 64) return 0;
    memcpy(A + 64 - an, a, an);
    memcpy(B + 64 - bn, b, bn);
    int borrow = 0;
    for (int i = 63; i >= 0; i--) {
        int d = (int)A[i] - B[i] - borrow;
        borrow = d < 0;
        out[i] = (uint8_t)(d + (borrow ? 256 : 0));
    }
    return !borrow;
}

/* types.Sender with EIP155Signer / HomesteadSigner / FrontierSigner
 * (core/types/transaction_signing.go:127-137, 182-184, 218-220;
 *  isProtectedV core/types/transaction.go:125-133; deriveChainId transaction_signing.go:250-260) */
static int tx_sender_decoded(uint8_t addr20[20], uint8_t sighash_out[32], const txdata_t *tx,
                             const uint8_t *cid, size_t cidlen, int signer_kind) {
    uint8_t h[32];
    if (signer_kind == 0) {
        size_t vbits = bitlen_be(tx->v.p, tx->v.n);
        int protected_ = 1;
        if (vbits <= 8) {
            uint64_t v = rlp_to_u64(&tx->v);
            protected_ = (v != 27 && v != 28);
        }
        if (protected_) {
            /* deriveChainId(V) = (V - 35) / 2 */
            uint8_t t[64], chain[64], want[64] = {0};
            const uint8_t k35 = 35;
            if (vbits <= 64) {
                uint64_t v = rlp_to_u64(&tx->v);
                uint64_t c = (v - 35) / 2; /* uint64 wrap-around exactly as Go does */
                memset(chain, 0, 64);
                for (int i = 0; i < 8; i++) chain[56 + i] = (uint8_t)(c >> (56 - 8 * i));
            } else {
                if (!be_sub(t, tx->v.p, tx->v.n, &k35, 1)) return OR_INVALID_CHAIN_ID;
                int rem = 0;
                for (int i = 0; i < 64; i++) {
                    int cur = rem * 256 + t[i];
                    chain[i] = (uint8_t)(cur / 2);
                    rem = cur % 2;
                }
            }
            if (cidlen > 64) return OR_INVALID_CHAIN_ID;
            memcpy(want + 64 - cidlen, cid, cidlen);
            if (memcmp(chain, want, 64) != 0) return OR_INVALID_CHAIN_ID;
            /* V = tx.V - 2*chainId - 8 */
            uint8_t two_c[64], vv[64];
            int carry = 0;
            for (int i = 63; i >= 0; i--) {
                int d = want[i] * 2 + carry;
                two_c[i] = (uint8_t)d;
                carry = d >> 8;
            }
            uint8_t eight = 8;
            if (!be_sub(t, tx->v.p, tx->v.n, two_c, 64) || !be_sub(vv, t, 64, &eight, 1))
                return OR_INVALID_SIG; /* negative V: BitLen of |V| is tiny but V-27 wraps */
            tx_sighash(h, tx, cid, cidlen, 1);
            if (sighash_out) memcpy(sighash_out, h, 32);
            return oracle_recover_plain(addr20, h, tx->r.p, tx->r.n, tx->s.p, tx->s.n, vv, 64, 1);
        }
        signer_kind = 1; /* unprotected -> HomesteadSigner */
    }
    tx_sighash(h, tx, NULL, 0, 0);
    if (sighash_out) memcpy(sighash_out, h, 32);
    return oracle_recover_plain(addr20, h, tx->r.p, tx->r.n, tx->s.p, tx->s.n, tx->v.p, tx->v.n,
                                signer_kind == 1);
}

int oracle_tx_sender(uint8_t addr20[20], const uint8_t *rlp, size_t len, const uint8_t *cid,
                     size_t cidlen, int signer_kind) {
    txdata_t tx;
    if (!tx_decode(&tx, rlp, len)) return OR_BAD_RLP;
    return tx_sender_decoded(addr20, NULL, &tx, cid, cidlen, signer_kind);
}

/* types.Sender over n RLP txs on `threads` host threads (the configs[0] CPU baseline loop) */
typedef struct {
    const uint8_t *rlp;
    const uint64_t *off;
    long lo, hi;
    const uint8_t *cid;
    size_t cidlen;
    int signer;
    uint8_t *addr, *status;
} sender_job;
static void *sender_worker(void *a) {
    sender_job *j = (sender_job *)a;
    for (long i = j->lo; i < j->hi; i++)
        j->status[i] = (uint8_t)oracle_tx_sender(j->addr + 20 * i, j->rlp + j->off[i], j->off[i + 1] - j->off[i],
                                                 j->cid, j->cidlen, j->signer);
    return NULL;
}
void oracle_tx_sender_many(const uint8_t *rlp, const uint64_t *off, long n, const uint8_t *cid, size_t cidlen,
                           int signer_kind, uint8_t *addr20, uint8_t *status, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    sender_job jobs[256];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (sender_job){rlp, off, n * t / threads, n * (t + 1) / threads, cid, cidlen, signer_kind, addr20,
                               status};
        pthread_create(&th[t], NULL, sender_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}

int oracle_tx_sighash(uint8_t out32[32], const uint8_t *rlp, size_t len, const uint8_t *cid,
                      size_t cidlen, int signer_kind) {
    txdata_t tx;
    if (!tx_decode(&tx, rlp, len)) return OR_BAD_RLP;
    tx_sighash(out32, &tx, cid, cidlen, signer_kind == 0);
    return OR_OK;
}

/* ===================================================================================
 * Merkle-Patricia trie over DeriveSha keys.
 *   core/types/derive_sha.go:32-41  key_i = rlp(uint(i)), value_i = list.GetRlp(i)
 *   sharding/collation.go:210-219   Chunks.GetRlp(i) = rlp(body[i])  (one byte per leaf)
 *   trie/trie.go:200-286            TryUpdate / insert (short + full nodes)
 *   trie/hasher.go:56-212           post-order hash; RLP < 32 bytes inlined (force on root)
 *   trie/encoding.go:37-75          hexToCompact / keybytesToHex
 *   trie/trie.go:471-478            empty trie -> emptyRoot = keccak(0x80)
 * =================================================================================== */
enum { NT_SHORT = 1, NT_FULL = 2, NT_VALUE = 3 };
#define MAXKEY 72
typedef struct mnode mnode;
struct mnode {
    uint8_t type, keylen;
    uint32_t vlen;
    const uint8_t *val;  /* value node bytes (points at vbuf or caller memory) */
    uint8_t vbuf[8];
    uint8_t key[MAXKEY]; /* short: nibble key (may end with terminator 16) */
    mnode *child[17];    /* short: child[0] = val */
};

typedef struct { mnode *blocks[4096]; int nb; int used; } arena_t;
#define ARENA_BLK 65536
static mnode *arena_new(arena_t *a) {
    if (a->nb == 0 || a->used == ARENA_BLK) {
        a->blocks[a->nb++] = (mnode *)calloc(ARENA_BLK, sizeof(mnode));
        a->used = 0;
    }
    return &a->blocks[a->nb - 1][a->used++];
}
static void arena_free(arena_t *a) {
    for (int i = 0; i < a->nb; i++) free(a->blocks[i]);
}

static mnode *mpt_insert(arena_t *A, mnode *n, const uint8_t *key, int klen, mnode *value) {
    if (klen == 0) return value;
    if (!n) {
        mnode *s = arena_new(A);
        s->type = NT_SHORT;
        s->keylen = (uint8_t)klen;
        memcpy(s->key, key, klen);
        s->child[0] = value;
        return s;
    }
    if (n->type == NT_SHORT) {
        int m = 0;
        while (m < klen && m < n->keylen && key[m] == n->key[m]) m++;
        if (m == n->keylen) {
            n->child[0] = mpt_insert(A, n->child[0], key + m, klen - m, value);
            return n;
        }
        mnode *br = arena_new(A);
        br->type = NT_FULL;
        br->child[n->key[m]] = mpt_insert(A, NULL, n->key + m + 1, n->keylen - m - 1, n->child[0]);
        br->child[key[m]] = mpt_insert(A, NULL, key + m + 1, klen - m - 1, value);
        if (m == 0) return br;
        mnode *s = arena_new(A);
        s->type = NT_SHORT;
        s->keylen = (uint8_t)m;
        memcpy(s->key, key, m);
        s->child[0] = br;
        return s;
    }
    if (n->type == NT_FULL) {
        n->child[key[0]] = mpt_insert(A, n->child[key[0]], key + 1, klen - 1, value);
        return n;
    }
    /* value node at a position where a longer key continues: cannot happen for
     * prefix-free key sets; mirror trie.go by replacing (insert on valueNode with len(key)>0
     * panics in the reference; we never reach it for DeriveSha keys). */
    return n;
}

/* encode node n; write its "reference" (raw RLP if < 32 bytes and !force, else 0xa0||hash)
 * into ref/reflen.  Returns the RLP encoding length (for testing). */
static void mpt_ref(const mnode *n, buf_t *out, int force);

static void mpt_encode(const mnode *n, buf_t *enc) {
    buf_t body = {0};
    if (n->type == NT_SHORT) {
        /* hexToCompact */
        uint8_t ck[MAXKEY / 2 + 2];
        int term = n->keylen > 0 && n->key[n->keylen - 1] == 16;
        int hl = n->keylen - term, ci = 1;
        const uint8_t *h = n->key;
        ck[0] = (uint8_t)(term << 5);
        if (hl & 1) { ck[0] |= 0x10 | h[0]; h++; hl--; }
        for (int i = 0; i < hl; i += 2) ck[ci++] = (uint8_t)(h[i] << 4 | h[i + 1]);
        rlp_string(&body, ck, ci);
        const mnode *c = n->child[0];
        if (c->type == NT_VALUE) rlp_string(&body, c->val, c->vlen);
        else mpt_ref(c, &body, 0);
    } else {
        for (int i = 0; i < 16; i++) {
            if (n->child[i]) mpt_ref(n->child[i], &body, 0);
            else rlp_header(&body, 0, 0x80);
        }
        if (n->child[16]) rlp_string(&body, n->child[16]->val, n->child[16]->vlen);
        else rlp_header(&body, 0, 0x80);
    }
    rlp_header(enc, body.n, 0xc0);
    buf_put(enc, body.p, body.n);
    free(body.p);
}

static void mpt_ref(const mnode *n, buf_t *out, int force) {
    buf_t enc = {0};
    mpt_encode(n, &enc);
    if (enc.n < 32 && !force) {
        buf_put(out, enc.p, enc.n);
    } else {
        uint8_t h[33];
        h[0] = 0xa0;
        oracle_keccak256(enc.p, enc.n, h + 1);
        buf_put(out, h, 33);
    }
    free(enc.p);
}

void oracle_derive_sha_bytes(const uint8_t *body, size_t n, uint8_t root[32]) {
    if (n == 0) {
        const uint8_t e = 0x80;
        oracle_keccak256(&e, 1, root);
        return;
    }
    arena_t *A = (arena_t *)calloc(1, sizeof(arena_t));
    mnode *rootn = NULL;
    for (size_t i = 0; i < n; i++) {
        buf_t kb = {0};
        uint8_t nib[MAXKEY];
        rlp_u64(&kb, (uint64_t)i); /* rlp.Encode(keybuf, uint(i)) */
        int kl = 0;
        for (size_t j = 0; j < kb.n; j++) {
            nib[kl++] = kb.p[j] >> 4;
            nib[kl++] = kb.p[j] & 15;
        }
        nib[kl++] = 16;
        free(kb.p);
        mnode *v = arena_new(A);
        v->type = NT_VALUE;
        /* Chunks.GetRlp(i) = rlp.EncodeToBytes(byte) */
        uint8_t b = body[i];
        v->val = v->vbuf;
        if (b == 0) { v->vbuf[0] = 0x80; v->vlen = 1; }
        else if (b < 0x80) { v->vbuf[0] = b; v->vlen = 1; }
        else { v->vbuf[0] = 0x81; v->vbuf[1] = b; v->vlen = 2; }
        rootn = mpt_insert(A, rootn, nib, kl, v);
    }
    buf_t ref = {0};
    mpt_ref(rootn, &ref, 1);
    memcpy(root, ref.p + 1, 32);
    free(ref.p);
    arena_free(A);
    free(A);
}

/* Generic trie root over (key, value) updates in order (trie.Update semantics for
 * non-empty values, trie/trie.go:186-216).  Used to pin the trie restatement against the
 * reference's own golden roots (trie/trie_test.go:154-178). Keys <= 35 bytes. */
int oracle_trie_root(const uint8_t *keys, const uint64_t *koff, const uint8_t *vals,
                     const uint64_t *voff, long n, uint8_t root[32]) {
    arena_t *A = (arena_t *)calloc(1, sizeof(arena_t));
    mnode *rootn = NULL;
    for (long i = 0; i < n; i++) {
        size_t kl = koff[i + 1] - koff[i];
        if (2 * kl + 1 > MAXKEY) { arena_free(A); free(A); return -1; }
        uint8_t nib[MAXKEY];
        for (size_t j = 0; j < kl; j++) {
            nib[2 * j] = keys[koff[i] + j] >> 4;
            nib[2 * j + 1] = keys[koff[i] + j] & 15;
        }
        nib[2 * kl] = 16;
        mnode *v = arena_new(A);
        v->type = NT_VALUE;
        v->val = vals + voff[i];
        v->vlen = (uint32_t)(voff[i + 1] - voff[i]);
        rootn = mpt_insert(A, rootn, nib, (int)(2 * kl + 1), v);
    }
    if (!rootn) {
        const uint8_t e = 0x80;
        oracle_keccak256(&e, 1, root);
    } else {
        buf_t ref = {0};
        mpt_ref(rootn, &ref, 1);
        memcpy(root, ref.p + 1, 32);
        free(ref.p);
    }
    arena_free(A);
    free(A);
    return 0;
}

/* ===================================================================================
 * Blob codec (sharding/utils/marshal.go:71-123 Serialize, :144-198 Deserialize).
 * 32-byte chunks = indicator byte + 31 data bytes; indicator = 0 for non-terminal chunks,
 * terminal length (| 0x80 when skipEvm) for the last chunk of each blob.
 * =================================================================================== */
long oracle_blob_serialize(const uint8_t *data, const uint64_t *off, const uint8_t *skip_evm, long n,
                           uint8_t *out, long cap) {
    long w = 0;
    for (long i = 0; i < n; i++) {
        long len = (long)(off[i + 1] - off[i]);
        const uint8_t *d = data + off[i];
        long chunks = (len + 30) / 31;
        for (long j = 0; j < chunks; j++) {
            long tl = (j != chunks - 1) ? 31 : len - (chunks - 1) * 31;
            uint8_t ind = (j != chunks - 1) ? 0 : (uint8_t)tl;
            if (j == chunks - 1 && skip_evm && skip_evm[i]) ind |= 0x80;
            if (w + 32 > cap) return -1;
            out[w++] = ind;
            memcpy(out + w, d + j * 31, tl);
            w += tl;
            if (tl != 31) {
                long fill = chunks * 31 - len;
                memset(out + w, 0, fill);
                w += fill;
            }
        }
    }
    return w;
}

long oracle_blob_deserialize(const uint8_t *data, size_t len, uint8_t *out, uint64_t *off,
                             uint8_t *skip_evm, long max_blobs) {
    long chunks = (long)(len / 32), nb = 0, parts = 0, cur = 0;
    uint64_t w = 0;
    off[0] = 0;
    /* first pass identifies blobs exactly as the reference (marshal.go:148-171) */
    for (long i = 0; i < chunks; i++) {
        int dl = data[i * 32] & 0x1F;
        if (dl == 0) { parts++; continue; }
        if (nb >= max_blobs) return -1;
        for (long c = 0; c < parts; c++) {
            memcpy(out + w, data + cur + 1, 31);
            w += 31;
            cur += 32;
        }
        skip_evm[nb] = (data[cur] & 0x80) ? 1 : 0;
        memcpy(out + w, data + cur + 1, dl);
        w += dl;
        cur += 32;
        off[++nb] = w;
        parts = 0;
    }
    return nb;
}

// secp256k1 public-key recovery core shared by the ecrecover, sender and notary kernels.
// See ecrecover.hip for the algorithm and the reference semantics it restates.
#pragma once
#include "gsv_internal.h"
#include "keccak_dev.cuh"
#include "secp256k1_dev.cuh"
// the rare p == q doubling of the mixed add runs out of line (see gej9_dbl_ool below)
namespace gsv { struct gej9; __device__ void gej9_dbl_rare(gej9& o, const gej9& p); }
#define GEJ9_DBL_RARE(o, p) gej9_dbl_rare(o, p)
#include "secp256k1_fe9.cuh"
#include "modinv30.cuh"

namespace gsv {

__device__ constexpr uint32_t BETA[8] = {0x719501EEu, 0xC1396C28u, 0x12F58995u, 0x9CF04975u,
                                         0xAC3434E9u, 0x6E64479Eu, 0x657C0710u, 0x7AE96A2Bu};
__device__ constexpr uint32_t MINUS_LAMBDA[8] = {0xB51283CFu, 0xE0CFC810u, 0x8EC739C2u, 0xA880B9FCu,
                                                 0x77ED9BA4u, 0x5AD9E3FDu, 0x3FA3CF1Fu, 0xAC9C52B3u};
__device__ constexpr uint32_t MINUS_B1[8] = {0x0ABFE4C3u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u,
                                             0u, 0u, 0u, 0u};
__device__ constexpr uint32_t MINUS_B2[8] = {0x3DB1562Cu, 0xD765CDA8u, 0x0774346Du, 0x8A280AC5u,
                                             0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
__device__ constexpr uint32_t GLV_G1[8] = {0xEB153DABu, 0x90E49284u, 0x6BCDE86Cu, 0xD221A7D4u,
                                           0x00003086u, 0u, 0u, 0u};
__device__ constexpr uint32_t GLV_G2[8] = {0xE4C42212u, 0x7FA90ABFu, 0x88286F54u, 0x7ED6010Eu,
                                           0x0000E443u, 0u, 0u, 0u};
__device__ constexpr uint32_t GX[8] = {0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu,
                                       0xCE870B07u, 0x55A06295u, 0xF9DCBBACu, 0x79BE667Eu};
__device__ constexpr uint32_t GY[8] = {0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u,
                                       0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u};
__device__ constexpr uint32_t P_MINUS_N[8] = {0x2FC9BAEEu, 0x402DA172u, 0x50B75FC4u, 0x45512319u,
                                              0x00000001u, 0u, 0u, 0u};
__device__ constexpr uint32_t HALF_N[8] = {0x681B20A0u, 0xDFE92F46u, 0x57A4501Du, 0x5D576E73u,
                                           0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu};

// u2 R's GLV halves are recoded into fixed-schedule odd digits of GLV_W bits: digits in
// {+-1, +-3, ..., +-(2^W - 1)}, a table of the 2^(W-1) odd multiples of R, W doublings per digit.
// (w = 5 measured slower, r02-r05: DESIGN.md §7.3)
constexpr int GLV_W = 4;
constexpr int GLV_NT = 1 << (GLV_W - 1);             // table entries
constexpr int GLV_DIGITS = (130 + GLV_W - 1) / GLV_W;  // |k| < 2^130: the split gives < 2^128, + a lattice vector (glv_make_odd) < 2^129.3
// digit code = sign bit above a (W - 1)-bit table index, packed in DIG_SLOT-bit slots
constexpr int DIG_SLOT = GLV_W <= 4 ? 4 : 8;
constexpr int DIG_PER_WORD = 32 / DIG_SLOT;
constexpr int DIG_WORDS = (GLV_DIGITS + DIG_PER_WORD - 1) / DIG_PER_WORD;
static_assert(GLV_W >= 3 && GLV_W <= 5, "GLV window width");
// where the per-lane GLV table lives: entries 0..3 in LDS ([word][256 lanes] per block), the rest in a
// private array (scratch: memory only for resident lanes, served by L1/L2).  Two waves per SIMD leave
// LDS room for 72 words a lane: four entries.  (The whole table private measured 107.2 vs 113.7-114.3 M
// recoveries/s, r05: profiles/r05/ab/ecrecover_options.txt.)
constexpr int GLV_LNT = 4;  // entries in LDS
static_assert(GLV_LNT <= GLV_NT, "LDS holds at most four entries at two waves per SIMD");
// LDS part: 18 GLV_LNT words per lane, lane-minor ([word][GSV_LTAB_STRIDE]); the kernels that call
// recover_core run 256-thread blocks and declare __shared__ uint32_t[GSV_LTAB_WORDS].
constexpr int GSV_LTAB_STRIDE = 256;
constexpr int GSV_LTAB_WORDS = 18 * GLV_LNT * GSV_LTAB_STRIDE;
// Measured and not kept (r02-r05): the lambda half's x coordinates (beta x_e) precomputed per entry in
// a private array (+0.3 %, but 4.6x the fetch bytes: profiles/r02/ab_betatab.txt), the private half
// read one add ahead (112.3-112.8 vs 113.7-114.3 M/s) and the two adds of a digit position as
// straight-line code (equal) (profiles/r05/ab/ecrecover_options.txt).
// waves per SIMD the recovery kernels are compiled for (register budget 512 / waves)
#define GSV_ECR_WAVES 2
#define GSV_LTAB_DECL __shared__ uint32_t ltab[GSV_LTAB_WORDS]
#define GSV_LTAB_LANE (ltab + threadIdx.x)

// ---------------------------------------------------------------------------- scalar helpers
GSV_DI void sc_from_const(sc& r, const uint32_t c[8]) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = c[i];
}

// (k * g) >> 272, rounded (libsecp256k1 scalar_8x32_impl.h mul_shift_var semantics)
GSV_DI void sc_mul_shift272(sc& r, const sc& k, const uint32_t g[8]) {
    GSV_OPC(OPC_SC_MUL);
    uint32_t t[16];
    mul_8x8_fx(t, k.v, g);
#pragma unroll
    for (int i = 0; i < 7; i++) r.v[i] = (t[8 + i] >> 16) | (t[9 + i] << 16);
    r.v[7] = t[15] >> 16;
    uint64_t c = (uint64_t)r.v[0] + ((t[8] >> 15) & 1u);
    r.v[0] = lo32(c);
#pragma unroll
    for (int i = 1; i < 8; i++) {
        c = (uint64_t)r.v[i] + hi32(c);
        r.v[i] = lo32(c);
    }
}

// k = r1 + r2 * lambda (mod n)  (libsecp256k1 scalar_impl.h secp256k1_scalar_split_lambda)
GSV_DI void sc_split_lambda(sc& r1, sc& r2, const sc& k) {
    sc c1, c2, t;
    sc_mul_shift272(c1, k, GLV_G1);
    sc_mul_shift272(c2, k, GLV_G2);
    sc_from_const(t, MINUS_B1);
    sc_mul(c1, c1, t);
    sc_from_const(t, MINUS_B2);
    sc_mul(c2, c2, t);
    sc_add(r2, c1, c2);
    sc_from_const(t, MINUS_LAMBDA);
    sc_mul(r1, r2, t);
    sc_add(r1, r1, k);
}

GSV_DI bool sc_is_high(const sc& a) { return limbs_lt(HALF_N, a.v); }

// Fixed-schedule odd-digit recoding, w = GLV_W: k (odd after skew) = sum d_i 2^(w i) with
// d_i odd in [-(2^w - 1), 2^w - 1].  Digit i packed in a DIG_SLOT-bit slot: bit w - 1 = negative,
// bits 0 .. w - 2 = (|d| - 1) / 2.
GSV_DI void recode_glv(uint32_t dig[DIG_WORDS], uint32_t& skew, const sc& kin) {
    constexpr uint32_t MASK = (2u << GLV_W) - 1u;
    constexpr int32_t OFF = 1 << GLV_W;
    uint32_t k[5] = {kin.v[0], kin.v[1], kin.v[2], kin.v[3], kin.v[4]};
    skew = (k[0] & 1u) ^ 1u;
    // k += skew  (k < 2^129 so no overflow out of 5 limbs)
    uint64_t c = (uint64_t)k[0] + skew;
    k[0] = lo32(c);
#pragma unroll
    for (int i = 1; i < 5; i++) {
        c = (uint64_t)k[i] + hi32(c);
        k[i] = lo32(c);
    }
#pragma unroll
    for (int i = 0; i < DIG_WORDS; i++) dig[i] = 0;
#pragma unroll
    for (int i = 0; i < GLV_DIGITS; i++) {
        int32_t d;
        if (i < GLV_DIGITS - 1) d = (int32_t)(k[0] & MASK) - OFF;
        else d = (int32_t)(k[0] & MASK);
        uint32_t neg = d < 0 ? 1u : 0u;
        uint32_t mag = (uint32_t)(d < 0 ? -d : d);
        uint32_t code = (neg << (GLV_W - 1)) | ((mag - 1u) >> 1);
        dig[i / DIG_PER_WORD] |= code << ((i % DIG_PER_WORD) * DIG_SLOT);
        // k = (k - d) >> w
        int64_t t = (int64_t)k[0] - d;
        uint32_t kk[5];
        kk[0] = (uint32_t)t;
        int64_t carry = t >> 32;
#pragma unroll
        for (int j = 1; j < 5; j++) {
            int64_t u = (int64_t)k[j] + carry;
            kk[j] = (uint32_t)u;
            carry = u >> 32;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) k[j] = (kk[j] >> GLV_W) | (kk[j + 1] << (32 - GLV_W));
        k[4] = kk[4] >> GLV_W;
    }
}

// ---------------------------------------------------------------------------- group helpers
// Field elements are fe9 (secp256k1_fe9.cuh); the magnitude of every intermediate is noted.
GSV_DI void fe9_from_const(fe9& r, const uint32_t c[8]) {
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = c[i];
    fe9_from_words(r, w);
}
GSV_DI void ge9_cmov(ge9& r, const ge9& a, bool f) {
    fe9_cmov(r.x, a.x, f);
    fe9_cmov(r.y, a.y, f);
}

// Doubling for the rare p == q case of the mixed add, out of line so the hot loops stay small
// in I-cache; the point travels in VGPR vectors (an aggregate or pointer argument would pin the
// caller's accumulator to scratch memory).
typedef uint32_t gsv_v32 __attribute__((ext_vector_type(32)));
__device__ __noinline__ gsv_v32 gej9_dbl_ool(gsv_v32 in) {
    gej9 p, d;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        p.x.v[i] = in[i];
        p.y.v[i] = in[9 + i];
        p.z.v[i] = in[18 + i];
    }
    gej9_dbl(d, p);
    gsv_v32 o;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        o[i] = d.x.v[i];
        o[9 + i] = d.y.v[i];
        o[18 + i] = d.z.v[i];
    }
#pragma unroll
    for (int i = 27; i < 32; i++) o[i] = 0;
    return o;
}
__device__ void gej9_dbl_rare(gej9& o, const gej9& p) {
    gsv_v32 in;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        in[i] = p.x.v[i];
        in[9 + i] = p.y.v[i];
        in[18 + i] = p.z.v[i];
    }
#pragma unroll
    for (int i = 27; i < 32; i++) in[i] = 0;
    gsv_v32 d = gej9_dbl_ool(in);
#pragma unroll
    for (int i = 0; i < 9; i++) {
        o.x.v[i] = d[i];
        o.y.v[i] = d[9 + i];
        o.z.v[i] = d[18 + i];
    }
}

GSV_DI void table_select9(ge9& out, const ge9 T[4], uint32_t idx) {
    out = T[0];
#pragma unroll
    for (int e = 1; e < 4; e++) ge9_cmov(out, T[e], idx == (uint32_t)e);
}
GSV_DI void table_select9_x(fe9& out, const fe9 X[4], uint32_t idx) {
    out = X[0];
#pragma unroll
    for (int e = 1; e < 4; e++) fe9_cmov(out, X[e], idx == (uint32_t)e);
}

// comb table entry (w, d) = d * 2^(COMB_BITS w) * G, affine, canonical fe9 limbs: x[9] y[9] + 2 pad words
constexpr int GTAB_ENTRY_U4 = GTAB_ENTRY_BYTES / 16;
GSV_DI void gtab_load(ge9& P, const uint4* e) {
    uint4 a = e[0], b = e[1], c = e[2], d = e[3], f = e[4];
    uint32_t w[20] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w,
                      d.x, d.y, d.z, d.w, f.x, f.y, f.z, f.w};
#pragma unroll
    for (int i = 0; i < 9; i++) {
        P.x.v[i] = w[i];
        P.y.v[i] = w[9 + i];
    }
}

// the scalar shifted right by COMB_BITS in place (8 words; v_alignbit pairs)
GSV_DI void comb_shift(uint32_t c[8]) {
#pragma unroll
    for (int i = 0; i < 7; i++) c[i] = __builtin_amdgcn_alignbit(c[i + 1], c[i], COMB_BITS);
    c[7] >>= COMB_BITS;
}
// u*G with the fixed-base comb table (COMB_WINDOWS mixed adds, no doublings).  The windows' digits are
// read from the bottom of a copy of u shifted by COMB_BITS per window (r05): comb_digit's word select
// with a loop-variant index was turned into a private array written to scratch and read back by a
// dynamic offset twice per window (72 bytes of scratch stores per window, ~0.8 KB per recovery; r04's
// 0.78 GB of writes per 2^20-recovery launch).
GSV_DI void comb_mul_g9(gej9& acc, bool& inf, const sc& u, const uint4* __restrict__ gtab) {
    constexpr uint32_t MASK = (1u << COMB_BITS) - 1u;
    uint32_t c[8] = {u.v[0], u.v[1], u.v[2], u.v[3], u.v[4], u.v[5], u.v[6], u.v[7]};
    ge9 Pn;
    const uint32_t d0 = c[0] & MASK;
    gtab_load(Pn, gtab + (size_t)d0 * GTAB_ENTRY_U4);
    // window 0 starts the sum: its entry is the accumulator (Z = 1), no add
    acc.x = Pn.x;
    acc.y = Pn.y;
    fe9_set_u32(acc.z, 1);
    inf = d0 == 0;
    comb_shift(c);  // c = u >> (COMB_BITS w) at the top of window w
    gtab_load(Pn, gtab + (((size_t)1 << COMB_BITS) + (c[0] & MASK)) * GTAB_ENTRY_U4);
#pragma unroll 1
    for (int w = 1; w < COMB_WINDOWS; w++) {
        uint32_t d = c[0] & MASK;
        ge9 P = Pn;
        if (w < COMB_WINDOWS - 1) {  // prefetch next window's entry
            comb_shift(c);
            gtab_load(Pn, gtab + (((size_t)(w + 1) << COMB_BITS) + (c[0] & MASK)) * GTAB_ENTRY_U4);
        }
        gej9 t;
        bool tinf = inf;
        gej9_add_ge(t, tinf, acc, P);
        if (d != 0) {
            acc = t;
            inf = tinf;
        }
    }
}

// Jacobian -> affine canonical 8 x 32-bit words
GSV_DI void gej9_to_affine_words(fe& ax, fe& ay, const gej9& q) {
    fe9 zi, zi2, x, y;
    {
        fe9 z = q.z;
        fe9_normalize_full(z);
        uint32_t zw[8], iw[8];
        fe9_to_words(zw, z);
        modinv30_words(iw, zw, MI30_P);  // Z^-1 mod p (safegcd)
        fe9_from_words(zi, iw);
    }
    fe9_sqr(zi2, zi);
    fe9_mul(x, q.x, zi2);
    fe9_mul(zi2, zi2, zi);
    fe9_mul(y, q.y, zi2);
    fe9_normalize_full(x);
    fe9_normalize_full(y);
    fe9_to_words(ax.v, x);
    fe9_to_words(ay.v, y);
}

// u2 R runs on the curve E_t: y^2 = x^3 + 7 c^3 (c = x_R^3 + 7), the image of E under
// (x, y) -> (t^2 x, t^3 y) for t = y_R, where R is (c x_R, c^2) whatever t is, so no square root is
// taken before the scalar multiplication.  A Jacobian (X, Y, Z) on E_t is (X, Y, t Z) on E; the sum with
// u1 G is carried as a + t b, and ONE exponentiation at the end, w = (c z^4)^((p-3)/4) = 1/(s0 z^2)
// with s0 = c^((p+1)/4), yields the root (s0 = c w z^2, t = +-s0 by the recid parity) and the inverse of
// Z (1/(s0 z) = w z): the separate Z^-1 safegcd is gone (r04; through r03 the square root came first,
// then the affine conversion by safegcd).

// Q = P1 + P2 with P1 = u1 G on E (Jacobian, inf flag p1inf) and P2 = u2 R given on E_t as (X*, Y*, Z*)
// (P2 on E = (X*, Y*, t Z*)), c = x_R^3 + 7, par = the parity y_R must have.  Returns false when c is
// not a square (no R), u2 R = O or Q = O; otherwise (qx, qy) is Q in canonical words.
// add-2001-b with Z2 = t Z*: Z2^2 = c Z*^2 is rational, S1 = Y1 Z2^3 = t S1' with S1' = Y1 Z* c Z*^2,
// rr = S2 - t S1', and X3 = X3a + t X3b, Y3 = Y3a + t Y3b, Z3 = t z.  (tests/test_recover_twist.py
// restates it with Python integers, exceptional cases included.)
GSV_DI bool recover_tail_twisted(fe& qx, fe& qy, const gej9& p1, bool p1inf, const gej9& p2, bool p2inf,
                                 const fe9& c, uint32_t par) {
    fe9 x3a, db, y3a, y3b, z;  // X3b = -db
    fe9 s1p, s2;
    bool exc;
    {
        fe9 z1z1, zz, z2z2, u1, h, t;
        fe9_sqr(z1z1, p1.z);                 // 2 -> 1
        fe9_sqr(zz, p2.z);                   // 1
        fe9_mul(z2z2, c, zz);                // Z2^2 = c Z*^2, 1
        fe9_mul(u1, p1.x, z2z2);             // 1
        fe9_neg<1>(t, u1);
        fe9_mul_add(h, p2.x, z1z1, t);       // H = U2 - U1, 1 (weakly normalised)
        fe9_mul(s1p, p1.y, p2.z);
        fe9_mul(s1p, s1p, z2z2);             // S1', 1
        fe9_mul(s2, p2.y, p1.z);             // 1*2
        fe9_mul(s2, s2, z1z1);               // S2, 1
        exc = !p1inf && fe9_is_zero_weak(h);
        fe9 hh, hhh, v, cs1, a1;
        fe9_sqr(hh, h);
        fe9_mul(hhh, h, hh);                 // H^3
        fe9_mul(v, u1, hh);                  // V = U1 H^2
        fe9_mul(cs1, c, s1p);                // c S1'
        fe9_negsum3<3>(t, hhh, v, v);        // -(H^3 + 2V)
        fe9_sqr_add(a1, s2, t);              // S2^2 - H^3 - 2V, 1
        fe9_mul_add(x3a, cs1, s1p, a1);      // X3a = S2^2 + c S1'^2 - H^3 - 2V, 1
        fe9_mul(t, s2, s1p);
        fe9_add(db, t, t);                   // db = 2 S2 S1' = -X3b, 2
        fe9 da, ndb, e;
        fe9_sub<1>(da, v, x3a);              // Da = V - X3a, 3
        fe9_neg<2>(ndb, db);                 // 3
        fe9_dot(y3a, s2, da, cs1, ndb);      // Y3a = S2 Da - c S1' Db, 1*3 + 1*3
        fe9_add(e, da, hhh);                 // 4
        fe9_normalize_weak(e);
        fe9_neg<1>(t, e);                    // 2
        fe9_dot(y3b, s2, db, s1p, t);        // Y3b = S2 Db - S1' (Da + H^3), 1*2 + 1*2
        fe9_mul(t, p1.z, p2.z);              // 2*1
        fe9_mul(z, t, h);                    // z = Z1 Z* H, 1
    }
    if (FE9_ANY(exc)) {  // P1 == +-P2 (rare; wave-uniform): 2 P2 on E_t, decided below by rr == 0
        gej9 d;
        gej9_dbl(d, p2);
        fe9_cmov(x3a, d.x, exc);
        fe9_cmov(y3a, d.y, exc);
        fe9_cmov(z, d.z, exc);
        fe9_cmov(db, s1p, exc);              // stash S1', S2 for the rr test
        fe9_cmov(y3b, s2, exc);
    }
    if (FE9_ANY(p1inf)) {  // u1 G = O: Q = P2
        fe9 zero;
        fe9_set_u32(zero, 0);
        fe9_cmov(x3a, p2.x, p1inf);
        fe9_cmov(y3a, p2.y, p1inf);
        fe9_cmov(z, p2.z, p1inf);
        fe9_cmov(db, zero, p1inf);
        fe9_cmov(y3b, zero, p1inf);
    }
    // the one exponentiation
    fe9 m, s0;
    bool ok;
    {
        fe9 z2, t, w;
        fe9_sqr(z2, z);                      // z magnitude <= 2
        fe9_sqr(t, z2);
        fe9_mul(t, t, c);                    // c z^4
        fe9_pow_pm3_4(w, t);                 // 1/(s0 z^2)
        fe9_mul(m, w, z);                    // 1/(s0 z)
        fe9_mul(t, c, m);
        fe9_mul(s0, t, z);                   // s0 = c w z^2
        fe9_sqr(t, s0);
        fe9_normalize_full(t);
        fe9 cc = c;
        fe9_normalize_full(cc);
        ok = fe9_eq_canon(t, cc) && !p2inf;  // c a square (R exists), u2 R != O
    }
    fe9 s0n = s0;
    fe9_normalize_full(s0n);
    bool flip = (s0n.v[0] & 1u) != par;     // t = -s0
    fe9 pb, qb;
    fe9_mul(pb, s0, db);                     // 1*2
    fe9_mul(qb, s0, y3b);
    if (FE9_ANY(exc)) {  // rr = S2 - t S1' = y3b - (+-pb): zero -> the doubling, else Q = O
        fe9 a, b2;
        fe9_add(a, y3b, pb);                 // t = -s0
        fe9_sub<1>(b2, y3b, pb);             // t = s0
        fe9_cmov(b2, a, flip);
        bool rr0 = fe9_is_zero(b2);
        ok = ok && !(exc && !rr0);
        fe9 zero;
        fe9_set_u32(zero, 0);
        fe9_cmov(pb, zero, exc);
        fe9_cmov(qb, zero, exc);
    }
    // x = (X3a - t db) m^2 with t = +-s0; y = Y3 / (t z)^3 = (+-Y3a + s0 Y3b) m^3 (1/t = +-1/s0)
    fe9 m2, m3, n, xs, ys;
    fe9_sqr(m2, m);
    fe9_mul(m3, m2, m);
    fe9_neg<1>(n, pb);
    fe9_cmov(n, pb, flip);                   // -t db = -(+-s0) db
    fe9_add(xs, x3a, n);                     // 1 + 2
    fe9_neg<1>(n, y3a);
    fe9_cmov(n, y3a, !flip);                 // sign(t) Y3a
    fe9_add(ys, n, qb);                      // 2 + 1
    fe9 x, y;
    fe9_mul(x, xs, m2);
    fe9_mul(y, ys, m3);
    fe9_normalize_full(x);
    fe9_normalize_full(y);
    fe9_to_words(qx.v, x);
    fe9_to_words(qy.v, y);
    return ok;
}

// Both GLV halves are made odd before the recoding by adding a vector of the GLV lattice
// ({(a, b) : a + b lambda == 0 mod n}, libsecp256k1 scalar_impl.h's basis), so the odd-digit recoding
// needs no skew and the two skew-correcting mixed adds at the end of u2 R disappear.  v1 = (a1, b1)
// has odd/odd coordinates, v2 = (a2, a1) even/odd, v1 + v2 odd/even: one of them (or none) turns the
// magnitudes |k1|, |k2| (parity of k mod n XOR its sign, n being odd) both odd.  |a1| < 2^126,
// |b1| < 2^128, |a2| < 2^129: |k| < 2^128 grows below 2^129.3 < 2^130, inside GLV_DIGITS' range.
__device__ constexpr uint32_t GLV_V1A[8] = {0x9284EB15u, 0xE86C90E4u, 0xA7D46BCDu, 0x3086D221u, 0u, 0u, 0u, 0u};
__device__ constexpr uint32_t GLV_V1B[8] = {0xC5765C7Eu, 0x507DDEE3u, 0xAE3A1813u, 0xD66B5E10u,
                                            0xFFFFFFFDu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
__device__ constexpr uint32_t GLV_V2A[8] = {0x9D44CFD8u, 0x57C1108Du, 0xA8E2F3F6u, 0x14CA50F7u, 1u, 0u, 0u, 0u};
__device__ constexpr uint32_t GLV_V3A[8] = {0x2FC9BAEDu, 0x402DA172u, 0x50B75FC4u, 0x45512319u, 1u, 0u, 0u, 0u};
__device__ constexpr uint32_t GLV_V3B[8] = {0x57FB4793u, 0x38EA6FC8u, 0x560E83E1u, 0x06F23032u,
                                            0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
GSV_DI void glv_make_odd(sc& k1, sc& k2) {
    bool odd1 = ((k1.v[0] & 1u) != 0) != sc_is_high(k1);  // parity of |k1|
    bool odd2 = ((k2.v[0] & 1u) != 0) != sc_is_high(k2);
    // (flip k1, flip k2): (1, 1) v1, (0, 1) v2 = (a2, a1), (1, 0) v1 + v2, (0, 0) nothing
    bool use1 = !odd1 && !odd2, use2 = odd1 && !odd2, use3 = !odd1 && odd2;
    sc A, B;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        A.v[i] = use1 ? GLV_V1A[i] : use2 ? GLV_V2A[i] : use3 ? GLV_V3A[i] : 0u;
        B.v[i] = use1 ? GLV_V1B[i] : use2 ? GLV_V1A[i] : use3 ? GLV_V3B[i] : 0u;
    }
    sc_add(k1, k1, A);
    sc_add(k2, k2, B);
}

// ---------------------------------------------------------------------------- recovery core
// Returns GSV_ST_OK or GSV_ST_RECOVER_FAILED; on OK (qx, qy) is the affine public key.
// msg/r/s are 256-bit values as little-endian limbs; recid in 0..3.
GSV_DI uint32_t recover_core(fe& qx, fe& qy, const uint32_t msg[8], const uint32_t r[8],
                             const uint32_t s[8], uint32_t recid, const uint4* __restrict__ gtab,
                             uint32_t* __restrict__ ltab) {
    bool ok = limbs_lt(r, SN) && limbs_lt(s, SN);
    sc rs, ss, m;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        rs.v[i] = r[i];
        ss.v[i] = s[i];
    }
    ok = ok && !sc_is_zero(rs) && !sc_is_zero(ss);
    sc_cond_sub_n(m.v, msg, 0);  // msg mod n (msg < 2^256 < 2n)

    // x = r (+ n when recid & 2; fails for r >= p - n)
    fe9 x;
    {
        bool hi = (recid & 2u) != 0;
        ok = ok && (!hi || limbs_lt(r, P_MINUS_N));
        uint32_t xw[8];
        uint64_t c = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            c = (uint64_t)r[i] + (hi ? SN[i] : 0u) + hi32(c);
            xw[i] = lo32(c);
        }
        fe9_from_words(x, xw);
    }
    fe9 y, t;
    // R on E_t (see recover_tail_twisted): (c x, c^2), c = x^3 + 7; the root is taken at the end
    fe9 c;
    fe9_sqr(t, x);
    fe9_mul(c, t, x);
    c.v[0] += 7u;
    fe9_mul(t, c, x);
    fe9_sqr(y, c);
    x = t;
    // u1 = -m / r, u2 = s / r
    sc rn, u1, u2;
    modinv30_words(rn.v, rs.v, MI30_N);  // r^-1 mod n (safegcd; r != 0 on every valid path)
    sc_mul(u1, rn, m);
    sc_neg(u1, u1);
    sc_mul(u2, rn, ss);

    // ---- u2 * R via GLV + fixed w = GLV_W odd digits
    sc k1, k2;
    sc_split_lambda(k1, k2, u2);
    glv_make_odd(k1, k2);  // both halves odd: the recoding's skews are 0, no correcting adds
    bool neg1 = sc_is_high(k1), neg2 = sc_is_high(k2);
    {
        sc nk;
        sc_neg(nk, k1);
#pragma unroll
        for (int i = 0; i < 8; i++) k1.v[i] = neg1 ? nk.v[i] : k1.v[i];
        sc_neg(nk, k2);
#pragma unroll
        for (int i = 0; i < 8; i++) k2.v[i] = neg2 ? nk.v[i] : k2.v[i];
    }
    uint32_t dig1[DIG_WORDS], dig2[DIG_WORDS], skew1, skew2;  // skews 0 (odd halves)
    recode_glv(dig1, skew1, k1);
    recode_glv(dig2, skew2, k2);

    // The GLV table {x[GLV_NT], y[GLV_NT]} of the odd multiples (2e+1)R lives in LDS (w = 3:
    // ltab = this lane's column of a [word][256 lanes] array, conflict-free for any per-lane entry
    // index) or in a private array (wider windows), not in VGPRs, which would cost occupancy.
    // Each add loads its entry by index (no selects); lambda(P) = (beta x, y) costs one product per
    // lambda add.
    // entry e < GLV_LNT: LDS words [e*9 + k] (x) and [9*GLV_LNT + e*9 + k] (y); the others: the
    // private array, x at [(e - GLV_LNT)*9 + k], y after all x
    constexpr int PNT = GLV_NT - GLV_LNT;
    uint32_t ptab[18 * (PNT > 0 ? PNT : 1)];
#define GLV_L(i) ltab[(i) * GSV_LTAB_STRIDE]
#define GLV_X(e, k) ((e) < GLV_LNT ? GLV_L((e) * 9 + (k)) : ptab[((e) - GLV_LNT) * 9 + (k)])
#define GLV_Y(e, k) ((e) < GLV_LNT ? GLV_L(9 * GLV_LNT + (e) * 9 + (k)) : ptab[9 * PNT + ((e) - GLV_LNT) * 9 + (k)])
#define GLV_SET(e, k, X, Y)                                           \
    do {                                                              \
        if ((e) < GLV_LNT) {                                          \
            GLV_L((e) * 9 + (k)) = (X);                               \
            GLV_L(9 * GLV_LNT + (e) * 9 + (k)) = (Y);                 \
        } else {                                                      \
            ptab[((e) - GLV_LNT) * 9 + (k)] = (X);                    \
            ptab[9 * PNT + ((e) - GLV_LNT) * 9 + (k)] = (Y);          \
        }                                                             \
    } while (0)
    // Odd multiples on an isomorphic curve E'' (affine there, no inversion): P_e = (2e+1)R' built
    // by mixed adds of D = 2R' with their z-ratios zr_e, stored unscaled, then every entry below the
    // last rescaled to the last one's Z by the product of the later z-ratios.  A Jacobian result
    // (X, Y, Z) on E'' is (X, Y, Z zfac) on E.
    // Built with co-Z arithmetic (secp256k1_fe9.cuh ge9_dblu / ge9_zaddu): the pair (2R, R) at the
    // common Z = 2y, then each P_e = D + P_{e-1} keeps D co-Z with it; z-ratios as above.
    fe9 zfac;
    {
        ge9 Dp, P;
        fe9 zd;
        ge9_dblu(Dp, P, zd, x, y);
        fe9 zr[GLV_NT];
#pragma unroll
        for (int e = 0; e < GLV_NT; e++) {
            if (e) {
                ge9 Pn;
                ge9_zaddu(Pn, Dp, zr[e], P);
                P = Pn;
            }
#pragma unroll
            for (int k = 0; k < 9; k++) GLV_SET(e, k, P.x.v[k], P.y.v[k]);
        }
        fe9 f = zr[GLV_NT - 1];
#pragma unroll
        for (int e = GLV_NT - 2; e >= 0; e--) {
            fe9 ex, ey;
#pragma unroll
            for (int k = 0; k < 9; k++) {
                ex.v[k] = GLV_X(e, k);
                ey.v[k] = GLV_Y(e, k);
            }
            ge9 q;
            scale_xy9(q, ex, ey, f);
#pragma unroll
            for (int k = 0; k < 9; k++) GLV_SET(e, k, q.x.v[k], q.y.v[k]);
            if (e) fe9_mul(f, f, zr[e]);  // 1
        }
        fe9_mul(zfac, f, zd);  // f = all the z-ratios: the entries' common Z on E is zd f
    }

    gej9 acc;
    bool ainf = true;
#pragma unroll
    for (int k = 0; k < 9; k++) {
        acc.x.v[k] = GLV_X(0, k);
        acc.y.v[k] = GLV_Y(0, k);
    }
    fe9_set_u32(acc.z, 1);
#pragma unroll 1
    for (int i = GLV_DIGITS - 1; i >= 0; i--) {
        if (i != GLV_DIGITS - 1) {
#pragma unroll 1
            for (int d = 0; d < GLV_W; d++) gej9_dbl(acc, acc);
        }
        constexpr uint32_t CMASK = (1u << DIG_SLOT) - 1u;
        uint32_t c1 = (sel_word(dig1, (uint32_t)i / DIG_PER_WORD) >> ((i % DIG_PER_WORD) * DIG_SLOT)) & CMASK;
        uint32_t c2 = (sel_word(dig2, (uint32_t)i / DIG_PER_WORD) >> ((i % DIG_PER_WORD) * DIG_SLOT)) & CMASK;
        // one add body, two passes: digit of k1 on T, digit of k2 on lambda(T) = (beta x, y)
#pragma unroll 1
        for (int j = 0; j < 2; j++) {
            uint32_t c = j ? c2 : c1;
            bool ng = j ? neg2 : neg1;
            uint32_t ei = c & (uint32_t)(GLV_NT - 1);
            ge9 P;
            if (GLV_LNT == GLV_NT || (GLV_LNT > 0 && ei < (uint32_t)GLV_LNT)) {
                uint32_t xo = ei * 9u;
#pragma unroll
                for (int k = 0; k < 9; k++) {
                    P.x.v[k] = GLV_L(xo + k);
                    P.y.v[k] = GLV_L(9u * GLV_LNT + xo + k);
                }
            } else {  // the lanes whose digit indexes the private part (divergent: each side loads only its lanes)
                uint32_t xo = (ei - (uint32_t)GLV_LNT) * 9u;
#pragma unroll
                for (int k = 0; k < 9; k++) {
                    P.x.v[k] = ptab[xo + k];
                    P.y.v[k] = ptab[9u * PNT + xo + k];
                }
            }
            if (j != 0) {  // wave-uniform
                fe9 beta;
                fe9_from_const(beta, BETA);
                fe9_mul(P.x, P.x, beta);
            }
            fe9 ny;
            fe9_neg<1>(ny, P.y);         // 2
            fe9_cmov(P.y, ny, ((c >> (GLV_W - 1)) != 0) != ng);
            if (i == GLV_DIGITS - 1 && j == 0) {  // the top digit starts the sum (Z = 1), no add
                acc.x = P.x;
                acc.y = P.y;
                fe9_normalize_weak(acc.y);
                fe9_set_u32(acc.z, 1);
                ainf = false;
                continue;
            }
            gej9_add_ge(acc, ainf, acc, P);
        }
    }
    fe9_mul(acc.z, acc.z, zfac);  // back from E'' to E_t (2*1 -> 1)

    // ---- u1 * G via comb
    gej9 accg;
    bool ginf;
    comb_mul_g9(accg, ginf, u1, gtab);

    // ---- Q = u2 R + u1 G
    ok = recover_tail_twisted(qx, qy, accg, ginf, acc, ainf, c, recid & 1u) && ok;
    return ok ? GSV_ST_OK : GSV_ST_RECOVER_FAILED;
}

GSV_DI void load32_be(uint32_t v[8], const uint8_t* p) { limbs_from_be(v, p); }

GSV_DI void store_pub_addr(uint8_t* pub65, uint8_t* addr20, bool ok, const fe& qx, const fe& qy) {
    if (pub65) {
        pub65[0] = ok ? 4 : 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            uint32_t xv = ok ? qx.v[7 - i] : 0u, yv = ok ? qy.v[7 - i] : 0u;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                pub65[1 + 4 * i + b] = (uint8_t)(xv >> (24 - 8 * b));
                pub65[33 + 4 * i + b] = (uint8_t)(yv >> (24 - 8 * b));
            }
        }
    }
    if (addr20) {
        uint32_t h[8];
        keccak256_xy(h, qx.v, qy.v);
        // hash bytes 12..31 = words 3..7 (little-endian byte order within words)
#pragma unroll
        for (int w = 3; w < 8; w++)
#pragma unroll
            for (int b = 0; b < 4; b++) addr20[(w - 3) * 4 + b] = ok ? (uint8_t)(h[w] >> (8 * b)) : 0;
    }
}


// ---------------------------------------------------------------------------- synthetic signer
// Bench/test data generator (signing is not on the validation path): key_i, msg_i, nonce_i are
// Keccak-256 of (le64(seed) || le64(i) || tag), keys/nonces reduced mod n (0 -> 1).
GSV_DI void derive32(uint32_t out_be_limbs[8], uint64_t seed, uint64_t i, uint32_t tag3) {
    uint64_t a[25];
#pragma unroll
    for (int k = 0; k < 25; k++) a[k] = 0;
    a[0] = seed;
    a[1] = i;
    a[2] = (uint64_t)(tag3 & 0xFFFFFFu) | (0x01ull << 24);
    a[16] = 0x8000000000000000ULL;
    keccakf(a);
    // hash bytes as a big-endian 256-bit number -> limbs
#pragma unroll
    for (int j = 0; j < 4; j++) {
        out_be_limbs[7 - 2 * j] = __builtin_bswap32((uint32_t)a[j]);
        out_be_limbs[6 - 2 * j] = __builtin_bswap32((uint32_t)(a[j] >> 32));
    }
}

// ECDSA signature with explicit nonce, low-s normalised (libsecp256k1 semantics); d, k are
// reduced mod n here (0 -> 1).  (px, py) = d*G.  m = message as limbs (any 256-bit value).
GSV_DI void ecdsa_sign(uint32_t r_out[8], uint32_t s_out[8], uint32_t& recid, fe& px, fe& py, sc d, sc k,
                       const uint32_t m[8], const uint4* __restrict__ gtab) {
    sc_cond_sub_n(d.v, d.v, 0);
    sc_cond_sub_n(k.v, k.v, 0);
    if (sc_is_zero(d)) d.v[0] = 1;
    if (sc_is_zero(k)) k.v[0] = 1;
    sc mr;
    sc_cond_sub_n(mr.v, m, 0);
    gej9 P;
    bool pinf;
    comb_mul_g9(P, pinf, d, gtab);
    gej9_to_affine_words(px, py, P);
    gej9 R;
    bool rinf;
    comb_mul_g9(R, rinf, k, gtab);
    fe rx, ry;
    gej9_to_affine_words(rx, ry, R);
    recid = ry.v[0] & 1u;
    sc r;
    bool over = !limbs_lt(rx.v, SN);
    sc_cond_sub_n(r.v, rx.v, 0);
    if (over) recid |= 2u;
    // s = k^-1 (m + r d)
    sc kinv, s, t;
    modinv30_words_ct(kinv.v, k.v, MI30_N);  // the nonce is secret: constant-time divsteps
    sc_mul(t, r, d);
    sc_add(t, t, mr);
    sc_mul(s, kinv, t);
    if (sc_is_high(s)) {
        sc_neg(s, s);
        recid ^= 1u;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
        r_out[i] = r.v[i];
        s_out[i] = s.v[i];
    }
}

}  // namespace gsv

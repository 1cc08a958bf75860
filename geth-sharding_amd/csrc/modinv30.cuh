// Constant-time modular inversion by Bernstein-Yang "safegcd" divsteps (20 batches of 30
// divsteps, signed 30-bit limbs), for the secp256k1 group order n and field prime p and the BN254
// base field prime.
//
// Why: the Fermat inversions it replaces cost ~255 squarings + ~15-75 products each (the scalar
// one in 8 x 32-bit carry-chain arithmetic: ~16 % of k_ecrecover).  A divstep is ~19 plain
// 32-bit VALU ops (xor/sub/and/add/shift — the full-rate class on gfx950), and every 30 of them
// cost one 2x2 matrix application to (d, e) and (f, g): ~8k issue slots per inversion instead of
// ~40-80k.  Branch-free (fixed 600 divsteps >= the 590 a 256-bit input needs), so every lane of a
// wave runs the same instruction stream.
//
// Restates the published algorithm (Bernstein & Yang, "Fast constant-time gcd computation and
// modular inversion", 2019) in the form libsecp256k1 later adopted (modinv32); the reference's
// vendored libsecp256k1 snapshot predates it and inverts by exponentiation
// (crypto/secp256k1/libsecp256k1/src/scalar_impl.h:262, field_impl.h:226) — results are the same
// residues.  Host-compilable: tests/test_fe9.py checks it against Python's pow(x, -1, m).
#pragma once
#include <stdint.h>

#include "opcount.cuh"

#if defined(__HIPCC__)
#define MI30_FN __device__ __forceinline__
#define MI30_CONST __device__ constexpr
#else
#define MI30_FN static inline
#define MI30_CONST static constexpr
#endif

namespace gsv {

struct s30 { int32_t v[9]; };  // value = sum v[i] 2^(30 i), limbs in (-2^30, 2^30)

struct modinfo30 {
    int32_t m[9];       // modulus in signed30 limbs
    uint32_t m_inv30;   // modulus^-1 mod 2^30
};
MI30_CONST modinfo30 MI30_N = {{0x10364141, 0x3F497A33, 0x348A03BB, 0x2BB739AB, 0x3FFFFEBA, 0x3FFFFFFF,
                                0x3FFFFFFF, 0x3FFFFFFF, 0xFFFF}, 0x2A774EC1u};
MI30_CONST modinfo30 MI30_P = {{0x3FFFFC2F, 0x3FFFFFFB, 0x3FFFFFFF, 0x3FFFFFFF, 0x3FFFFFFF, 0x3FFFFFFF,
                                0x3FFFFFFF, 0x3FFFFFFF, 0xFFFF}, 0x2DDACACFu};
// the BN254 base field prime (crypto/bn256/cloudflare/constants.go:22), for F_p inversions
MI30_CONST modinfo30 MI30_BN = {{0x187CFD47, 0x3082305B, 0x071CA8D3, 0x205AA45A, 0x01585D97, 0x0116DA06,
                                 0x1A029B85, 0x139CB84C, 0x00003064}, 0x1B799C77u};

constexpr int32_t MI30_M30 = 0x3FFFFFFF;

// 1: variable-time divsteps (mi30_divsteps_var; +0.95 % on ecrecover, profiles/r02/ab_vargcd.txt),
// 0: the constant-time 600 fixed divsteps
#ifndef MI30_VAR
#define MI30_VAR 1
#endif

struct trans2x2 { int32_t u, v, q, r; };

// 30 divsteps on the low limbs of f (odd) and g; returns the new zeta = -(delta + 1/2)
MI30_FN int32_t mi30_divsteps(int32_t zeta, uint32_t f0, uint32_t g0, trans2x2& t) {
    uint32_t u = 1, v = 0, q = 0, r = 1, f = f0, g = g0;
#pragma unroll
    for (int i = 0; i < 30; i++) {
        uint32_t c1 = (uint32_t)(zeta >> 31);  // zeta < 0
        uint32_t c2 = 0u - (g & 1u);           // g odd
        uint32_t x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
        g += x & c2;
        q += y & c2;
        r += z & c2;
        c1 &= c2;                               // zeta < 0 and g odd: swap
        zeta = (int32_t)(((uint32_t)zeta ^ c1) - 1u);
        f += g & c1;
        u += q & c1;
        v += r & c1;
        g >>= 1;
        u <<= 1;
        v <<= 1;
    }
    t.u = (int32_t)u;
    t.v = (int32_t)v;
    t.q = (int32_t)q;
    t.r = (int32_t)r;
    return zeta;
}

// The variable-time form (Bernstein-Yang's divstep with eta = -delta, as libsecp256k1's later
// modinv32_var): a run of zero low bits of g is one shift (count trailing zeros), and each odd step
// clears up to 8 more bits at once with w = -g f^-1 mod 2^limit.  The 30-step transition matrix is
// the same kind of matrix (|u| + |v| <= 2^30 ...), so update_de / update_fg apply unchanged.  Nothing
// here is secret (signatures and public keys are public), so data-dependent timing is harmless; on
// the GPU a wave runs as many inner iterations as its slowest lane (~12 per 30 divsteps instead of
// 30 fixed steps).
#if defined(__HIPCC__)
#define MI30_CTZ(x) ((uint32_t)__builtin_ctz(x))
#define MI30_MUL8(a, b) __umul24((a), (b))  /* only the low 8 bits of the product are used */
#define MI30_ANY(x) (__any(x) != 0)
#else
#define MI30_CTZ(x) ((uint32_t)__builtin_ctz(x))
#define MI30_MUL8(a, b) ((a) * (b))
#define MI30_ANY(x) (x)
#endif
MI30_FN int32_t mi30_divsteps_var(int32_t eta, uint32_t f0, uint32_t g0, trans2x2& t) {
    uint32_t u = 1, v = 0, q = 0, r = 1, f = f0, g = g0;
    int32_t i = 30;
    for (;;) {
        uint32_t zeros = MI30_CTZ(g | (0xFFFFFFFFu << i));  // <= i
        g >>= zeros;
        u <<= zeros;
        v <<= zeros;
        eta -= (int32_t)zeros;
        i -= (int32_t)zeros;
        if (i == 0) break;
        if (eta < 0) {  // g odd and eta < 0: (f, g) <- (g, -f), (u, q) <- (q, -u), (v, r) <- (r, -v)
            uint32_t x;
            eta = -eta;
            x = f; f = g; g = 0u - x;
            x = u; u = q; q = 0u - x;
            x = v; v = r; r = 0u - x;
        }
        int32_t limit = (eta + 1) > i ? i : (eta + 1);
        uint32_t m = (0xFFFFFFFFu >> (32 - limit)) & 255u;
        // f^-1 mod 256 by Newton from f (correct mod 8 for odd f): two steps give mod 2^12
        uint32_t fl = f & 255u, x = fl;
        x = MI30_MUL8(x, 2u - MI30_MUL8(fl, x)) & 255u;
        x = MI30_MUL8(x, 2u - MI30_MUL8(fl, x)) & 255u;
        uint32_t w = (0u - MI30_MUL8(g & 255u, x)) & m;  // g + f w == 0 mod 2^limit
        g = (uint32_t)((uint64_t)f * w + g);
        q = (uint32_t)((uint64_t)u * w + q);
        r = (uint32_t)((uint64_t)v * w + r);
    }
    t.u = (int32_t)u;
    t.v = (int32_t)v;
    t.q = (int32_t)q;
    t.r = (int32_t)r;
    return eta;
}

// [d, e] <- t [d, e] / 2^30 (mod m), keeping d, e in (-2m, m)
MI30_FN void mi30_update_de(s30& d, s30& e, const trans2x2& t, const modinfo30& mi) {
    const int32_t u = t.u, v = t.v, q = t.q, r = t.r;
    int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
    int32_t md = (u & sd) + (v & se);
    int32_t me = (q & sd) + (r & se);
    int32_t di = d.v[0], ei = e.v[0];
    int64_t cd = (int64_t)u * di + (int64_t)v * ei;
    int64_t ce = (int64_t)q * di + (int64_t)r * ei;
    md -= (int32_t)((mi.m_inv30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)MI30_M30);
    me -= (int32_t)((mi.m_inv30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)MI30_M30);
    cd += (int64_t)mi.m[0] * md;
    ce += (int64_t)mi.m[0] * me;
    cd >>= 30;
    ce >>= 30;
#pragma unroll
    for (int i = 1; i < 9; i++) {
        di = d.v[i];
        ei = e.v[i];
        cd += (int64_t)u * di + (int64_t)v * ei;
        ce += (int64_t)q * di + (int64_t)r * ei;
        cd += (int64_t)mi.m[i] * md;
        ce += (int64_t)mi.m[i] * me;
        d.v[i - 1] = (int32_t)cd & MI30_M30;
        cd >>= 30;
        e.v[i - 1] = (int32_t)ce & MI30_M30;
        ce >>= 30;
    }
    d.v[8] = (int32_t)cd;
    e.v[8] = (int32_t)ce;
}

// [f, g] <- t [f, g] / 2^30 (exact)
MI30_FN void mi30_update_fg(s30& f, s30& g, const trans2x2& t) {
    const int32_t u = t.u, v = t.v, q = t.q, r = t.r;
    int32_t fi = f.v[0], gi = g.v[0];
    int64_t cf = (int64_t)u * fi + (int64_t)v * gi;
    int64_t cg = (int64_t)q * fi + (int64_t)r * gi;
    cf >>= 30;
    cg >>= 30;
#pragma unroll
    for (int i = 1; i < 9; i++) {
        fi = f.v[i];
        gi = g.v[i];
        cf += (int64_t)u * fi + (int64_t)v * gi;
        cg += (int64_t)q * fi + (int64_t)r * gi;
        f.v[i - 1] = (int32_t)cf & MI30_M30;
        cf >>= 30;
        g.v[i - 1] = (int32_t)cg & MI30_M30;
        cg >>= 30;
    }
    f.v[8] = (int32_t)cf;
    g.v[8] = (int32_t)cg;
}

// r in (-2m, m), negated when sign < 0  ->  [0, m)
MI30_FN void mi30_normalize(s30& r, int32_t sign, const modinfo30& mi) {
    int32_t ca = r.v[8] >> 31;
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] += mi.m[i] & ca;
    int32_t cn = sign >> 31;
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] = (r.v[i] ^ cn) - cn;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        r.v[i + 1] += r.v[i] >> 30;
        r.v[i] &= MI30_M30;
    }
    ca = r.v[8] >> 31;
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] += mi.m[i] & ca;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        r.v[i + 1] += r.v[i] >> 30;
        r.v[i] &= MI30_M30;
    }
}

// 8 x 32-bit little-endian words <-> signed30 (non-negative values < 2^256)
MI30_FN void s30_from_words(s30& r, const uint32_t w[8]) {
#pragma unroll
    for (int i = 0; i < 9; i++) {
        int bit = 30 * i, wi = bit >> 5, sh = bit & 31;
        uint32_t lo = w[wi] >> sh;
        uint32_t hi = (sh > 2 && wi + 1 < 8) ? (w[wi + 1] << (32 - sh)) : 0u;
        r.v[i] = (int32_t)((lo | hi) & (uint32_t)MI30_M30);
    }
}
MI30_FN void s30_to_words(uint32_t w[8], const s30& a) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
        int bit = 32 * j, li = bit / 30, sh = bit % 30;
        uint32_t x = (uint32_t)a.v[li] >> sh;
        if (li + 1 < 9) x |= (uint32_t)a.v[li + 1] << (30 - sh);
        if (sh > 28 && li + 2 < 9) x |= (uint32_t)a.v[li + 2] << (60 - sh);
        w[j] = x;
    }
}

// out = x^-1 mod m (x < m; 0 -> 0), words in and out.  VAR: variable-time divsteps (public inputs
// only: the recovery path's r and Z); the constant-time form is used for a secret input (the
// synthetic signer's nonce, modinv30_words_ct) whatever MI30_VAR says.
template <bool VAR>
MI30_FN void modinv30_words_t(uint32_t out[8], const uint32_t x[8], const modinfo30& mi) {
    GSV_OPC(gsv::OPC_MODINV);
    s30 d, e, f, g;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        d.v[i] = 0;
        e.v[i] = 0;
        f.v[i] = mi.m[i];
    }
    e.v[0] = 1;
    s30_from_words(g, x);
    if constexpr (VAR) {
    // variable-time divsteps until g == 0 in every lane of the wave (a lane that is done keeps
    // d and f: its matrix is then diag(2^30, 1)); 25 batches cover the original divstep's bound
    // for 256-bit inputs (724), ~19 are typical
    int32_t eta = -1;
#if defined(__HIPCC__)
#pragma unroll 1
#endif
    for (int it = 0; it < 25; it++) {
        trans2x2 t;
        eta = mi30_divsteps_var(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
        mi30_update_de(d, e, t, mi);
        mi30_update_fg(f, g, t);
        uint32_t gz = 0;
#pragma unroll
        for (int k = 0; k < 9; k++) gz |= (uint32_t)g.v[k];
        if (!MI30_ANY(gz != 0)) break;
    }
    } else {
    int32_t zeta = -1;
#if defined(__HIPCC__)
#pragma unroll 1
#endif
    for (int it = 0; it < 20; it++) {
        trans2x2 t;
        zeta = mi30_divsteps(zeta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
        mi30_update_de(d, e, t, mi);
        mi30_update_fg(f, g, t);
    }
    }
    mi30_normalize(d, f.v[8], mi);
    s30_to_words(out, d);
}
MI30_FN void modinv30_words(uint32_t out[8], const uint32_t x[8], const modinfo30& mi) {
    modinv30_words_t<MI30_VAR != 0>(out, x, mi);
}
MI30_FN void modinv30_words_ct(uint32_t out[8], const uint32_t x[8], const modinfo30& mi) {
    modinv30_words_t<false>(out, x, mi);
}

}  // namespace gsv

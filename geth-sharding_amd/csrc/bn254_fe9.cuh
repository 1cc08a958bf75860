// BN254 base field for the pairing kernels: 9 x 29-bit limbs, Montgomery form with R = 2^261, lazy
// (carry-free) reduction — the F_p layer of crypto/bn256/cloudflare (gfp.go, gfp_generic.go) and the
// F_p^2 / F_p^6 towers above it (gfp2.go, gfp6.go), re-designed for gfx950.
//
// Why.  The reference's gfP is 4 x 64-bit words with a carry after every word product; on CDNA4 a
// carry (v_addc) costs as much as a v_mad_u64_u32 (both issue at a quarter of the 64-lane rate) and
// every carry -> carry pair is padded with an s_nop.  With 29-bit limbs a Montgomery product is
// carry-free: each of its 17 columns is a v_mad_u64_u32 chain into one 64-bit accumulator (the a*b
// terms and the m*p reduction terms of the column), and additions / subtractions are limb-wise 32-bit
// adds with no carry at all.  Values are kept "lazily reduced".
//
// Magnitudes.  fqm<L, V> is an element whose limbs are all <= L M (M = 2^29 - 1) and whose integer
// value is < V p.  The bounds are template parameters, so the compiler checks every precondition:
//   * product:  La Lb <= 6  (column sums (9 La Lb + 9) 2^58 + carry < 2^64), and the Montgomery
//               output of T < Va Vb p^2 is < (Va Vb p / R + 1) p < (Va Vb / 168 + 2) p  (R / p > 168.7),
//               kept <= FQ_VMAX by reducing an input only when Va Vb (+ Vc Vd) > FQ_PROD_MAX;
//   * sum:      L <= 8 (limbs < 2^32), V <= FQ_VMAX;
//   * a - b:    a + Q - b, Q = c p with limbs i < 8 in [Lb M, Lb M + 2^29), so Q - b has limbs in
//               [0, (Lb + 1) M] (bn9_consts.inc, tools/gen_bn9_consts.py).
// When an operation's inputs would break a bound, the template normalises (carry-propagates the limbs,
// cheap) or reduces (subtracts q p, q from the top limb: value < 3 p) an input at compile time; the
// stored type fq = fqm<1, VS> is what every F_p field of a point / tower element holds.
// Equality and zero tests, and everything that leaves the kernels, go through fq_canon (< p).
//
// The F_p^2 product is two "dual" Montgomery products: x = REDC(ax by + ay bx), y = REDC(ay by +
// ax (Q - bx)) — one reduction per output coordinate and no post-subtraction (4 F_p products' worth of
// multiplications, 2 reductions).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define FQ_FN __device__ __forceinline__
#define FQ_DEVCONST __device__ constexpr
#else
#define FQ_FN static inline
#define FQ_DEVCONST static constexpr
static inline uint32_t __umulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
#endif

#include "opcount.cuh"

namespace gsv {
namespace bn {

#include "bn9_consts.inc"

#if defined(__HIP_DEVICE_COMPILE__) && !defined(BN_NO_ASM)
#include "bn9_asm.cuh"
#define BN9_ASM 1
#endif

constexpr uint32_t FQ_M29 = 0x1FFFFFFFu;
constexpr int FQ_LMAX = 8;    // limbs <= 8 (2^29 - 1) < 2^32
constexpr int FQ_VMAX = 160;  // value < 160 p: limb 8 of a normalised element stays < 2^29
constexpr int VS = 20;        // value bound of a stored element

template <int L, int V>
struct fqm {
    static_assert(L >= 1 && L <= FQ_LMAX && V >= 1 && V <= FQ_VMAX, "fqm bounds");
    uint32_t v[9];
};
using fq = fqm<1, VS>;

constexpr int fq_prod_v(int va, int vb) { return va * vb / 168 + 2; }
// the largest sum of value-bound products a Montgomery product accepts: its output bound is then
// <= FQ_VMAX (inputs are not reduced unless this would be exceeded)
constexpr int FQ_PROD_MAX = 168 * (FQ_VMAX - 2);
constexpr int imax(int a, int b) { return a > b ? a : b; }
constexpr int fq_vclass(int v) {
    for (int i = 0; i < FQ_NVCLASS; i++)
        if (FQ_VCLASS[i] >= v) return i;
    return -1;
}
constexpr int fq_qc(int l, int v) { return FQ_QC[l - 1][fq_vclass(v)]; }

// ---------------------------------------------------------------------------- normalise / reduce
template <int L, int V>
FQ_FN fqm<1, V> fq_normalize(const fqm<L, V>& a) {
    if constexpr (L == 1) {
        return fqm<1, V>{{a.v[0], a.v[1], a.v[2], a.v[3], a.v[4], a.v[5], a.v[6], a.v[7], a.v[8]}};
    } else {
        fqm<1, V> r;
        uint32_t c = 0;  // limb + carry <= 8 (2^29 - 1) + 7 < 2^32
#pragma unroll
        for (int i = 0; i < 8; i++) {
            uint32_t t = a.v[i] + c;
            r.v[i] = t & FQ_M29;
            c = t >> 29;
        }
        r.v[8] = a.v[8] + c;  // value < V p: limb 8 < V 2^21.6 + 1
        return r;
    }
}

// value < 3 p: q = an under-estimate of floor(value / p) from limb 8 (off by at most 2), minus q p
template <int L, int V>
FQ_FN fqm<1, 3> fq_reduce(const fqm<L, V>& a) {
    fqm<1, V> n = fq_normalize(a);
    uint32_t q = __umulhi(n.v[8], FQ_P8_DIV);
    fqm<1, 3> r;
    int64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        acc += (int64_t)n.v[i] - (int64_t)((uint64_t)q * FQ_P[i]);
        if (i < 8) {
            r.v[i] = (uint32_t)acc & FQ_M29;
            acc >>= 29;  // arithmetic: the borrow
        } else {
            r.v[8] = (uint32_t)acc;
        }
    }
    return r;
}

// r = x - p if x >= p, else x (x normalised, value < 2p... any value: one subtraction)
FQ_FN void fq_csub_p(uint32_t r[9], const uint32_t x[9]) {
    uint32_t d[9];
    int32_t b = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        int32_t t = (int32_t)x[i] - (int32_t)FQ_P[i] + b;
        if (i < 8) {
            d[i] = (uint32_t)t & FQ_M29;
            b = t >> 29;  // arithmetic: 0 or -1
        } else {
            d[8] = (uint32_t)t;
            b = t >> 31;
        }
    }
    bool take = b == 0;
#pragma unroll
    for (int i = 0; i < 9; i++) r[i] = take ? d[i] : x[i];
}

// the canonical residue (< p)
template <int L, int V>
FQ_FN fqm<1, 1> fq_canon(const fqm<L, V>& a) {
    fqm<1, 3> t = fq_reduce(a);
    fqm<1, 1> r;
    fq_csub_p(r.v, t.v);
    fq_csub_p(r.v, r.v);
    return r;
}

// value below Vt p with limbs normalised as needed: the form an operand is brought to before an
// operation whose bounds it would break
template <int Lt, int Vt, int L, int V>
FQ_FN auto fq_fit(const fqm<L, V>& a) {
    if constexpr (V > Vt) {
        return fq_reduce(a);
    } else if constexpr (L > Lt) {
        return fq_normalize(a);
    } else {
        return a;
    }
}

template <int L, int V>
FQ_FN fq fq_store(const fqm<L, V>& a) {
    auto t = fq_fit<1, VS>(a);
    auto n = fq_normalize(t);
    return fq{{n.v[0], n.v[1], n.v[2], n.v[3], n.v[4], n.v[5], n.v[6], n.v[7], n.v[8]}};
}

// ---------------------------------------------------------------------------- linear ops
template <int La, int Va, int Lb, int Vb>
FQ_FN auto fq_add(const fqm<La, Va>& a, const fqm<Lb, Vb>& b) {
    if constexpr (Va + Vb > FQ_VMAX) {
        if constexpr (Va >= Vb) return fq_add(fq_reduce(a), b);
        else return fq_add(a, fq_reduce(b));
    } else if constexpr (La + Lb > FQ_LMAX) {
        if constexpr (La >= Lb) return fq_add(fq_normalize(a), b);
        else return fq_add(a, fq_normalize(b));
    } else {
        fqm<La + Lb, Va + Vb> r;
#pragma unroll
        for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + b.v[i];
        return r;
    }
}

// a - b = a + Q - b
template <int La, int Va, int Lb, int Vb>
FQ_FN auto fq_sub(const fqm<La, Va>& a, const fqm<Lb, Vb>& b) {
    if constexpr (Vb > 48) {
        return fq_sub(a, fq_reduce(b));
    } else if constexpr (Lb > 6) {  // FQ_Q covers subtrahends of limb bound <= 6
        return fq_sub(a, fq_normalize(b));
    } else if constexpr (Va + fq_qc(Lb, Vb) > FQ_VMAX) {
        return fq_sub(fq_reduce(a), b);
    } else if constexpr (La + Lb + 1 > FQ_LMAX) {
        if constexpr (Lb > 1 && La + 2 <= FQ_LMAX) return fq_sub(a, fq_normalize(b));
        else return fq_sub(fq_normalize(a), b);
    } else {
        constexpr int ci = fq_vclass(Vb);
        fqm<La + Lb + 1, Va + FQ_QC[Lb - 1][ci]> r;
#pragma unroll
        for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + (FQ_Q[Lb - 1][ci][i] - b.v[i]);
        return r;
    }
}

template <int Lb, int Vb>
FQ_FN auto fq_neg(const fqm<Lb, Vb>& b) {
    if constexpr (Vb > 48) {
        return fq_neg(fq_reduce(b));
    } else if constexpr (Lb > 6) {  // FQ_Q covers subtrahends of limb bound <= 6
        return fq_neg(fq_normalize(b));
    } else {
        constexpr int ci = fq_vclass(Vb);
        fqm<Lb + 1, FQ_QC[Lb - 1][ci]> r;
#pragma unroll
        for (int i = 0; i < 9; i++) r.v[i] = FQ_Q[Lb - 1][ci][i] - b.v[i];
        return r;
    }
}

// k a for a small constant k
template <int K, int L, int V>
FQ_FN auto fq_mul_small(const fqm<L, V>& a) {
    if constexpr (V * K > FQ_VMAX) {
        return fq_mul_small<K>(fq_reduce(a));
    } else if constexpr (L * K > FQ_LMAX) {
        static_assert(K <= FQ_LMAX, "fq_mul_small constant");
        return fq_mul_small<K>(fq_normalize(a));
    } else {
        fqm<L * K, V * K> r;
#pragma unroll
        for (int i = 0; i < 9; i++) r.v[i] = a.v[i] * (uint32_t)K;
        return r;
    }
}

template <int L, int V>
FQ_FN void fq_cmov(fqm<L, V>& r, const fqm<L, V>& a, bool f) {
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] = f ? a.v[i] : r.v[i];
}

// ---------------------------------------------------------------------------- Montgomery products
// REDC(a b [+ c d]) by product scanning: column k accumulates the a_i b_j (c_i d_j) terms and the
// m_i p_j terms of the digits chosen so far; for k < 9 the digit m_k = acc n0' mod 2^29 clears the
// column's low 29 bits.  Output limbs < 2^29 (limb 8: the final carry).
template <bool DUAL>
FQ_FN void fq_redc_core(uint32_t r[9], const uint32_t a[9], const uint32_t b[9], const uint32_t c[9],
                        const uint32_t d[9]) {
#if defined(BN9_ASM)
    if constexpr (DUAL) {
        uint32_t A[2][9], B[2][9];
#pragma unroll
        for (int i = 0; i < 9; i++) {
            A[0][i] = a[i];
            A[1][i] = c[i];
            B[0][i] = b[i];
            B[1][i] = d[i];
        }
        fq_redc_asm<2>(r, A, B);
    } else {
        uint32_t A[1][9], B[1][9];
#pragma unroll
        for (int i = 0; i < 9; i++) {
            A[0][i] = a[i];
            B[0][i] = b[i];
        }
        fq_redc_asm<1>(r, A, B);
    }
    return;
#endif
    uint32_t m[9];
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 17; k++) {
#pragma unroll
        for (int i = 0; i < 9; i++) {
            int j = k - i;
            if (j >= 0 && j < 9) {
                acc += (uint64_t)a[i] * b[j];
                if (DUAL) acc += (uint64_t)c[i] * d[j];
            }
        }
#pragma unroll
        for (int i = 0; i < 9; i++) {
            int j = k - i;
            if (i < k && j >= 0 && j < 9) acc += (uint64_t)m[i] * FQ_P[j];
        }
        if (k < 9) {
            m[k] = ((uint32_t)acc * FQ_N0) & FQ_M29;
            acc += (uint64_t)m[k] * FQ_P[0];
        } else {
            r[k - 9] = (uint32_t)acc & FQ_M29;
        }
        acc >>= 29;
    }
    r[8] = (uint32_t)acc;
}

#if defined(__HIPCC__)
// out-of-line device functions (one copy in the I-cache); the F_p products themselves stay inline
// (out of line, every value live across a call would have to sit in a callee-saved register)
#define BN_NI __device__ __noinline__
#endif

// a * b R^-1 (mod p)
template <int La, int Va, int Lb, int Vb>
FQ_FN auto fq_mul(const fqm<La, Va>& a, const fqm<Lb, Vb>& b) {
    if constexpr (Va * Vb > FQ_PROD_MAX) {
        if constexpr (Va >= Vb) return fq_mul(fq_reduce(a), b);
        else return fq_mul(a, fq_reduce(b));
    } else if constexpr (La * Lb > 6) {
        if constexpr (La >= Lb) return fq_mul(fq_normalize(a), b);
        else return fq_mul(a, fq_normalize(b));
    } else {
        GSV_OPC(gsv::OPC_BN_MUL);
        GSV_OPC(gsv::OPC_BN_REDC);
        fqm<1, fq_prod_v(Va, Vb)> r;
        fq_redc_core<false>(r.v, a.v, b.v, a.v, b.v);
        return r;
    }
}

// (a b + c d) R^-1 (mod p) with one reduction
template <int La, int Va, int Lb, int Vb, int Lc, int Vc, int Ld, int Vd>
FQ_FN auto fq_mul2(const fqm<La, Va>& a, const fqm<Lb, Vb>& b, const fqm<Lc, Vc>& c, const fqm<Ld, Vd>& d) {
    if constexpr (Va * Vb + Vc * Vd > FQ_PROD_MAX) {  // reduce the operand of the largest bound
        constexpr int m = imax(imax(Va, Vb), imax(Vc, Vd));
        if constexpr (Va == m) return fq_mul2(fq_reduce(a), b, c, d);
        else if constexpr (Vb == m) return fq_mul2(a, fq_reduce(b), c, d);
        else if constexpr (Vc == m) return fq_mul2(a, b, fq_reduce(c), d);
        else return fq_mul2(a, b, c, fq_reduce(d));
    } else if constexpr (La * Lb + Lc * Ld > 6) {
        return fq_mul2(fq_normalize(a), fq_normalize(b), fq_normalize(c), fq_normalize(d));
    } else {
        GSV_OPC(gsv::OPC_BN_MUL);
        GSV_OPC(gsv::OPC_BN_MUL);
        GSV_OPC(gsv::OPC_BN_REDC);
        fqm<1, (Va * Vb + Vc * Vd) / 168 + 2> r;
        fq_redc_core<true>(r.v, a.v, b.v, c.v, d.v);
        return r;
    }
}

// REDC(sum_t a_t b_t) over N products with one reduction (N <= 6 when every operand is normalised:
// the column bound is sum_t La_t Lb_t <= 6).  The F_p^6 product's output coordinates are such sums
// (three F_p^2 products each), so it needs 6 reductions instead of 12 and no intermediate additions.
template <int N>
FQ_FN void fq_redc_n(uint32_t r[9], const uint32_t (&a)[N][9], const uint32_t (&b)[N][9]) {
#if defined(BN9_ASM)
    fq_redc_asm<N>(r, a, b);
    return;
#endif
    uint32_t m[9];
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 17; k++) {
#pragma unroll
        for (int t = 0; t < N; t++) {
#pragma unroll
            for (int i = 0; i < 9; i++) {
                int j = k - i;
                if (j >= 0 && j < 9) acc += (uint64_t)a[t][i] * b[t][j];
            }
        }
#pragma unroll
        for (int i = 0; i < 9; i++) {
            int j = k - i;
            if (i < k && j >= 0 && j < 9) acc += (uint64_t)m[i] * FQ_P[j];
        }
        if (k < 9) {
            m[k] = ((uint32_t)acc * FQ_N0) & FQ_M29;
            acc += (uint64_t)m[k] * FQ_P[0];
        } else {
            r[k - 9] = (uint32_t)acc & FQ_M29;
        }
        acc >>= 29;
    }
    r[8] = (uint32_t)acc;
}
template <class T>
struct fq_traits;
template <int L, int V>
struct fq_traits<fqm<L, V>> {
    static constexpr int l = L, v = V;
};
// fq_dot(a0, b0, a1, b1, ...) = (a0 b0 + a1 b1 + ...) R^-1: operands' bounds checked at compile time
template <class... T>
FQ_FN auto fq_dot(const T&... xs) {
    constexpr int N = (int)sizeof...(T) / 2;
    constexpr int Ls[] = {fq_traits<T>::l...};
    constexpr int Vs[] = {fq_traits<T>::v...};
    constexpr int LL = [&] { int s = 0; for (int t = 0; t < N; t++) s += Ls[2 * t] * Ls[2 * t + 1]; return s; }();
    constexpr int S = [&] { int s = 0; for (int t = 0; t < N; t++) s += Vs[2 * t] * Vs[2 * t + 1]; return s; }();
    static_assert(2 * N == (int)sizeof...(T) && LL <= 6 && S <= FQ_PROD_MAX, "fq_dot operand bounds");
    const uint32_t* p[] = {xs.v...};
    uint32_t A[N][9], B[N][9];
#pragma unroll
    for (int t = 0; t < N; t++) {
        GSV_OPC(gsv::OPC_BN_MUL);
#pragma unroll
        for (int i = 0; i < 9; i++) {
            A[t][i] = p[2 * t][i];
            B[t][i] = p[2 * t + 1][i];
        }
    }
    GSV_OPC(gsv::OPC_BN_REDC);
    fqm<1, S / 168 + 2> r;
    fq_redc_n<N>(r.v, A, B);
    return r;
}

// ---------------------------------------------------------------------------- conversions / tests
FQ_FN fqm<1, 1> fq_const(const uint32_t c[9]) {
    fqm<1, 1> r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] = c[i];
    return r;
}
FQ_FN fq fq_zero() { return fq{{0, 0, 0, 0, 0, 0, 0, 0, 0}}; }
FQ_FN fq fq_one() { return fq_store(fq_const(FQ_ONE)); }
// 8 x 32-bit little-endian words (value < 2^256) -> limbs
FQ_FN fqm<1, 6> fq_from_words(const uint32_t w[8]) {
    fqm<1, 6> r;  // < 2^256 < 6p
#pragma unroll
    for (int i = 0; i < 9; i++) {
        int bit = 29 * i, wi = bit >> 5, sh = bit & 31;
        uint32_t lo = w[wi] >> sh;
        uint32_t hi = (sh > 3 && wi + 1 < 8) ? (w[wi + 1] << (32 - sh)) : 0u;
        r.v[i] = (lo | hi) & FQ_M29;
    }
    return r;
}
// canonical limbs -> 8 words
FQ_FN void fq_to_words(uint32_t w[8], const fqm<1, 1>& a) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
        int bit = 32 * j, li = bit / 29, sh = bit % 29;
        uint32_t x = a.v[li] >> sh;
        if (li + 1 < 9) x |= a.v[li + 1] << (29 - sh);
        if (sh > 26 && li + 2 < 9) x |= a.v[li + 2] << (58 - sh);
        w[j] = x;
    }
}
template <int L, int V>
FQ_FN bool fq_is_zero(const fqm<L, V>& a) {
    fqm<1, 1> c = fq_canon(a);
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) o |= c.v[i];
    return o == 0;
}
template <int La, int Va, int Lb, int Vb>
FQ_FN bool fq_eq(const fqm<La, Va>& a, const fqm<Lb, Vb>& b) {
    return fq_is_zero(fq_sub(a, b));
}

// a bound is an upper bound: an element satisfies any larger one
template <int L2, int V2, int L, int V>
FQ_FN fqm<L2, V2> fq_widen(const fqm<L, V>& a) {
    static_assert(L2 >= L && V2 >= V, "fq_widen narrows");
    fqm<L2, V2> r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] = a.v[i];
    return r;
}

// ============================================================================ F_p^2 (gfp2.go): x i + y
template <int L, int V>
struct fp2m {
    fqm<L, V> x, y;
};
using fp2 = fp2m<1, VS>;

// two coordinates of (possibly) different bounds -> one F_p^2 element of their common bound
template <class TX, class TY>
FQ_FN auto fp2_of(const TX& x, const TY& y) {
    constexpr int l = imax(fq_traits<TX>::l, fq_traits<TY>::l), v = imax(fq_traits<TX>::v, fq_traits<TY>::v);
    return fp2m<l, v>{fq_widen<l, v>(x), fq_widen<l, v>(y)};
}
template <int L, int V>
FQ_FN fp2 fp2_store(const fp2m<L, V>& a) { return fp2{fq_store(a.x), fq_store(a.y)}; }
FQ_FN fp2 fp2_zero() { return fp2{fq_zero(), fq_zero()}; }
FQ_FN fp2 fp2_one() { return fp2{fq_zero(), fq_one()}; }
FQ_FN fp2 fp2_const(const uint32_t x[9], const uint32_t y[9]) {
    return fp2{fq_store(fq_const(x)), fq_store(fq_const(y))};
}
template <int L, int V>
FQ_FN bool fp2_is_zero(const fp2m<L, V>& a) { return fq_is_zero(a.x) && fq_is_zero(a.y); }
template <int La, int Va, int Lb, int Vb>
FQ_FN bool fp2_eq(const fp2m<La, Va>& a, const fp2m<Lb, Vb>& b) { return fq_eq(a.x, b.x) && fq_eq(a.y, b.y); }

template <int La, int Va, int Lb, int Vb>
FQ_FN auto fp2_add(const fp2m<La, Va>& a, const fp2m<Lb, Vb>& b) { return fp2_of(fq_add(a.x, b.x), fq_add(a.y, b.y)); }
template <int La, int Va, int Lb, int Vb>
FQ_FN auto fp2_sub(const fp2m<La, Va>& a, const fp2m<Lb, Vb>& b) { return fp2_of(fq_sub(a.x, b.x), fq_sub(a.y, b.y)); }
template <int L, int V>
FQ_FN auto fp2_neg(const fp2m<L, V>& a) { return fp2_of(fq_neg(a.x), fq_neg(a.y)); }
template <int L, int V>
FQ_FN auto fp2_dbl(const fp2m<L, V>& a) { return fp2_add(a, a); }
// conj(x i + y) = -x i + y (gfp2.go:53-57)
template <int L, int V>
FQ_FN auto fp2_conj(const fp2m<L, V>& a) { return fp2_of(fq_neg(a.x), a.y); }
template <int K, int L, int V>
FQ_FN auto fp2_mul_small(const fp2m<L, V>& a) { return fp2_of(fq_mul_small<K>(a.x), fq_mul_small<K>(a.y)); }
template <int L, int V>
FQ_FN auto fp2_normalize(const fp2m<L, V>& a) { return fp2_of(fq_normalize(a.x), fq_normalize(a.y)); }
template <int L, int V>
FQ_FN void fp2_cmov(fp2& r, const fp2m<L, V>& a, bool f) {
    fp2 t = fp2_store(a);
    fq_cmov(r.x, t.x, f);
    fq_cmov(r.y, t.y, f);
}

// gfp2.go:83-98: (ax i + ay)(bx i + by) = (ax by + ay bx) i + (ay by - ax bx), each coordinate one
// dual Montgomery product
template <int La, int Va, int Lb, int Vb>
FQ_FN auto fp2_mul(const fp2m<La, Va>& a, const fp2m<Lb, Vb>& b) {
    if constexpr (La * Lb > 2) {  // (La Lb + La (Lb + 1)) <= 6 for the y product
        if constexpr (La >= Lb) return fp2_mul(fp2_normalize(a), b);
        else return fp2_mul(a, fp2_normalize(b));
    } else {
        auto x = fq_mul2(a.x, b.y, a.y, b.x);
        auto y = fq_mul2(a.y, b.y, a.x, fq_neg(b.x));
        return fp2_of(x, y);
    }
}
// gfp2.go:130-143: (x i + y)^2 = 2xy i + (y - x)(y + x)
template <int L, int V>
FQ_FN auto fp2_sqr(const fp2m<L, V>& a) {
    if constexpr (L > 1) {
        return fp2_sqr(fp2_normalize(a));
    } else {
        auto x = fq_mul(fq_add(a.x, a.x), a.y);
        auto y = fq_mul(fq_sub(a.y, a.x), fq_add(a.y, a.x));
        return fp2_of(x, y);
    }
}
template <int La, int Va, int Lb, int Vb>
FQ_FN auto fp2_mul_fp(const fp2m<La, Va>& a, const fqm<Lb, Vb>& b) { return fp2_of(fq_mul(a.x, b), fq_mul(a.y, b)); }
// gfp2.go:107-128: (x i + y)(i + 9) = (9x + y) i + (9y - x)
template <int L, int V>
FQ_FN auto fp2_mul_xi(const fp2m<L, V>& a) {
    if constexpr (L > 1 || V > 12) {
        return fp2_mul_xi(fp2_of(fq_fit<1, 12>(a.x), fq_fit<1, 12>(a.y)));
    } else {
        auto x = fq_add(fq_add(fq_normalize(fq_mul_small<8>(a.x)), a.x), a.y);
        auto y = fq_sub(fq_add(fq_normalize(fq_mul_small<8>(a.y)), a.y), a.x);
        return fp2_of(x, y);
    }
}

// ============================================================================ inversion
// (aR)^-1 by safegcd (modinv30.cuh, the BN254 prime) times R^3 by one Montgomery product: a^-1 R, the
// inverse the reference computes as a^(p-2) (gfp.go:31-49)
}  // namespace bn
}  // namespace gsv
#include "modinv30.cuh"
namespace gsv {
namespace bn {
template <int L, int V>
FQ_FN fq fq_inv(const fqm<L, V>& a) {
    uint32_t w[8], iw[8];
    fq_to_words(w, fq_canon(a));
    modinv30_words(iw, w, MI30_BN);
    return fq_store(fq_mul(fq_from_words(iw), fq_const(FQ_R3)));
}
// gfp2.go:145-156
template <int L, int V>
FQ_FN fp2 fp2_inv(const fp2m<L, V>& a) {
    auto n = fq_add(fq_mul(a.x, a.x), fq_mul(a.y, a.y));
    fq inv = fq_inv(n);
    return fp2_store(fp2_of(fq_mul(fq_neg(a.x), inv), fq_mul(a.y, inv)));
}

// ============================================================================ F_p^6 (gfp6.go): x tau^2 + y tau + z
// fp6t<E>: coordinates of F_p^2 type E (lazy bounds); fp6 is the stored form
template <class E>
struct fp6t {
    E x, y, z;
};
using fp6 = fp6t<fp2>;
template <class T>
struct fp2_traits;
template <int L, int V>
struct fp2_traits<fp2m<L, V>> {
    static constexpr int l = L, v = V;
};
template <int L2, int V2, int L, int V>
FQ_FN fp2m<L2, V2> fp2_widen(const fp2m<L, V>& a) { return fp2m<L2, V2>{fq_widen<L2, V2>(a.x), fq_widen<L2, V2>(a.y)}; }
// three coordinates -> one F_p^6 element of their common bound
template <class X, class Y, class Z>
FQ_FN auto fp6_of(const X& x, const Y& y, const Z& z) {
    constexpr int l = imax(imax(fp2_traits<X>::l, fp2_traits<Y>::l), fp2_traits<Z>::l);
    constexpr int v = imax(imax(fp2_traits<X>::v, fp2_traits<Y>::v), fp2_traits<Z>::v);
    return fp6t<fp2m<l, v>>{fp2_widen<l, v>(x), fp2_widen<l, v>(y), fp2_widen<l, v>(z)};
}
template <class E>
FQ_FN fp6 fp6_store(const fp6t<E>& a) { return fp6{fp2_store(a.x), fp2_store(a.y), fp2_store(a.z)}; }
template <class E>
FQ_FN auto fp6_normalize(const fp6t<E>& a) { return fp6_of(fp2_normalize(a.x), fp2_normalize(a.y), fp2_normalize(a.z)); }
FQ_FN fp6 fp6_zero() { return fp6{fp2_zero(), fp2_zero(), fp2_zero()}; }
FQ_FN fp6 fp6_one() { return fp6{fp2_zero(), fp2_zero(), fp2_one()}; }
template <class A>
FQ_FN auto fp6_neg(const fp6t<A>& a) { return fp6_of(fp2_neg(a.x), fp2_neg(a.y), fp2_neg(a.z)); }
template <class A, class B>
FQ_FN auto fp6_add(const fp6t<A>& a, const fp6t<B>& b) {
    return fp6_of(fp2_add(a.x, b.x), fp2_add(a.y, b.y), fp2_add(a.z, b.z));
}
template <class A, class B>
FQ_FN auto fp6_sub(const fp6t<A>& a, const fp6t<B>& b) {
    return fp6_of(fp2_sub(a.x, b.x), fp2_sub(a.y, b.y), fp2_sub(a.z, b.z));
}
// gfp6.go:140-149: tau (x tau^2 + y tau + z) = y tau^2 + z tau + x xi
template <class A>
FQ_FN auto fp6_mul_tau(const fp6t<A>& a) { return fp6_of(a.y, a.z, fp2_mul_xi(a.x)); }

// gfp6.go:96-123.  The reference's product, with each output coordinate's three F_p^2 products
// summed before one reduction (fq_dot over six F_p products per F_p coordinate): with u = a.i,
// v = b.j, [u v] = (ux vy + uy vx) i + (uy vy + (-ux) vx), and xi folded into b:
//   c.x = a.x b.z + a.y b.y + a.z b.x,  c.y = a.y b.z + a.z b.y + a.x (xi b.x),
//   c.z = a.z b.z + a.x (xi b.y) + a.y (xi b.x).
// Operands are brought to limb bound 1 (normalised) and, if their value bounds would overflow the
// six-term sum, reduced.
template <class A, class B>
FQ_FN auto fp6_mul(const fp6t<A>& a_, const fp6t<B>& b_) {
    constexpr int va = fp2_traits<A>::v, vb = fp2_traits<B>::v;
    if constexpr (6 * va * (vb + 2) > FQ_PROD_MAX || 6 * va * 34 > FQ_PROD_MAX) {
        if constexpr (va >= vb) return fp6_mul(fp6_of(fp2_of(fq_reduce(a_.x.x), fq_reduce(a_.x.y)), fp2_of(fq_reduce(a_.y.x), fq_reduce(a_.y.y)), fp2_of(fq_reduce(a_.z.x), fq_reduce(a_.z.y))), b_);
        else return fp6_mul(a_, fp6_of(fp2_of(fq_reduce(b_.x.x), fq_reduce(b_.x.y)), fp2_of(fq_reduce(b_.y.x), fq_reduce(b_.y.y)), fp2_of(fq_reduce(b_.z.x), fq_reduce(b_.z.y))));
    } else {
        auto a = fp6_normalize(a_);
        auto b = fp6_normalize(b_);
        auto nax = fq_normalize(fq_neg(a.x.x)), nay = fq_normalize(fq_neg(a.y.x)), naz = fq_normalize(fq_neg(a.z.x));
        auto xbx = fp2_normalize(fp2_mul_xi(b.x)), xby = fp2_normalize(fp2_mul_xi(b.y));
        auto cxx = fq_dot(a.x.x, b.z.y, a.x.y, b.z.x, a.y.x, b.y.y, a.y.y, b.y.x, a.z.x, b.x.y, a.z.y, b.x.x);
        auto cxy = fq_dot(a.x.y, b.z.y, nax, b.z.x, a.y.y, b.y.y, nay, b.y.x, a.z.y, b.x.y, naz, b.x.x);
        auto cyx = fq_dot(a.y.x, b.z.y, a.y.y, b.z.x, a.z.x, b.y.y, a.z.y, b.y.x, a.x.x, xbx.y, a.x.y, xbx.x);
        auto cyy = fq_dot(a.y.y, b.z.y, nay, b.z.x, a.z.y, b.y.y, naz, b.y.x, a.x.y, xbx.y, nax, xbx.x);
        auto czx = fq_dot(a.z.x, b.z.y, a.z.y, b.z.x, a.x.x, xby.y, a.x.y, xby.x, a.y.x, xbx.y, a.y.y, xbx.x);
        auto czy = fq_dot(a.z.y, b.z.y, naz, b.z.x, a.x.y, xby.y, nax, xby.x, a.y.y, xbx.y, nay, xbx.x);
        return fp6_of(fp2_of(cxx, cxy), fp2_of(cyx, cyy), fp2_of(czx, czy));
    }
}
// a * (by tau + bz): a line's sparse factor (x coefficient 0), four F_p products per coordinate:
//   c.x = a.x bz + a.y by,  c.y = a.y bz + a.z by,  c.z = a.z bz + a.x (xi by)
template <class A, int L1, int V1, int L2, int V2>
FQ_FN auto fp6_mul_sparse(const fp6t<A>& a_, const fp2m<L1, V1>& by_, const fp2m<L2, V2>& bz_) {
    constexpr int va = fp2_traits<A>::v, vb = imax(imax(V1, V2), 34);
    if constexpr (4 * va * (vb + 2) > FQ_PROD_MAX) {
        return fp6_mul_sparse(fp6_of(fp2_of(fq_reduce(a_.x.x), fq_reduce(a_.x.y)), fp2_of(fq_reduce(a_.y.x), fq_reduce(a_.y.y)), fp2_of(fq_reduce(a_.z.x), fq_reduce(a_.z.y))), by_, bz_);
    } else {
        auto a = fp6_normalize(a_);
        auto by = fp2_normalize(by_);
        auto bz = fp2_normalize(bz_);
        auto nax = fq_normalize(fq_neg(a.x.x)), nay = fq_normalize(fq_neg(a.y.x)), naz = fq_normalize(fq_neg(a.z.x));
        auto xby = fp2_normalize(fp2_mul_xi(by));
        auto cxx = fq_dot(a.x.x, bz.y, a.x.y, bz.x, a.y.x, by.y, a.y.y, by.x);
        auto cxy = fq_dot(a.x.y, bz.y, nax, bz.x, a.y.y, by.y, nay, by.x);
        auto cyx = fq_dot(a.y.x, bz.y, a.y.y, bz.x, a.z.x, by.y, a.z.y, by.x);
        auto cyy = fq_dot(a.y.y, bz.y, nay, bz.x, a.z.y, by.y, naz, by.x);
        auto czx = fq_dot(a.z.x, bz.y, a.z.y, bz.x, a.x.x, xby.y, a.x.y, xby.x);
        auto czy = fq_dot(a.z.y, bz.y, naz, bz.x, a.x.y, xby.y, nax, xby.x);
        return fp6_of(fp2_of(cxx, cxy), fp2_of(cyx, cyy), fp2_of(czx, czy));
    }
}
template <class A, int L, int V>
FQ_FN auto fp6_mul_fp2(const fp6t<A>& a, const fp2m<L, V>& b) {
    return fp6_of(fp2_mul(a.x, b), fp2_mul(a.y, b), fp2_mul(a.z, b));
}
template <class A, int L, int V>
FQ_FN auto fp6_mul_fp(const fp6t<A>& a, const fqm<L, V>& b) {
    return fp6_of(fp2_mul_fp(a.x, b), fp2_mul_fp(a.y, b), fp2_mul_fp(a.z, b));
}
template <class A>
FQ_FN auto fp6_sqr(const fp6t<A>& a) { return fp6_mul(a, a); }
// gfp6.go:54-62
FQ_FN fp6 fp6_frob(const fp6& a) {
    return fp6{fp2_store(fp2_mul(fp2_conj(a.x), fp2_const(FQ_XI_2P2_3_X, FQ_XI_2P2_3_Y))),
               fp2_store(fp2_mul(fp2_conj(a.y), fp2_const(FQ_XI_P1_3_X, FQ_XI_P1_3_Y))), fp2_store(fp2_conj(a.z))};
}
// gfp6.go:65-73
FQ_FN fp6 fp6_frob_p2(const fp6& a) {
    return fp6{fp2_store(fp2_mul_fp(a.x, fq_const(FQ_XI_2PSQ2_3))), fp2_store(fp2_mul_fp(a.y, fq_const(FQ_XI_PSQ1_3))),
               a.z};
}
// gfp6.go:172-213
FQ_FN fp6 fp6_inv(const fp6& a) {
    fp2 A = fp2_store(fp2_sub(fp2_sqr(a.z), fp2_mul_xi(fp2_mul(a.x, a.y))));
    fp2 B = fp2_store(fp2_sub(fp2_mul_xi(fp2_sqr(a.x)), fp2_mul(a.y, a.z)));
    fp2 C = fp2_store(fp2_sub(fp2_sqr(a.y), fp2_mul(a.x, a.z)));
    fp2 F = fp2_store(fp2_add(fp2_add(fp2_mul_xi(fp2_mul(C, a.y)), fp2_mul(A, a.z)), fp2_mul_xi(fp2_mul(B, a.x))));
    F = fp2_inv(F);
    return fp6{fp2_store(fp2_mul(C, F)), fp2_store(fp2_mul(B, F)), fp2_store(fp2_mul(A, F))};
}

}  // namespace bn
}  // namespace gsv

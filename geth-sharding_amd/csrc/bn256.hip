// Batched BN254 PairingCheck on gfx950 (bn256.PairingCheck as driven by the bn256Pairing
// precompile, core/vm/contracts.go:333-360; crypto/bn256/cloudflare/bn256.go:313-327).
//
// One lane per pair for decode + G2 subgroup check, one lane per check for the multi-Miller loop
// and the final exponentiation.  Three launches:
//   k_bn_lines    (or k_bn_lines_w2, large batches) one lane per pair:
//                 (0) decode the 192-byte pair (bn256.go:120-164 G1.Unmarshal, :256-306 G2.Unmarshal):
//                 coordinates < p, Montgomery encode, infinity detection, y^2 = x^3 + 3 on G1,
//                 on-twist + subgroup membership on G2 (twist.go:47-63)  -> pair status + points;
//                 (1) the pair's 91 Miller-loop lines (optate.go:3-92, 122-210: the twist point's
//                 doubling / addition steps evaluated at P)                  -> line coefficients
//   k_bn_miller   optimal-ate Miller loop (optate.go:122-210) over all of a check's pairs with one
//                 shared accumulator (the product of the per-pair values), multiplying in the
//                 precomputed lines                                          -> F_p^12 per check
//   k_bn_final    finalExponentiation (optate.go:212-261), IsOne          -> verdict per check
// The field arithmetic is bn254_fe9.cuh: 9 x 29-bit limbs, Montgomery R = 2^261, lazily reduced —
// elements are congruent to, not equal to, the reference's gfP words, so every decision (equality,
// zero, IsOne) and every value leaving the kernels goes through the canonical residue (fq_canon).
// Tower and curve formulas restate crypto/bn256/cloudflare/{gfp12,twist,curve,optate}.go operation
// for operation (file:line at each function).
// HBM layout is structure-of-arrays, word-major ([word][pair]), so each lane's word loads and
// stores coalesce across the wave.
#include "opcount.cuh"
#include "bn254_fe9.cuh"
#include "gsv_internal.h"
#include "keccak_dev.cuh"

namespace gsv {
namespace bn {

#ifndef GSV_DI
#define GSV_DI __device__ __forceinline__
#endif

// p as eight little-endian 32-bit words (constants.go:31 P)
__device__ constexpr uint32_t BN_P_W[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                           0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
// sixuPlus2NAF (optate.go:114-118) digits 0..63 as two bit masks (digit 64 is the leading 1)
constexpr uint64_t NAF_POS = 0xa1818041c0864428ULL;  // bit i set where digit i == +1
constexpr uint64_t NAF_NEG = 0x0408100802100880ULL;  // bit i set where digit i == -1
// NAF of u (constants.go:17): u = U_NAF_POS - U_NAF_NEG, digit 62 = +1
constexpr uint64_t U_NAF_POS = 0x450a14044a890a01ULL;
constexpr uint64_t U_NAF_NEG = 0x0020815000200010ULL;

struct fp12 { fp6 x, y; };        // x*omega + y (gfp12.go)
struct g1a { fq x, y; };          // affine G1 point (Montgomery)
struct g2a { fp2 x, y; };         // affine G2 point
struct g2j { fp2 x, y, z, t; };   // twistPoint (Jacobian, t = z^2 where maintained)

template <class T>
GSV_DI fp2 s2(const T& a) { return fp2_store(a); }
GSV_DI fq fq_c(const uint32_t c[9]) { return fq_store(fq_const(c)); }

// F_p^6 products of the F_p^12 routines (inline; one out-of-line copy per operand type pair measured
// no better, r02)
template <class A, class B>
GSV_DI auto fp6_mulx(const fp6t<A>& a, const fp6t<B>& b) {
    return fp6_mul(a, b);
}

// ---------------------------------------------------------------- F_p^12 (gfp12.go)
GSV_DI fp12 fp12_one() { return fp12{fp6_zero(), fp6_one()}; }
// IsOne (gfp12.go:34-37) on canonical residues: y.z.y == R mod p (one), everything else zero
GSV_DI bool fp12_is_one(const fp12& e) {
    int z = (int)fp2_is_zero(e.x.x) & (int)fp2_is_zero(e.x.y) & (int)fp2_is_zero(e.x.z) & (int)fp2_is_zero(e.y.x) &
            (int)fp2_is_zero(e.y.y) & (int)fq_is_zero(e.y.z.x);
    return (z & (int)fq_eq(e.y.z.y, fq_const(FQ_ONE))) != 0;
}
GSV_DI fp12 fp12_conj(const fp12& a) { return fp12{fp6_store(fp6_neg(a.x)), a.y}; }
// gfp12.go:94-106.  Karatsuba over F_p^6: x = (a.x + a.y)(b.x + b.y) - a.x b.x - a.y b.y equals the
// reference's a.x b.y + b.x a.y (3 F_p^6 products instead of 4, the same field element).
GSV_DI fp12 fp12_mul_i(const fp12& a, const fp12& b) {
    auto v0 = fp6_mulx(a.x, b.x);
    auto v1 = fp6_mulx(a.y, b.y);
    fp6 tx = fp6_store(fp6_sub(fp6_sub(fp6_mulx(fp6_add(a.x, a.y), fp6_add(b.x, b.y)), v0), v1));
    return fp12{tx, fp6_store(fp6_add(v1, fp6_mul_tau(v0)))};
}
// gfp12.go:129-143
GSV_DI fp12 fp12_sqr_i(const fp12& a) {
    fp6 v0 = fp6_store(fp6_mulx(a.x, a.y));
    auto t = fp6_add(fp6_mul_tau(a.x), a.y);
    fp6 ty = fp6_store(fp6_sub(fp6_sub(fp6_mulx(fp6_add(a.x, a.y), t), v0), fp6_mul_tau(v0)));
    return fp12{fp6_store(fp6_add(v0, v0)), ty};
}
// Squaring in the cyclotomic subgroup (Granger-Scott, "Faster squaring in the cyclotomic subgroup of
// sixth degree extensions", PKC 2010): 9 F_p^2 squarings instead of two F_p^6 products.  Valid for
// every element of norm 1 over F_p^6 — everything finalExponentiation squares after its easy part
// (optate.go:218-222) — and it yields the same field element as fp12_sqr there.  Coefficients of
// a = sum c_k w^k over F_p^2 (w^2 = tau, tau^3 = xi): c0 = y.z, c1 = x.z, c2 = y.y, c3 = x.y,
// c4 = y.x, c5 = x.x.  One coefficient pair (p, q) gives sq = p^2 xi + q^2 and tc = 2 p q.
// The inputs are reduced once (value < 3p), so every product below has a tiny output bound and
// only the outputs c0', c2', c4' (and c1' after its xi factor) need a reduction when stored.
struct cyc_pair { fp2 lo, hi; };
using fp2r = fp2m<1, 3>;
template <int L, int V>
GSV_DI fp2r fp2_reduce(const fp2m<L, V>& a) { return fp2r{fq_reduce(a.x), fq_reduce(a.y)}; }
// 2 p q by two dual products: x = 2(px qy + py qx), y = 2(py qy - px qx)
GSV_DI auto fp2_mul2x(const fp2r& p, const fp2r& q) {
    auto px2 = fq_add(p.x, p.x), py2 = fq_add(p.y, p.y);
    return fp2_of(fq_dot(px2, q.y, py2, q.x), fq_dot(py2, q.y, px2, fq_neg(q.x)));
}
template <bool XI_TC>
GSV_DI cyc_pair cyclo_pair(const fp2r& p, const fp2r& q, const fp2r& m1, const fp2r& m2) {
    auto sq = fp2_add(fp2_mul_xi(fp2_sqr(p)), fp2_sqr(q));  // p^2 xi + q^2
    auto tc = fp2_mul2x(p, q);                               // 2 p q
    cyc_pair r;
    r.lo = s2(fp2_add(fp2_dbl(fp2_sub(sq, m1)), sq));        // 3 sq - 2 m1
    if constexpr (XI_TC) {
        auto tcx = fp2_mul_xi(tc);
        r.hi = s2(fp2_add(fp2_dbl(fp2_add(tcx, m2)), tcx));  // 3 xi tc + 2 m2
    } else {
        r.hi = s2(fp2_add(fp2_dbl(fp2_add(tc, m2)), tc));    // 3 tc + 2 m2
    }
    return r;
}
GSV_DI fp12 fp12_cyclo_sqr_i(const fp12& a) {
    fp2r x0 = fp2_reduce(a.y.z), x1 = fp2_reduce(a.y.y), x2 = fp2_reduce(a.y.x);
    fp2r x3 = fp2_reduce(a.x.z), x4 = fp2_reduce(a.x.y), x5 = fp2_reduce(a.x.x);
    cyc_pair r0 = cyclo_pair<false>(x4, x0, x0, x4);  // c0', c3'
    cyc_pair r1 = cyclo_pair<false>(x2, x3, x1, x5);  // c2', c5'
    cyc_pair r2 = cyclo_pair<true>(x5, x1, x2, x3);   // c4', c1'
    fp12 e;
    e.y.z = r0.lo;
    e.x.y = r0.hi;
    e.y.y = r1.lo;
    e.x.x = r1.hi;
    e.y.x = r2.lo;
    e.x.z = r2.hi;
    return e;
}
// ---- three-lane cooperative F_p^12 operations (k_bn_final3), for batches too small to give every
// SIMD a wave.  The three lanes of a triple (wave lanes base, base+1, base+2) all hold the whole F_p^12
// value; each operation is split into three equal parts selected by the lane's role (same instruction
// stream, different operands: no divergence), and the parts are exchanged with ds_bpermute.  The
// dependent chain per step becomes a third as long; every part computes the same formula as the
// one-lane routine, so results are the same field elements.
GSV_DI uint32_t bperm(uint32_t v, int lane) { return (uint32_t)__builtin_amdgcn_ds_bpermute(lane << 2, (int)v); }
template <class T>
GSV_DI void gather3(T out[3], const T& mine, int base) {  // out[r] = lane (base + r)'s `mine`
    static_assert(sizeof(T) % 4 == 0, "word-sized");
    const uint32_t* m = (const uint32_t*)&mine;
#pragma unroll
    for (int r = 0; r < 3; r++) {
        uint32_t* o = (uint32_t*)&out[r];
#pragma unroll
        for (int w = 0; w < (int)(sizeof(T) / 4); w++) o[w] = bperm(m[w], base + r);
    }
}
// fp12_cyclo_sqr_i split by coefficient pairs: role 0 squares (x4, x0) and yields c0', c3'; role 1
// (x2, x3) -> c2', c5'; role 2 (x5, x1) -> c4', c1'
GSV_DI void fp12_cyclo_sqr3_i(fp12* pe, const fp12& a, int role, int base) {
    const fp2 &x0 = a.y.z, &x1 = a.y.y, &x2 = a.y.x, &x3 = a.x.z, &x4 = a.x.y, &x5 = a.x.x;
    fp2r p = fp2_reduce(role == 0 ? x4 : role == 1 ? x2 : x5);
    fp2r q = fp2_reduce(role == 0 ? x0 : role == 1 ? x3 : x1);
    fp2r m1 = fp2_reduce(role == 0 ? x0 : role == 1 ? x1 : x2);
    fp2r m2 = fp2_reduce(role == 0 ? x4 : role == 1 ? x5 : x3);
    // the xi factor on tc only for role 2, as a select after the shared formula
    auto sq = fp2_add(fp2_mul_xi(fp2_sqr(p)), fp2_sqr(q));
    fp2 tc = s2(fp2_mul2x(p, q));
    fp2 tcx = s2(fp2_mul_xi(tc));
    if (role == 2) tc = tcx;
    cyc_pair mine, all[3];
    mine.lo = s2(fp2_add(fp2_dbl(fp2_sub(sq, m1)), sq));
    mine.hi = s2(fp2_add(fp2_dbl(fp2_add(tc, m2)), tc));
    gather3(all, mine, base);
    pe->y.z = all[0].lo;
    pe->x.y = all[0].hi;
    pe->y.y = all[1].lo;
    pe->x.x = all[1].hi;
    pe->y.x = all[2].lo;
    pe->x.z = all[2].hi;
}
// ---------------------------------------------------------------- twist points (twist.go)
// twist.go:136-162 dbl-2009-l (t is not updated, as in the reference)
GSV_DI g2j g2_double_i(const g2j& a) {
    fp2 A = s2(fp2_sqr(a.x));
    fp2 B = s2(fp2_sqr(a.y));
    fp2 C = s2(fp2_sqr(B));
    fp2 d = s2(fp2_dbl(fp2_sub(fp2_sub(fp2_sqr(fp2_add(a.x, B)), A), C)));
    fp2 e = s2(fp2_add(fp2_dbl(A), A));
    auto f = fp2_sqr(e);
    g2j r;
    r.x = s2(fp2_sub(f, fp2_dbl(d)));
    r.y = s2(fp2_sub(fp2_mul(e, fp2_sub(d, r.x)), fp2_mul_small<8>(C)));
    r.z = s2(fp2_dbl(fp2_mul(a.y, a.z)));
    r.t = a.t;
    return r;
}
static BN_NI void g2_double_p(g2j* pc, const g2j* pa) { *pc = g2_double_i(*pa); }
// twist.go:73-134 add-2007-bl with its infinity / doubling cases
GSV_DI g2j g2_add_i(const g2j& a, const g2j& b) {
    if (fp2_is_zero(a.z)) return b;
    if (fp2_is_zero(b.z)) return a;
    fp2 z12 = s2(fp2_sqr(a.z));
    fp2 z22 = s2(fp2_sqr(b.z));
    fp2 u1 = s2(fp2_mul(a.x, z22));
    fp2 u2 = s2(fp2_mul(b.x, z12));
    fp2 s1 = s2(fp2_mul(a.y, fp2_mul(b.z, z22)));
    fp2 s2_ = s2(fp2_mul(b.y, fp2_mul(a.z, z12)));
    fp2 h = s2(fp2_sub(u2, u1));
    bool xeq = fp2_is_zero(h);
    fp2 i = s2(fp2_sqr(fp2_dbl(h)));
    fp2 j = s2(fp2_mul(h, i));
    fp2 t = s2(fp2_sub(s2_, s1));
    bool yeq = fp2_is_zero(t);
    if (xeq && yeq) {
        g2j c;
        g2_double_p(&c, &a);
        return c;
    }
    fp2 r = s2(fp2_dbl(t));
    fp2 v = s2(fp2_mul(u1, i));
    g2j o;
    o.x = s2(fp2_sub(fp2_sub(fp2_sqr(r), j), fp2_dbl(v)));
    o.y = s2(fp2_sub(fp2_mul(r, fp2_sub(v, o.x)), fp2_dbl(fp2_mul(s1, j))));
    o.z = s2(fp2_mul(fp2_sub(fp2_sub(fp2_sqr(fp2_add(a.z, b.z)), z12), z22), h));
    o.t = a.t;
    return o;
}
static BN_NI void g2_add_p(g2j* pc, const g2j* pa, const g2j* pb) { *pc = g2_add_i(*pa, *pb); }
// c = a + q with q affine (z = 1): madd-2007-bl, 8M + 3S instead of the general 11M + 5S.  Used only
// inside the subgroup predicate, whose boolean outcome does not depend on the formulas chosen.
GSV_DI g2j g2_add_mixed_i(const g2j& a, const g2a& q) {
    if (fp2_is_zero(a.z)) return g2j{q.x, q.y, fp2_one(), fp2_one()};
    fp2 z12 = s2(fp2_sqr(a.z));
    fp2 u2 = s2(fp2_mul(q.x, z12));
    fp2 s2_ = s2(fp2_mul(q.y, fp2_mul(a.z, z12)));
    fp2 h = s2(fp2_sub(u2, a.x));
    fp2 t = s2(fp2_sub(s2_, a.y));
    if (fp2_is_zero(h) && fp2_is_zero(t)) {  // out of line: never taken on the hot path
        g2j c;
        g2_double_p(&c, &a);
        return c;
    }
    fp2 i = s2(fp2_sqr(fp2_dbl(h)));
    fp2 j = s2(fp2_mul(h, i));
    fp2 r = s2(fp2_dbl(t));
    fp2 v = s2(fp2_mul(a.x, i));
    g2j o;
    o.x = s2(fp2_sub(fp2_sub(fp2_sqr(r), j), fp2_dbl(v)));
    o.y = s2(fp2_sub(fp2_mul(r, fp2_sub(v, o.x)), fp2_dbl(fp2_mul(a.y, j))));
    o.z = s2(fp2_dbl(fp2_mul(a.z, h)));  // (Z1 + H)^2 - Z1^2 - H^2 = 2 Z1 H
    o.t = a.t;
    return o;
}
// psi(X : Y : Z) = (conj(X) xi^((p-1)/3) : conj(Y) xi^((p-1)/2) : conj(Z)) — the p-power
// Frobenius carried through the twist isomorphism (optate.go:173-176 applies it to affine Q)
GSV_DI g2j g2_psi(const g2j& a) {
    g2j o;
    o.x = s2(fp2_mul(fp2_conj(a.x), fp2_const(FQ_XI_P1_3_X, FQ_XI_P1_3_Y)));
    o.y = s2(fp2_mul(fp2_conj(a.y), fp2_const(FQ_XI_P1_2_X, FQ_XI_P1_2_Y)));
    o.z = s2(fp2_conj(a.z));
    o.t = a.t;
    return o;
}
// twist.go:47-58: y^2 == x^3 + 3/xi
GSV_DI bool g2_on_twist(const g2a& q) {
    return fp2_eq(fp2_sqr(q.y), fp2_add(fp2_mul(fp2_sqr(q.x), q.x), fp2_const(FQ_TWIST_B_X, FQ_TWIST_B_Y)));
}
// Subgroup membership from the line chain's own final point (r03).  The lines of a pair leave
// r = [6u+2]Q + psi(Q) - psi^2(Q) (optate.go:122-210: the NAF doublings / additions, then the two
// Frobenius additions), and for every Q on E'(F_p^2) of BN254
//     [r]Q == O (twist.go:60-62)   <=>   r + psi^3(Q) == O.
// On G2, psi acts as [p] and 6u+2 + p - p^2 + p^3 == 0 mod r (the optimal-ate relation).  E'(F_p^2)
// = G2 x H with #H = h = 2p - r coprime to r; psi satisfies psi^2 - t psi + p = 0, so
// f(psi) = 6u+2 + psi - psi^2 + psi^3 = a + b psi with a = p + 6u+2 - tp, b = t^2 - t - p + 1, and
// (a + b psi~)(a + b psi) = a^2 + abt + b^2 p is coprime to h: f(psi) is injective on H, so
// r + psi^3(Q) == O only for Q in G2 (tests/test_g2_frob_relation.py checks these numbers and the
// relation on random points in G2, in H and in neither).  The chain's formulas meet an exceptional
// case (r == +-q at an addition, a 2-torsion r at a doubling) only when they output Z = 0, which every
// later step keeps at 0; that reads as "not in G2", and for Q in G2 no multiple the chain meets is
// +-Q (6u+2 -+ p, 6u+2 + p -+ p^2 are nonzero mod r), so members never get there.  It replaces the
// separate 63-bit psi test of r02 (the ISA-level membership test of Dai-Lin-Zhao-Zhou, eprint 2022/348,
// [u+1]Q + psi([u]Q) + psi^2([u]Q) == psi^3([2u]Q), on a second G2 chain per pair, in check waves beside
// the lines): prepare 10.5 -> 6.5 ms per 65,536 checks (profiles/r03/ab_subfrob.txt).
GSV_DI bool g2_frob_check(const g2j& r, const g2a& Q) {
    fp2 x = Q.x, y = Q.y;
#pragma unroll
    for (int k = 0; k < 3; k++) {  // psi^3(Q) = (x', y'); r == -psi^3(Q) <=> Z != 0, X == x' Z^2, Y == -y' Z^3
        x = s2(fp2_mul(fp2_conj(x), fp2_const(FQ_XI_P1_3_X, FQ_XI_P1_3_Y)));
        y = s2(fp2_mul(fp2_conj(y), fp2_const(FQ_XI_P1_2_X, FQ_XI_P1_2_Y)));
    }
    fp2 z2 = s2(fp2_sqr(r.z));
    return !fp2_is_zero(r.z) && fp2_eq(r.x, fp2_mul(x, z2)) && fp2_eq(fp2_neg(r.y), fp2_mul(y, fp2_mul(z2, r.z)));
}

// ---------------------------------------------------------------- Miller loop (optate.go)
struct line { fp2 a, b, c; };
// optate.go:3-50 (mixed addition r + p, p affine with t = 1; r2 = p.y^2)
GSV_DI line line_add_i(g2j& r, const g2a& p, const g1a& q, const fp2& r2) {
    fp2 B = s2(fp2_mul(p.x, r.t));
    fp2 D = s2(fp2_mul(fp2_sub(fp2_sub(fp2_sqr(fp2_add(p.y, r.z)), r2), r.t), r.t));
    fp2 H = s2(fp2_sub(B, r.x));
    fp2 I = s2(fp2_sqr(H));
    fp2 E = s2(fp2_mul_small<4>(I));
    fp2 J = s2(fp2_mul(H, E));
    fp2 L1 = s2(fp2_sub(D, fp2_dbl(r.y)));
    fp2 V = s2(fp2_mul(r.x, E));
    g2j o;
    o.x = s2(fp2_sub(fp2_sub(fp2_sqr(L1), J), fp2_dbl(V)));
    o.z = s2(fp2_sub(fp2_sub(fp2_sqr(fp2_add(r.z, H)), r.t), I));
    o.y = s2(fp2_sub(fp2_mul(fp2_sub(V, o.x), L1), fp2_dbl(fp2_mul(r.y, J))));
    o.t = s2(fp2_sqr(o.z));
    line l;
    l.a = s2(fp2_sub(fp2_dbl(fp2_mul(L1, p.x)), fp2_sub(fp2_sub(fp2_sqr(fp2_add(p.y, o.z)), r2), o.t)));
    l.c = s2(fp2_mul_fp(fp2_dbl(o.z), q.y));
    l.b = s2(fp2_mul_fp(fp2_dbl(fp2_neg(L1)), q.x));
    r = o;
    return l;
}
// optate.go:52-92
GSV_DI line line_double_i(g2j& r, const g1a& q) {
    fp2 A = s2(fp2_sqr(r.x));
    fp2 B = s2(fp2_sqr(r.y));
    fp2 C = s2(fp2_sqr(B));
    fp2 D = s2(fp2_dbl(fp2_sub(fp2_sub(fp2_sqr(fp2_add(r.x, B)), A), C)));
    fp2 E = s2(fp2_add(fp2_dbl(A), A));
    fp2 G = s2(fp2_sqr(E));
    line l;
    g2j o;
    // optate.go's values in the order that ends each input's life earliest (r.x with l.a, r.y / r.z / B
    // with o.z, r.t with l.b / l.c), against the line role's register pressure
    l.a = s2(fp2_sub(fp2_sub(fp2_sub(fp2_sqr(fp2_add(r.x, E)), A), G), fp2_mul_small<4>(B)));
    o.z = s2(fp2_sub(fp2_sub(fp2_sqr(fp2_add(r.y, r.z)), B), r.t));
    l.b = s2(fp2_mul_fp(fp2_neg(fp2_dbl(fp2_mul(E, r.t))), q.x));
    l.c = s2(fp2_mul_fp(fp2_dbl(fp2_mul(o.z, r.t)), q.y));
    o.x = s2(fp2_sub(G, fp2_dbl(D)));
    o.y = s2(fp2_sub(fp2_mul(fp2_sub(D, o.x), E), fp2_mul_small<8>(C)));
    o.t = s2(fp2_sqr(o.z));
    r = o;
    return l;
}
// optate.go:94-112: ret * (x = (0, a, b), y = (0, 0, c))
GSV_DI void mul_line_i(fp12& ret, const line& l) {
    // ordered (in place) so that at most ret + one F_p^6 temporary + the line are live at a time
    fp6 a2 = fp6_store(fp6_mul_sparse(ret.x, l.a, l.b));  // (0, a, b) * ret.x
    auto s = fp6_add(ret.x, ret.y);                        // ret.x + ret.y
    fp6 t3 = fp6_store(fp6_mul_fp2(ret.y, l.c));
    ret.x = fp6_store(fp6_sub(fp6_sub(fp6_mul_sparse(s, l.a, fp2_add(l.b, l.c)), a2), t3));  // s * (0, a, b + c)
    ret.y = fp6_store(fp6_add(t3, fp6_mul_tau(a2)));
}
static BN_NI void mul_line_p(fp12* ret, const line* l) { mul_line_i(*ret, *l); }

// ---------------------------------------------------------------- SoA helpers
// field element k (of K per item) of item i in a [K*9 words][n] word-major array
GSV_DI fq soa_load(const uint32_t* __restrict__ base, uint32_t n, uint32_t i, int k) {
    fq r;
#pragma unroll
    for (int w = 0; w < 9; w++) r.v[w] = base[(size_t)(k * 9 + w) * n + i];
    return r;
}
GSV_DI void soa_store(uint32_t* __restrict__ base, uint32_t n, uint32_t i, int k, const fq& r) {
#pragma unroll
    for (int w = 0; w < 9; w++) base[(size_t)(k * 9 + w) * n + i] = r.v[w];
}
GSV_DI fp2 soa_load2(const uint32_t* __restrict__ base, uint32_t n, uint32_t i, int k) {
    return fp2{soa_load(base, n, i, k), soa_load(base, n, i, k + 1)};
}
GSV_DI void soa_store2(uint32_t* __restrict__ base, uint32_t n, uint32_t i, int k, const fp2& r) {
    soa_store(base, n, i, k, r.x);
    soa_store(base, n, i, k + 1, r.y);
}
GSV_DI fp12 fp12_load(const uint32_t* base, uint32_t n, uint32_t i) {
    fp12 e;
    fq* f = (fq*)&e;
#pragma unroll
    for (int k = 0; k < 12; k++) f[k] = soa_load(base, n, i, k);
    return e;
}
GSV_DI void fp12_store(uint32_t* base, uint32_t n, uint32_t i, const fp12& e) {
    const fq* f = (const fq*)&e;
#pragma unroll
    for (int k = 0; k < 12; k++) soa_store(base, n, i, k, f[k]);
}
// lines per pair: 64 doublings, one addition per nonzero NAF digit, the two Frobenius additions
constexpr int BN_NLINES = 64 + __builtin_popcountll(NAF_POS | NAF_NEG) + 2;
static_assert(BN_NLINES == 91, "sixuPlus2NAF has 25 nonzero digits below the leading one");
// line li of pair j: 6 F_p elements (a, b, c) in a [BN_NLINES * 54 words][npairs] array
GSV_DI void line_store(uint32_t* __restrict__ lines, uint32_t n, uint32_t j, int li, const line& l) {
    soa_store2(lines, n, j, li * 6 + 0, l.a);
    soa_store2(lines, n, j, li * 6 + 2, l.b);
    soa_store2(lines, n, j, li * 6 + 4, l.c);
}
GSV_DI line line_load(const uint32_t* __restrict__ lines, uint32_t n, uint32_t j, int li) {
    return line{soa_load2(lines, n, j, li * 6 + 0), soa_load2(lines, n, j, li * 6 + 2), soa_load2(lines, n, j, li * 6 + 4)};
}

// gfP.Unmarshal (gfp.go:61-78) + montEncode: big-endian bytes -> Montgomery form (R = 2^261);
// false if the coordinate is >= p
GSV_DI bool fp_unmarshal(fq& r, const uint8_t* p) {
    uint32_t x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint8_t* q = p + 28 - 4 * i;
        x[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
    }
    int64_t br = 0;  // x - p: the final borrow says x < p
#pragma unroll
    for (int i = 0; i < 8; i++) br = ((int64_t)x[i] - (int64_t)BN_P_W[i] + br) >> 32;
    bool ok = br != 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = ok ? x[i] : 0u;
    r = fq_store(fq_mul(fq_from_words(x), fq_const(FQ_R2)));
    return ok;
}
// montDecode + big-endian marshal (gfp.go:51-59): the canonical residue of a R^-1
GSV_DI void fp_marshal(uint8_t* out, const fq& a) {
    fqm<1, 1> one{{1, 0, 0, 0, 0, 0, 0, 0, 0}};
    uint32_t w[8];
    fq_to_words(w, fq_canon(fq_mul(a, one)));
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint32_t x = w[7 - i];
        out[4 * i] = (uint8_t)(x >> 24);
        out[4 * i + 1] = (uint8_t)(x >> 16);
        out[4 * i + 2] = (uint8_t)(x >> 8);
        out[4 * i + 3] = (uint8_t)x;
    }
}

// ---------------------------------------------------------------- kernels
enum : uint8_t { PS_OK = 0, PS_SKIP = 1, PS_BAD = 2 };

// The lines of one pair (optate.go:122-210 for affine Q and P, neither at infinity: the loop's
// doubling / addition steps and the two Frobenius additions), in the order the Miller loop
// multiplies them in.  Lines of an invalid or infinite pair are computed but never used.
GSV_DI g2j pair_lines(uint32_t* __restrict__ lines, uint32_t npairs, uint32_t j, const g1a& P, const g2a& Q) {
    g2j r{Q.x, Q.y, fp2_one(), fp2_one()};
    int li = 0;
    // -Q and r2 = Q.y^2 are formed at each addition step (27 of the 91) instead of living in VGPRs
    // through all of them: 36 fewer registers held against the line role's spills
#pragma unroll 1
    for (int i = 64; i > 0; i--) {
        line_store(lines, npairs, j, li++, line_double_i(r, P));
        uint64_t bit = 1ull << (i - 1);
        if ((NAF_POS | NAF_NEG) & bit) {
            g2a q{Q.x, (NAF_POS & bit) ? Q.y : s2(fp2_neg(Q.y))};
            line_store(lines, npairs, j, li++, line_add_i(r, q, P, s2(fp2_sqr(Q.y))));
        }
    }
    // Q1 = pi(Q), -Q2 = -pi^2(Q) (optate.go:168-209)
    g2a q1{s2(fp2_mul(fp2_conj(Q.x), fp2_const(FQ_XI_P1_3_X, FQ_XI_P1_3_Y))),
           s2(fp2_mul(fp2_conj(Q.y), fp2_const(FQ_XI_P1_2_X, FQ_XI_P1_2_Y)))};
    g2a mq2{s2(fp2_mul_fp(Q.x, fq_const(FQ_XI_PSQ1_3))), Q.y};
    line_store(lines, npairs, j, li++, line_add_i(r, q1, P, s2(fp2_sqr(q1.y))));
    line_store(lines, npairs, j, li, line_add_i(r, mq2, P, s2(fp2_sqr(mq2.y))));
    return r;
}

// One lane does a whole pair: decode (bn256.go:120-164, 256-306), curve checks, the 91 lines, and
// membership from the lines' final point (g2_frob_check).
GSV_DI void prepare_pair(uint32_t i, const uint8_t* __restrict__ in, const uint64_t* __restrict__ pair_src,
                         uint32_t npairs, uint8_t* __restrict__ pstat, uint32_t* __restrict__ lines) {
    const uint8_t* s = in + pair_src[i];
    g1a P;
    g2a Q;
    bool ok = fp_unmarshal(P.x, s);
    ok = fp_unmarshal(P.y, s + 32) && ok;
    ok = fp_unmarshal(Q.x.x, s + 64) && ok;  // imaginary part first (bn256.go:267-278)
    ok = fp_unmarshal(Q.x.y, s + 96) && ok;
    ok = fp_unmarshal(Q.y.x, s + 128) && ok;
    ok = fp_unmarshal(Q.y.y, s + 160) && ok;
    bool inf1 = fq_is_zero(P.x) && fq_is_zero(P.y);
    bool inf2 = fp2_is_zero(Q.x) && fp2_is_zero(Q.y);
    if (ok && !inf1)  // curve.go:39-52: y^2 == x^3 + 3
        ok = fq_eq(fq_mul(P.y, P.y), fq_add(fq_mul(fq_mul(P.x, P.x), P.x), fq_const(FQ_THREE)));
    if (ok && !inf2) ok = g2_on_twist(Q);
    g2j r = pair_lines(lines, npairs, i, P, Q);
    if (ok && !inf2) ok = g2_frob_check(r, Q);
    pstat[i] = !ok ? PS_BAD : (inf1 || inf2) ? PS_SKIP : PS_OK;
}

// k_bn_lines: one wave per SIMD (no spills).  A two-wave budget of the same code (k_bn_prepare through
// r05) spilled 696 B per lane and took the same time at 65,536 checks (7.26 vs 7.27 ms, r04); large
// batches take k_bn_lines_w2 below.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1))) void k_bn_lines(const uint8_t* __restrict__ in,
                                                   const uint64_t* __restrict__ pair_src,
                                                   uint32_t npairs, uint32_t* __restrict__ lines,
                                                   uint8_t* __restrict__ pstat) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < npairs) prepare_pair(i, in, pair_src, npairs, pstat, lines);
}

// ---- the lines role at TWO waves per SIMD (k_bn_lines_w2).  A configs[4] batch has 4 x 65,536 pairs:
// 4,096 waves, two rounds of the GPU's wave slots even at two per SIMD, so unlike the Miller loop the
// lines need no extra split to fill a second wave.  k_bn_lines holds 256 + 125 registers; what moves
// here: P and Q wait in LDS ([54 words][64 lanes], 13.8 KB per wave) and are read where a line needs
// them, and each line coefficient is stored to HBM as soon as it is computed instead of after the step.
// The formulas and their order are line_double_i / line_add_i's, so the lines are the
// same F_p^2 values.
#define LW2_SEQ __builtin_amdgcn_sched_barrier(0)
GSV_DI void lw2_put(uint32_t* l, int j, const fq& v) {
#pragma unroll
    for (int w = 0; w < 9; w++) l[(j * 9 + w) * 64] = v.v[w];
}
GSV_DI fq lw2_get(const uint32_t* l, int j) {
    fq r;
#pragma unroll
    for (int w = 0; w < 9; w++) r.v[w] = l[(j * 9 + w) * 64];
    return r;
}
// the lane's LDS column: P.x, P.y, Q.x.x, Q.x.y, Q.y.x, Q.y.y
GSV_DI g2a lw2_q(const uint32_t* l) { return g2a{fp2{lw2_get(l, 2), lw2_get(l, 3)}, fp2{lw2_get(l, 4), lw2_get(l, 5)}}; }
// optate.go:52-92 (line_double_i, LEAN order), l.a / l.b / l.c stored as computed
GSV_DI void line_double_w2(g2j& r, const uint32_t* l, uint32_t* __restrict__ lines, uint32_t n, uint32_t j, int li) {
    const fp2 A = s2(fp2_sqr(r.x));
    const fp2 B = s2(fp2_sqr(r.y));
    const fp2 C = s2(fp2_sqr(B));
    const fp2 D = s2(fp2_dbl(fp2_sub(fp2_sub(fp2_sqr(fp2_add(r.x, B)), A), C)));
    const fp2 E = s2(fp2_add(fp2_dbl(A), A));
    const fp2 G = s2(fp2_sqr(E));
    LW2_SEQ;
    soa_store2(lines, n, j, li * 6 + 0, s2(fp2_sub(fp2_sub(fp2_sub(fp2_sqr(fp2_add(r.x, E)), A), G), fp2_mul_small<4>(B))));
    LW2_SEQ;
    const fp2 oz = s2(fp2_sub(fp2_sub(fp2_sqr(fp2_add(r.y, r.z)), B), r.t));
    LW2_SEQ;
    soa_store2(lines, n, j, li * 6 + 2, s2(fp2_mul_fp(fp2_neg(fp2_dbl(fp2_mul(E, r.t))), lw2_get(l, 0))));
    LW2_SEQ;
    soa_store2(lines, n, j, li * 6 + 4, s2(fp2_mul_fp(fp2_dbl(fp2_mul(oz, r.t)), lw2_get(l, 1))));
    LW2_SEQ;
    r.x = s2(fp2_sub(G, fp2_dbl(D)));
    r.y = s2(fp2_sub(fp2_mul(fp2_sub(D, r.x), E), fp2_mul_small<8>(C)));
    r.z = oz;
    r.t = s2(fp2_sqr(oz));
}
// optate.go:3-50 (line_add_i: r + p, p affine, r2 = p.y^2), ordered to end each value's life early
GSV_DI void line_add_w2(g2j& r, const g2a& p, const fp2& r2, const uint32_t* l, uint32_t* __restrict__ lines, uint32_t n,
                        uint32_t j, int li) {
    const fp2 H = s2(fp2_sub(fp2_mul(p.x, r.t), r.x));  // B - r.x
    const fp2 L1 = s2(fp2_sub(fp2_mul(fp2_sub(fp2_sub(fp2_sqr(fp2_add(p.y, r.z)), r2), r.t), r.t), fp2_dbl(r.y)));  // D - 2 r.y
    LW2_SEQ;
    const fp2 I = s2(fp2_sqr(H));
    const fp2 E = s2(fp2_mul_small<4>(I));
    const fp2 J = s2(fp2_mul(H, E));
    const fp2 V = s2(fp2_mul(r.x, E));
    LW2_SEQ;
    g2j o;
    o.z = s2(fp2_sub(fp2_sub(fp2_sqr(fp2_add(r.z, H)), r.t), I));
    o.x = s2(fp2_sub(fp2_sub(fp2_sqr(L1), J), fp2_dbl(V)));
    o.y = s2(fp2_sub(fp2_mul(fp2_sub(V, o.x), L1), fp2_dbl(fp2_mul(r.y, J))));
    o.t = s2(fp2_sqr(o.z));
    LW2_SEQ;
    soa_store2(lines, n, j, li * 6 + 0, s2(fp2_sub(fp2_dbl(fp2_mul(L1, p.x)), fp2_sub(fp2_sub(fp2_sqr(fp2_add(p.y, o.z)), r2), o.t))));
    LW2_SEQ;
    soa_store2(lines, n, j, li * 6 + 2, s2(fp2_mul_fp(fp2_dbl(fp2_neg(L1)), lw2_get(l, 0))));
    LW2_SEQ;
    soa_store2(lines, n, j, li * 6 + 4, s2(fp2_mul_fp(fp2_dbl(o.z), lw2_get(l, 1))));
    r = o;
}
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_bn_lines_w2(const uint8_t* __restrict__ in,
                                                   const uint64_t* __restrict__ pair_src,
                                                   uint32_t npairs, uint32_t* __restrict__ lines,
                                                   uint8_t* __restrict__ pstat) {
    __shared__ uint32_t lds[54 * 64];
    uint32_t* l = lds + threadIdx.x;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npairs) return;
    bool ok, inf1, inf2;
    {
        const uint8_t* s = in + pair_src[i];
        g1a P;
        g2a Q;
        ok = fp_unmarshal(P.x, s);
        ok = fp_unmarshal(P.y, s + 32) && ok;
        ok = fp_unmarshal(Q.x.x, s + 64) && ok;  // imaginary part first (bn256.go:267-278)
        ok = fp_unmarshal(Q.x.y, s + 96) && ok;
        ok = fp_unmarshal(Q.y.x, s + 128) && ok;
        ok = fp_unmarshal(Q.y.y, s + 160) && ok;
        inf1 = fq_is_zero(P.x) && fq_is_zero(P.y);
        inf2 = fp2_is_zero(Q.x) && fp2_is_zero(Q.y);
        if (ok && !inf1)  // curve.go:39-52: y^2 == x^3 + 3
            ok = fq_eq(fq_mul(P.y, P.y), fq_add(fq_mul(fq_mul(P.x, P.x), P.x), fq_const(FQ_THREE)));
        if (ok && !inf2) ok = g2_on_twist(Q);
        lw2_put(l, 0, P.x), lw2_put(l, 1, P.y), lw2_put(l, 2, Q.x.x), lw2_put(l, 3, Q.x.y), lw2_put(l, 4, Q.y.x),
            lw2_put(l, 5, Q.y.y);
    }
    LW2_SEQ;
    g2a Q = lw2_q(l);
    g2j r{Q.x, Q.y, fp2_one(), fp2_one()};
    int li = 0;
#pragma unroll 1
    for (int k = 64; k > 0; k--) {
        line_double_w2(r, l, lines, npairs, i, li++);
        const uint64_t bit = 1ull << (k - 1);
        if ((NAF_POS | NAF_NEG) & bit) {
            LW2_SEQ;
            Q = lw2_q(l);
            const fp2 r2 = s2(fp2_sqr(Q.y));
            if (!(NAF_POS & bit)) Q.y = s2(fp2_neg(Q.y));
            line_add_w2(r, Q, r2, l, lines, npairs, i, li++);
        }
        LW2_SEQ;
    }
    // Q1 = pi(Q), -Q2 = -pi^2(Q) (optate.go:168-209)
    Q = lw2_q(l);
    {
        g2a q1{s2(fp2_mul(fp2_conj(Q.x), fp2_const(FQ_XI_P1_3_X, FQ_XI_P1_3_Y))),
               s2(fp2_mul(fp2_conj(Q.y), fp2_const(FQ_XI_P1_2_X, FQ_XI_P1_2_Y)))};
        line_add_w2(r, q1, s2(fp2_sqr(q1.y)), l, lines, npairs, i, li++);
    }
    LW2_SEQ;
    Q = lw2_q(l);
    {
        g2a mq2{s2(fp2_mul_fp(Q.x, fq_const(FQ_XI_PSQ1_3))), Q.y};
        line_add_w2(r, mq2, s2(fp2_sqr(mq2.y)), l, lines, npairs, i, li);
    }
    LW2_SEQ;
    Q = lw2_q(l);
    if (ok && !inf2) ok = g2_frob_check(r, Q);
    pstat[i] = !ok ? PS_BAD : (inf1 || inf2) ? PS_SKIP : PS_OK;
}
#undef LW2_SEQ

// ---- per-check multi-Miller loop.  The product of a check's Miller values equals one loop that
// squares the shared accumulator once per step and multiplies in every pair's lines
// (prod f_i^2 l_i = (prod f_i)^2 prod l_i, exact in F_p^12), so a check of k pairs spends one
// F_p^12 squaring per step instead of k; the verdict is the reference's bit for bit.  One lane per
// check; pair j of a check lives at slot-major index pidx[first + j] (the j-th pairs of all checks
// contiguous), so the per-pair twist point R and the decoded points load/store coalesced.
enum : uint8_t { CS_OK = 0, CS_BAD = 1, CS_ONE = 2 };  // CS_ONE: no finite pair -> product is 1

// A lane runs the loop over a group of <= k of its check's pairs (k = 4 covers a whole 4-pair check;
// smaller k when the batch is too small to give every SIMD work — the host's choice), and k_bn_final
// multiplies a check's lane values: the same exact product, so the same verdict.
constexpr int BN_MILLER_WAVES = 1;  // the Miller kernels' register budget: one wave per SIMD (256 + 256)
// (Through r04 a BN_MILLER_PREFETCH form loaded each line one multiplication ahead; the held line cost
// 177 AGPRs and ~650 accumulator moves, and without it the Miller kernel ran 8.75 -> 8.30 ms at 65,536
// checks, profiles/r04/ab/pf_prefetch{1,0}_*.json.  Unused since, removed in r05.)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BN_MILLER_WAVES))) void k_bn_miller(const uint32_t* __restrict__ lane_first, uint32_t nlanes,
                                                  const uint32_t* __restrict__ pidx, const uint8_t* __restrict__ pstat,
                                                  const uint32_t* __restrict__ lines, uint32_t npairs,
                                                  uint8_t* __restrict__ cstat,
                                                  uint32_t* __restrict__ fv /* [108 words][nlanes] */) {
    uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nlanes) return;
    uint32_t b = lane_first[c], e = lane_first[c + 1];
    bool bad = false, any = false;
    for (uint32_t q = b; q < e; q++) {
        uint8_t st = pstat[pidx[q]];
        bad = bad || st == PS_BAD;
        any = any || st == PS_OK;
    }
    cstat[c] = bad ? CS_BAD : any ? CS_OK : CS_ONE;
    if (bad || !any) return;
    fp12 f = fp12_one();
    int li = 0;
#pragma unroll 1
    for (int i = 64; i > 0; i--) {
        if (i != 64) f = fp12_sqr_i(f);
        uint64_t bit = 1ull << (i - 1);
        int nl = ((NAF_POS | NAF_NEG) & bit) ? 2 : 1;
#pragma unroll 1
        for (uint32_t q = b; q < e; q++) {
            uint32_t j = pidx[q];
            if (pstat[j] != PS_OK) continue;
#pragma unroll 1
            for (int k = 0; k < nl; k++) mul_line_i(f, line_load(lines, npairs, j, li + k));
        }
        li += nl;
    }
#pragma unroll 1
    for (uint32_t q = b; q < e; q++) {
        uint32_t j = pidx[q];
        if (pstat[j] != PS_OK) continue;
#pragma unroll 1
        for (int k = 0; k < 2; k++) mul_line_i(f, line_load(lines, npairs, j, li + k));
    }
    fp12_store(fv, nlanes, c, f);
}

// ---- the same loop at TWO waves per SIMD (k_bn_miller_w2; GSV_BN_MILLER_W2 = 1, not the default: it
// measured slower, r05 — at 65,536 checks k = 2 11.2 vs 9.8 ms of Miller and k = 4 17.0 vs 8.3 ms,
// profiles/r05/ab/miller_w2_sweep_*.txt: the per-coordinate form runs 10.5 k instead of 8.8 k VALU
// instructions per line product, and at two waves the LDS round trips and line loads stay exposed).  At one wave per SIMD every VALU
// instruction holds the SIMD 4.4-5.1 cycles whatever it is (profiles/r01_microbench_lat.txt); with a
// second wave the 43 % of the loop's instructions that are not multiply-adds cost half that.  Two waves
// need <= 256 registers a lane (k_bn_miller: 256 + 65).  What moves out of the register file: one
// F_p^6 value per lane in LDS ([54 words][64 lanes], conflict-free ds_read/write_b32; 13.8 KB per
// wave, eight waves per CU = 110 KB of the 160 KB), and the F_p^6 products are computed one output
// coordinate at a time (each coordinate one fq_dot REDC; scheduling barriers between them), so a
// product's working set is its inputs plus one output.  The field elements are those of mul_line_i /
// fp12_sqr_i (the same Karatsuba formulas), so the Miller values are the same F_p^12 elements.
template <int J, class E>
GSV_DI auto fp6_coord(const fp6t<E>& v) {  // F_p coordinate J of an F_p^6 value (x.x, x.y, y.x, y.y, z.x, z.y)
    if constexpr (J == 0) return v.x.x;
    else if constexpr (J == 1) return v.x.y;
    else if constexpr (J == 2) return v.y.x;
    else if constexpr (J == 3) return v.y.y;
    else if constexpr (J == 4) return v.z.x;
    else return v.z.y;
}
GSV_DI fq& fp6_at(fp6& v, int j) { return ((fq*)&v)[j]; }
GSV_DI void w2_put(uint32_t* l, int j, const fq& v) {
#pragma unroll
    for (int w = 0; w < 9; w++) l[(j * 9 + w) * 64] = v.v[w];
}
GSV_DI fq w2_get(const uint32_t* l, int j) {
    fq r;
#pragma unroll
    for (int w = 0; w < 9; w++) r.v[w] = l[(j * 9 + w) * 64];
    return r;
}
#define W2_SEQ __builtin_amdgcn_sched_barrier(0)
// An empty asm that "redefines" an F_p^6 value in place (no instruction): the per-coordinate products
// below then cannot share their operand preparation (negations, xi multiples) through common-
// subexpression elimination, which would compute them for all six coordinates up front and hold them
// live through the whole product.
GSV_DI void w2_opaque(fq& a) {
    asm volatile("" : "+v"(a.v[0]), "+v"(a.v[1]), "+v"(a.v[2]), "+v"(a.v[3]), "+v"(a.v[4]), "+v"(a.v[5]), "+v"(a.v[6]),
                 "+v"(a.v[7]), "+v"(a.v[8]));
}
GSV_DI void w2_opaque(fp2& a) { w2_opaque(a.x), w2_opaque(a.y); }
GSV_DI void w2_opaque(fp6& a) { w2_opaque(a.x), w2_opaque(a.y), w2_opaque(a.z); }
// the sparse product a (by tau + bz), one coordinate at a time: only the coordinate asked for survives
// dead-code elimination of the fused routine
template <int J, class B>
GSV_DI fq w2_sparse(const fp6& a, const fp2& by, const B& bz) { return fq_store(fp6_coord<J>(fp6_mul_sparse(a, by, bz))); }
template <int J>
GSV_DI fq w2_dense(const fp6& a, const fp6& b) { return fq_store(fp6_coord<J>(fp6_mul(a, b))); }

// mul_line_i (optate.go:94-112) with a2 = f.x (a tau + b) in LDS:
//   a2 -> LDS;  s = f.x + f.y;  t3 = f.y c;  new.y = t3 + tau a2;
//   d = tau a2 - a2 -> LDS;  new.x = s (a tau + b + c) - a2 - t3 = s (a tau + b + c) - new.y + d
// The line is loaded in two parts where its coefficients are first needed (a, b; then c), so the
// loads are not hoisted above the first products.
GSV_DI void mul_line_w2(fp12& f, const uint32_t* __restrict__ lines, uint32_t n, uint32_t pj, int li, uint32_t* l) {
    line L;
    L.a = soa_load2(lines, n, pj, li * 6 + 0);
    L.b = soa_load2(lines, n, pj, li * 6 + 2);
    W2_SEQ;
    w2_opaque(f.x), w2_opaque(L.a), w2_put(l, 0, w2_sparse<0>(f.x, L.a, L.b)); W2_SEQ;
    w2_opaque(f.x), w2_opaque(L.a), w2_put(l, 1, w2_sparse<1>(f.x, L.a, L.b)); W2_SEQ;
    w2_opaque(f.x), w2_opaque(L.a), w2_put(l, 2, w2_sparse<2>(f.x, L.a, L.b)); W2_SEQ;
    w2_opaque(f.x), w2_opaque(L.a), w2_put(l, 3, w2_sparse<3>(f.x, L.a, L.b)); W2_SEQ;
    w2_opaque(f.x), w2_opaque(L.a), w2_put(l, 4, w2_sparse<4>(f.x, L.a, L.b)); W2_SEQ;
    w2_opaque(f.x), w2_opaque(L.a), w2_put(l, 5, w2_sparse<5>(f.x, L.a, L.b)); W2_SEQ;
    L.c = soa_load2(lines, n, pj, li * 6 + 4);
    const fp2 bc = s2(fp2_add(L.b, L.c));
    W2_SEQ;
    f.x = fp6_store(fp6_add(f.x, f.y));      // s
    f.y = fp6_store(fp6_mul_fp2(f.y, L.c));  // t3
    W2_SEQ;
    // new.y = t3 + tau a2 = (t3.x + a2.y, t3.y + a2.z, t3.z + xi a2.x) in place, and d = tau a2 - a2 =
    // (a2.y - a2.x, a2.z - a2.y, xi a2.x - a2.z) over a2 in LDS, in an order that holds at most two of
    // a2's coordinates and one of d's at a time
    {
        fp2 a2x{w2_get(l, 0), w2_get(l, 1)}, a2y{w2_get(l, 2), w2_get(l, 3)};
        fp2 d = s2(fp2_sub(a2y, a2x));
        w2_put(l, 0, d.x), w2_put(l, 1, d.y);
        const fp2 xa = s2(fp2_mul_xi(a2x));
        f.y.x = s2(fp2_add(f.y.x, a2y));
        W2_SEQ;
        fp2 a2z{w2_get(l, 4), w2_get(l, 5)};
        d = s2(fp2_sub(a2z, a2y));
        w2_put(l, 2, d.x), w2_put(l, 3, d.y);
        f.y.y = s2(fp2_add(f.y.y, a2z));
        f.y.z = s2(fp2_add(f.y.z, xa));
        d = s2(fp2_sub(xa, a2z));
        w2_put(l, 4, d.x), w2_put(l, 5, d.y);
    }
    W2_SEQ;
    // new.x = s (a tau + (b + c)) - new.y + d, coordinate by coordinate (the output replaces d in LDS)
#define W2_NX(J)                                                                                      \
    w2_opaque(f.x), w2_opaque(L.a);                                                                   \
    w2_put(l, J, fq_store(fq_add(fq_sub(w2_sparse<J>(f.x, L.a, bc), fp6_at(f.y, J)), w2_get(l, J)))); \
    W2_SEQ;
    W2_NX(0) W2_NX(1) W2_NX(2) W2_NX(3) W2_NX(4) W2_NX(5)
#undef W2_NX
#pragma unroll
    for (int j = 0; j < 6; j++) fp6_at(f.x, j) = w2_get(l, j);
}
// fp12_sqr_i (gfp12.go:129-143) with v0 = f.x f.y in LDS:
//   new.x = 2 v0;  new.y = (f.x + f.y)(tau f.x + f.y) - v0 - tau v0
GSV_DI void sqr_w2(fp12& f, uint32_t* l) {
    w2_opaque(f.x), w2_opaque(f.y), w2_put(l, 0, w2_dense<0>(f.x, f.y)); W2_SEQ;
    w2_opaque(f.x), w2_opaque(f.y), w2_put(l, 1, w2_dense<1>(f.x, f.y)); W2_SEQ;
    w2_opaque(f.x), w2_opaque(f.y), w2_put(l, 2, w2_dense<2>(f.x, f.y)); W2_SEQ;
    w2_opaque(f.x), w2_opaque(f.y), w2_put(l, 3, w2_dense<3>(f.x, f.y)); W2_SEQ;
    w2_opaque(f.x), w2_opaque(f.y), w2_put(l, 4, w2_dense<4>(f.x, f.y)); W2_SEQ;
    w2_opaque(f.x), w2_opaque(f.y), w2_put(l, 5, w2_dense<5>(f.x, f.y)); W2_SEQ;
    fp6 t = fp6_store(fp6_add(fp6_mul_tau(f.x), f.y));
    f.x = fp6_store(fp6_add(f.x, f.y));
    W2_SEQ;
    // new.y_J = (s t)_J - v0_J - (tau v0)_J, tau v0 = (v0.y, v0.z, xi v0.x); xi (x i + y) = (9x + y) i + (9y - x)
    fp6 ny;
#define W2_NY(J, TV)                                                                       \
    w2_opaque(f.x), w2_opaque(t);                                                          \
    fp6_at(ny, J) = fq_store(fq_sub(fq_sub(w2_dense<J>(f.x, t), w2_get(l, J)), TV)); \
    W2_SEQ;
    W2_NY(0, w2_get(l, 2))
    W2_NY(1, w2_get(l, 3))
    W2_NY(2, w2_get(l, 4))
    W2_NY(3, w2_get(l, 5))
    W2_NY(4, fq_add(fq_normalize(fq_mul_small<8>(w2_get(l, 0))), fq_add(w2_get(l, 0), w2_get(l, 1))))
    W2_NY(5, fq_sub(fq_add(fq_normalize(fq_mul_small<8>(w2_get(l, 1))), w2_get(l, 1)), w2_get(l, 0)))
#undef W2_NY
    f.y = ny;
#pragma unroll
    for (int j = 0; j < 6; j++) fp6_at(f.x, j) = fq_store(fq_add(w2_get(l, j), w2_get(l, j)));
}
#undef W2_SEQ
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_bn_miller_w2(
    const uint32_t* __restrict__ lane_first, uint32_t nlanes, const uint32_t* __restrict__ pidx,
    const uint8_t* __restrict__ pstat, const uint32_t* __restrict__ lines, uint32_t npairs,
    uint8_t* __restrict__ cstat, uint32_t* __restrict__ fv /* [108 words][nlanes] */) {
    __shared__ uint32_t lds[54 * 64];
    uint32_t* l = lds + threadIdx.x;
    uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nlanes) return;
    uint32_t b = lane_first[c], e = lane_first[c + 1];
    bool bad = false, any = false;
    for (uint32_t q = b; q < e; q++) {
        uint8_t st = pstat[pidx[q]];
        bad = bad || st == PS_BAD;
        any = any || st == PS_OK;
    }
    cstat[c] = bad ? CS_BAD : any ? CS_OK : CS_ONE;
    if (bad || !any) return;
    fp12 f = fp12_one();
    int li = 0;
#pragma unroll 1
    for (int i = 64; i > 0; i--) {
        if (i != 64) sqr_w2(f, l);
        uint64_t bit = 1ull << (i - 1);
        int nl = ((NAF_POS | NAF_NEG) & bit) ? 2 : 1;
#pragma unroll 1
        for (uint32_t q = b; q < e; q++) {
            uint32_t j = pidx[q];
            if (pstat[j] != PS_OK) continue;
#pragma unroll 1
            for (int k = 0; k < nl; k++) mul_line_w2(f, lines, npairs, j, li + k, l);
        }
        li += nl;
    }
#pragma unroll 1
    for (uint32_t q = b; q < e; q++) {
        uint32_t j = pidx[q];
        if (pstat[j] != PS_OK) continue;
#pragma unroll 1
        for (int k = 0; k < 2; k++) mul_line_w2(f, lines, npairs, j, li + k, l);
    }
    fp12_store(fv, nlanes, c, f);
}

// ---- the loop at TWO waves per SIMD with the line in LDS (k_bn_miller_l; GSV_BN_MILLER_L = 1).  A lane
// has 54 words of LDS ([word][lane], 13.8 KB per wave, 110 KB for the eight waves of a CU) that hold, in
// turn: the line (HBM -> LDS by global_load_lds_dword, no VGPRs on the way), then new.y of the line
// product while its second sparse product runs, and v0 of the squaring while (x + y)(tau x + y) runs.
// The formulas are mul_line_i's / fp12_sqr_i's Karatsuba, ordered so that at most about 245 registers
// are live: line product a2 = f.x (a tau + b); s = f.x + f.y; t3 = f.y c; (a, b + c to registers; new.y
// = t3 + tau a2 to LDS); d = a2 + t3; new.x = s (a tau + b + c) - d — the same field elements
// (s (..) - a2 - t3 = s (..) - d); squaring v0 = f.x f.y to LDS; t = tau f.x + f.y; s = f.x + f.y;
// new.y = s t - v0 - tau v0; new.x = 2 v0.
typedef __attribute__((address_space(3))) uint32_t lds_w;
GSV_DI fq ll_get(const lds_w* l, int j) {
    fq r;
#pragma unroll
    for (int w = 0; w < 9; w++) r.v[w] = l[(j * 9 + w) * 64];
    return r;
}
GSV_DI fp2 ll_get2(const lds_w* l, int j) { return fp2{ll_get(l, j), ll_get(l, j + 1)}; }
GSV_DI fp6 ll_get6(const lds_w* l) { return fp6{ll_get2(l, 0), ll_get2(l, 2), ll_get2(l, 4)}; }
GSV_DI void ll_put6(lds_w* l, const fp6& v) {
    const uint32_t* w = (const uint32_t*)&v;
#pragma unroll
    for (int q = 0; q < 54; q++) l[q * 64] = w[q];
}
// line li of pair j (word q at lines[(li * 54 + q) * n + j]) -> LDS row q of this wave ([word][lane])
GSV_DI void line_fetch_lds(lds_w* row0, const uint32_t* __restrict__ lines, uint32_t n, uint32_t j, int li) {
    const uint32_t row = (uint32_t)(uintptr_t)row0;
    const uint32_t* wb = lines + (size_t)li * 54u * n;
#pragma unroll
    for (int q = 0; q < 54; q++)
        asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dword %0, %1" ::"v"(j * 4u), "s"(wb + (size_t)q * n),
                     "s"(row + (uint32_t)q * 256u)
                     : "memory", "m0");
}
GSV_DI void line_lds_wait() {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    asm volatile("" ::: "memory");
}
// an opaque copy of the lane's LDS pointer: loads through it are not merged with earlier ones, so a
// value read twice is not held live in between
template <class T>
GSV_DI T* ll_fresh(T* l) {
    asm volatile("" : "+v"(l));
    return l;
}
#ifdef LL_MARKS
#define LL_STR2(x) #x
#define LL_STR(x) LL_STR2(x)
#define LL_SEQ __builtin_amdgcn_sched_barrier(0); asm volatile("; LLMARK " LL_STR(__LINE__)); __builtin_amdgcn_sched_barrier(0)
#else
#define LL_SEQ __builtin_amdgcn_sched_barrier(0)
#endif
GSV_DI void ll_put2(lds_w* l, int j, const fp2& v) {
    const uint32_t* w = (const uint32_t*)&v;
#pragma unroll
    for (int q = 0; q < 18; q++) l[(j * 9 + q) * 64] = w[q];
}
GSV_DI void mul_line_l(fp12& f, lds_w* l) {
    fp6 a2 = fp6_store(fp6_mul_sparse(f.x, ll_get2(ll_fresh(l), 0), ll_get2(ll_fresh(l), 2)));  // f.x (a tau + b)
    LL_SEQ;
    f.x = fp6_store(fp6_add(f.x, f.y));  // s
    LL_SEQ;
    fp6 t3 = fp6_store(fp6_mul_fp2(f.y, ll_get2(ll_fresh(l), 4)));  // f.y c
    LL_SEQ;
    const lds_w* p = ll_fresh(l);
    const fp2 la = ll_get2(p, 0);
    const fp2 bc = s2(fp2_add(ll_get2(p, 2), ll_get2(p, 4)));
    LL_SEQ;
    // new.y = t3 + tau a2 = (t3.x + a2.y, t3.y + a2.z, t3.z + xi a2.x) -> LDS (over the line), one
    // coordinate at a time, then d = a2 + t3 in place
    ll_put2(ll_fresh(l), 0, s2(fp2_add(t3.x, a2.y)));
    LL_SEQ;
    ll_put2(ll_fresh(l), 2, s2(fp2_add(t3.y, a2.z)));
    LL_SEQ;
    ll_put2(ll_fresh(l), 4, s2(fp2_add(t3.z, fp2_mul_xi(a2.x))));
    LL_SEQ;
    a2 = fp6_store(fp6_add(a2, t3));  // d
    LL_SEQ;
    f.x = fp6_store(fp6_sub(fp6_mul_sparse(f.x, la, bc), a2));  // s (a tau + b + c) - d
    LL_SEQ;
    f.y = ll_get6(ll_fresh(l));
}
GSV_DI void sqr_l(fp12& f, lds_w* l) {
    ll_put6(ll_fresh(l), fp6_store(fp6_mulx(f.x, f.y)));  // v0 -> LDS
    LL_SEQ;
    fp6 t = fp6_store(fp6_add(fp6_mul_tau(f.x), f.y));
    f.x = fp6_store(fp6_add(f.x, f.y));  // s
    fp6 st = fp6_store(fp6_mulx(f.x, t));
    LL_SEQ;
    fp6 v0 = ll_get6(ll_fresh(l));
    f.y = fp6_store(fp6_sub(fp6_sub(st, v0), fp6_mul_tau(v0)));
    f.x = fp6_store(fp6_add(v0, v0));
}
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_bn_miller_l(
    const uint32_t* __restrict__ lane_first, uint32_t nlanes, const uint32_t* __restrict__ pidx,
    const uint8_t* __restrict__ pstat, const uint32_t* __restrict__ lines, uint32_t npairs,
    uint8_t* __restrict__ cstat, uint32_t* __restrict__ fv /* [108 words][nlanes] */) {
    __shared__ uint32_t lds[54 * 64];
    lds_w* row0 = (lds_w*)lds;
    lds_w* l = row0 + threadIdx.x;
    uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nlanes) return;
    uint32_t b = lane_first[c], e = lane_first[c + 1];
    bool bad = false, any = false;
    for (uint32_t q = b; q < e; q++) {
        uint8_t st = pstat[pidx[q]];
        bad = bad || st == PS_BAD;
        any = any || st == PS_OK;
    }
    cstat[c] = bad ? CS_BAD : any ? CS_OK : CS_ONE;
    if (bad || !any) return;
    fp12 f = fp12_one();
    int li = 0;
#pragma unroll 1
    for (int i = 64; i > 0; i--) {
        if (i != 64) sqr_l(f, l);
        uint64_t bit = 1ull << (i - 1);
        int nl = ((NAF_POS | NAF_NEG) & bit) ? 2 : 1;
#pragma unroll 1
        for (uint32_t q = b; q < e; q++) {
            uint32_t j = pidx[q];
            if (pstat[j] != PS_OK) continue;
#pragma unroll 1
            for (int k = 0; k < nl; k++) {
                line_fetch_lds(row0, lines, npairs, j, li + k);
                line_lds_wait();
                mul_line_l(f, l);
            }
        }
        li += nl;
    }
#pragma unroll 1
    for (uint32_t q = b; q < e; q++) {
        uint32_t j = pidx[q];
        if (pstat[j] != PS_OK) continue;
#pragma unroll 1
        for (int k = 0; k < 2; k++) {
            line_fetch_lds(row0, lines, npairs, j, li + k);
            line_lds_wait();
            mul_line_l(f, l);
        }
    }
    fp12_store(fv, nlanes, c, f);
}

// ---- two-lane Miller step, for batches too small to give every SIMD a wave: lanes (2c, 2c+1) run
// Miller lane c together.  Both hold the whole accumulator; each F_p^12 squaring's two F_p^6
// products and each line product's two sparse products (plus half of its F_p^2-scalar product)
// are split by the lane's role (one instruction stream: the operands are selected, not branched on)
// and exchanged with ds_bpermute, so the dependent chain per step is about half as long.  Every part
// computes the same formula as the one-lane routine: the same field elements.
template <class E, class F>
GSV_DI auto sel6(bool r, const fp6t<E>& a, const fp6t<F>& b) {  // r ? b : a, at their common bound
    auto w = fp6_of(a.x, a.y, a.z);
    auto v = fp6_of(b.x, b.y, b.z);
    constexpr int l = imax(fp2_traits<decltype(w.x)>::l, fp2_traits<decltype(v.x)>::l);
    constexpr int vv = imax(fp2_traits<decltype(w.x)>::v, fp2_traits<decltype(v.x)>::v);
    fp6t<fp2m<l, vv>> o, bw;
    o = fp6t<fp2m<l, vv>>{fp2_widen<l, vv>(w.x), fp2_widen<l, vv>(w.y), fp2_widen<l, vv>(w.z)};
    bw = fp6t<fp2m<l, vv>>{fp2_widen<l, vv>(v.x), fp2_widen<l, vv>(v.y), fp2_widen<l, vv>(v.z)};
    uint32_t* po = (uint32_t*)&o;
    const uint32_t* pb = (const uint32_t*)&bw;
#pragma unroll
    for (int k = 0; k < 54; k++) po[k] = r ? pb[k] : po[k];
    return o;
}
template <int L1, int V1, int L2, int V2>
GSV_DI auto sel2(bool r, const fp2m<L1, V1>& a, const fp2m<L2, V2>& b) {
    constexpr int l = imax(L1, L2), v = imax(V1, V2);
    fp2m<l, v> o = fp2_widen<l, v>(a), bw = fp2_widen<l, v>(b);
#pragma unroll
    for (int k = 0; k < 9; k++) {
        o.x.v[k] = r ? bw.x.v[k] : o.x.v[k];
        o.y.v[k] = r ? bw.y.v[k] : o.y.v[k];
    }
    return o;
}
template <class T>
GSV_DI void gather2(T out[2], const T& mine, int base) {
    static_assert(sizeof(T) % 4 == 0, "word-sized");
    const uint32_t* m = (const uint32_t*)&mine;
#pragma unroll
    for (int r = 0; r < 2; r++) {
        uint32_t* o = (uint32_t*)&out[r];
#pragma unroll
        for (int w = 0; w < (int)(sizeof(T) / 4); w++) o[w] = bperm(m[w], base + r);
    }
}
// fp12_sqr_i: role 0 v0 = x y, role 1 (x + y)(tau x + y)
GSV_DI fp12 fp12_sqr2(const fp12& a, bool role, int base) {
    auto sum = fp6_add(a.x, a.y);
    auto t = fp6_add(fp6_mul_tau(a.x), a.y);
    auto prod = fp6_mul(sel6(role, a.x, sum), sel6(role, a.y, t));
    decltype(prod) v[2];
    gather2(v, prod, base);
    fp6 v0 = fp6_store(v[0]);
    return fp12{fp6_store(fp6_add(v0, v0)), fp6_store(fp6_sub(fp6_sub(v[1], v0), fp6_mul_tau(v0)))};
}
// mul_line_i: role 0 a2 = ret.x (a tau + b) and t3.x, t3.y; role 1 (ret.x + ret.y)(a tau + b + c) and t3.z
struct line2_part {
    fp6 q;
    fp2 t0, t1;
};
GSV_DI void mul_line2(fp12& ret, const line& l, bool role, int base) {
    auto s = fp6_add(ret.x, ret.y);
    line2_part mine, all[2];
    mine.q = fp6_store(fp6_mul_sparse(sel6(role, ret.x, s), l.a, sel2(role, l.b, fp2_add(l.b, l.c))));
    mine.t0 = s2(fp2_mul(sel2(role, ret.y.x, ret.y.z), l.c));
    mine.t1 = s2(fp2_mul(ret.y.y, l.c));
    gather2(all, mine, base);
    fp6 t3{all[0].t0, all[0].t1, all[1].t0};
    const fp6& a2 = all[0].q;
    ret.x = fp6_store(fp6_sub(fp6_sub(all[1].q, a2), t3));
    ret.y = fp6_store(fp6_add(t3, fp6_mul_tau(a2)));
}
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BN_MILLER_WAVES))) void k_bn_miller2(
    const uint32_t* __restrict__ lane_first, uint32_t nlanes, const uint32_t* __restrict__ pidx,
    const uint8_t* __restrict__ pstat, const uint32_t* __restrict__ lines, uint32_t npairs,
    uint8_t* __restrict__ cstat, uint32_t* __restrict__ fv) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t c = t >> 1;
    bool role = (t & 1u) != 0;
    int base = (int)(threadIdx.x & ~1u);
    if (c >= nlanes) return;  // both lanes of a pair leave together (nlanes counts pairs of lanes)
    uint32_t b = lane_first[c], e = lane_first[c + 1];
    bool bad = false, any = false;
    for (uint32_t q = b; q < e; q++) {
        uint8_t st = pstat[pidx[q]];
        bad = bad || st == PS_BAD;
        any = any || st == PS_OK;
    }
    if (!role) cstat[c] = bad ? CS_BAD : any ? CS_OK : CS_ONE;
    if (bad || !any) return;
    fp12 f = fp12_one();
    int li = 0;
#pragma unroll 1
    for (int i = 64; i > 0; i--) {
        if (i != 64) f = fp12_sqr2(f, role, base);
        uint64_t bit = 1ull << (i - 1);
        int nl = ((NAF_POS | NAF_NEG) & bit) ? 2 : 1;
#pragma unroll 1
        for (uint32_t q = b; q < e; q++) {
            uint32_t j = pidx[q];
            if (pstat[j] != PS_OK) continue;
#pragma unroll 1
            for (int k = 0; k < nl; k++) mul_line2(f, line_load(lines, npairs, j, li + k), role, base);
        }
        li += nl;
    }
#pragma unroll 1
    for (uint32_t q = b; q < e; q++) {
        uint32_t j = pidx[q];
        if (pstat[j] != PS_OK) continue;
#pragma unroll 1
        for (int k = 0; k < 2; k++) mul_line2(f, line_load(lines, npairs, j, li + k), role, base);
    }
    if (!role) fp12_store(fv, nlanes, c, f);
}

// ---------------------------------------------------------------- final exponentiation (optate.go:212-261)
// The final exponentiation runs as a PROGRAM of F_p^12 operations on two values: X (the accumulator,
// in registers) and A (the operand, in LDS: one F_p^12 per lane; with a product's packed v0 beside it,
// 156 words per lane = 39,936 B per 64-lane workgroup, so CDNA4's 160 KB of LDS per CU holds four
// workgroups — more than the one wave per SIMD the kernel's registers allow).  One loop executes it; its body holds a single copy of each operation,
// so k_bn_final's code stays small, and nothing is called: no call frames, no callee-saved register
// spills, no private segment.  A product streams A's halves from LDS, so its working set is X plus
// one F_p^6 product's (a dense F_p^6 product alone needs ~240 VGPRs of operands and column
// accumulators; with both F_p^12 operands in registers the kernel spilled 1.3 KB per lane).  Values
// that outlive X and A go to an explicit per-check workspace in HBM ([slot][108 words][check],
// coalesced), written and read once each: 7 stores + 8 loads of 432 bytes per check.  The program is
// the reference's sequence regrouped (the same group element, so the same IsOne verdict):
//   t1 = conj(in) in^-1,  t1 *= frob^2(t1)                                   (easy part)
//   fu = t1^u, fu2 = fu^u, fu3 = fu2^u  (NAF of u: 62 cyclotomic squarings, 23 products each)
//   y0 = frob(t1 frob(t1 frob(t1))) = frob(t1) frob^2(t1) frob^3(t1),  C = y0 y1^2  (y1 = conj t1)
//   y3 = conj frob(fu), y4 = conj(fu frob(fu2)), y5 = conj fu2, y2 = frob^2(fu2), y6 = conj(fu3 frob(fu3))
//   B = y4 y5, D = (y3 y5)^2 y2, t0 = y6^2 B,  T = (D t0^3)^2,  result = T^3 C
// which expands to the reference's t0 = y6^2 y4 y5, t1 = ((y3 y5 t0)^2 t0 y2)^2, (t1 y1)^2 (t1 y0):
// 15 F_p^12 products outside the exponentiations (as the reference) and two more cyclotomic squarings.
enum : uint8_t {
    FE_END = 0,
    FE_MUL,    // X = X A
    FE_MULC,   // X = X conj(A)
    FE_CSQR,   // X = X^2 (cyclotomic)
    FE_FROB,   // X = frob(X)
    FE_FROB2,  // X = frob^2(X)
    FE_CONJ,   // X = conj(X)
    FE_INV,    // X = X^-1
    FE_XA,     // A = X
    FE_AX,     // X = A
    FE_SWAP,   // X <-> A
    FE_LDX,    // X = ws[slot]
    FE_LDA,    // A = ws[slot]
    FE_STX,    // ws[slot] = X
    FE_LDFV,   // A = the next Miller-lane value of the check (prologue; not in the program)
    FE_CSQR_LDA,  // X = X^2 while A = ws[slot] is fetched (the loads issue before the squaring)
};
// The exponentiations by u use width-4 signed digits of u (13 products below the leading digit instead
// of the NAF's 23, plus 3 for the odd powers a^3, a^5, a^7).  The odd powers go to workspace slots 4..7;
// each digit's power is fetched into A during the squaring after the previous product, so its load
// latency hides under that squaring.  (The NAF form, A = a throughout, moves ~0.45 instead of 1.76 GB
// per 65,536-check launch at 8-14 % more time, r04.)
// width-4 digits of u below bit 62 (u = 2^62 + sum d_i 2^i, constants.go:17): bit i of U_W4_NZ set
// where d_i != 0, of U_W4_NEG where d_i < 0; (|d_i| - 1) / 2 = U_W4_I0 bit + 2 U_W4_I1 bit
constexpr uint64_t U_W4_NZ = 0x108844442110211ULL, U_W4_NEG = 0x8004400010010ULL;
constexpr uint64_t U_W4_I0 = 0x8800400110000ULL, U_W4_I1 = 0x100044002110200ULL;
static_assert(BN_FINAL_SLOTS == 8, "the program uses slots 0..3, the odd powers 4..7");
constexpr int FE_T0 = 4;  // slots FE_T0 + k: a^(2k+1) of the exponentiation in progress
constexpr int FE_MAXOPS = 384;
struct FeProg {
    uint8_t op[FE_MAXOPS];
    int n;
};
struct FeBuild {
    FeProg p{};
    constexpr void e(int k, int slot = 0) { p.op[p.n++] = (uint8_t)(k | slot << 5); }
    // X = A^u (gfp12.go:113-127 on the NAF of u, constants.go:17; a^-1 = conj(a) in the cyclotomic
    // subgroup); A unchanged
    constexpr void exp_u() {
        e(FE_AX), e(FE_STX, FE_T0), e(FE_CSQR), e(FE_XA), e(FE_LDX, FE_T0);  // A = a^2, X = a
        for (int k = 1; k < 4; k++) e(FE_MUL), e(FE_STX, FE_T0 + k);         // a^3, a^5, a^7
        e(FE_LDX, FE_T0);                                                     // the leading digit
        int held = -1;  // the power A holds (-1: a^2, no longer needed)
        bool free = true;  // A may be overwritten (its last product is done)
        for (int i = 61; i >= 0; i--) {
            // the next digit's power, fetched during the first squaring after the previous product
            int nxt = -1;
            for (int j = i; j >= 0 && nxt < 0; j--)
                if ((U_W4_NZ >> j) & 1) nxt = (int)((U_W4_I0 >> j) & 1) | (int)(((U_W4_I1 >> j) & 1) << 1);
            if (free && nxt >= 0 && nxt != held) {
                e(FE_CSQR_LDA, FE_T0 + nxt);
                held = nxt;
            } else {
                e(FE_CSQR);
            }
            free = true;
            if ((U_W4_NZ >> i) & 1) {
                e((U_W4_NEG >> i) & 1 ? FE_MULC : FE_MUL);
                free = true;
            }
        }
        e(FE_LDA, FE_T0);  // A = a again
    }
    constexpr FeProg build() {
        // easy part: X = in
        e(FE_XA), e(FE_INV), e(FE_MULC);             // X = in^-1 conj(in)
        e(FE_XA), e(FE_FROB2), e(FE_MUL);            // X = t1
        e(FE_XA);                                    // A = t1
        exp_u();                                     // X = fu
        e(FE_STX, 0);                                // s0 = fu
        e(FE_AX), e(FE_FROB), e(FE_MUL), e(FE_FROB), e(FE_MUL), e(FE_FROB);  // X = y0
        e(FE_SWAP), e(FE_CSQR), e(FE_SWAP), e(FE_MULC);  // X = y0 conj(t1)^2 = C
        e(FE_STX, 1);                                // s1 = C
        e(FE_LDA, 0), e(FE_AX), e(FE_FROB), e(FE_CONJ), e(FE_STX, 2);  // s2 = y3, A = fu
        exp_u();                                     // X = fu2
        e(FE_STX, 0);                                // s0 = fu2
        e(FE_FROB), e(FE_MUL), e(FE_CONJ);           // X = y4
        e(FE_LDA, 0), e(FE_MULC), e(FE_STX, 3);      // s3 = B = y4 y5, A = fu2
        e(FE_LDX, 2), e(FE_MULC), e(FE_CSQR), e(FE_STX, 2);  // s2 = (y3 y5)^2
        e(FE_AX), e(FE_FROB2), e(FE_LDA, 2), e(FE_MUL), e(FE_STX, 2);  // s2 = D
        e(FE_LDA, 0);                                // A = fu2
        exp_u();                                     // X = fu3
        e(FE_XA), e(FE_FROB), e(FE_MUL), e(FE_CONJ);  // X = y6
        e(FE_CSQR), e(FE_LDA, 3), e(FE_MUL);         // X = t0
        e(FE_XA), e(FE_CSQR), e(FE_MUL);             // X = t0^3
        e(FE_LDA, 2), e(FE_MUL), e(FE_CSQR);         // X = T
        e(FE_XA), e(FE_CSQR), e(FE_MUL);             // X = T^3
        e(FE_LDA, 1), e(FE_MUL);                     // X = T^3 C
        e(FE_END);
        return p;
    }
};
constexpr FeProg fe_program() { return FeBuild{}.build(); }
__device__ constexpr FeProg FE_PROG = fe_program();
static_assert(fe_program().n <= FE_MAXOPS, "program length");

GSV_DI fp12 fp12_frob_i(const fp12& a) {  // gfp12.go:60-66
    return fp12{fp6_store(fp6_mul_fp2(fp6_frob(a.x), fp2_const(FQ_XI_P1_6_X, FQ_XI_P1_6_Y))), fp6_frob(a.y)};
}
GSV_DI fp12 fp12_frob_p2_i(const fp12& a) {  // gfp12.go:68-74
    return fp12{fp6_store(fp6_mul_fp(fp6_frob_p2(a.x), fq_c(FQ_XI_PSQ1_6))), fp6_frob_p2(a.y)};
}
GSV_DI fp12 fp12_inv_i(const fp12& a) {  // gfp12.go:145-160
    fp6 t1 = fp6_store(fp6_sub(fp6_sqr(a.y), fp6_mul_tau(fp6_sqr(a.x))));
    fp6 t2 = fp6_inv(t1);
    return fp12{fp6_store(fp6_mul(fp6_neg(a.x), t2)), fp6_store(fp6_mul(a.y, t2))};
}
// explicit per-check F_p^12 storage: [slot][108 words][n] (coalesced across the wave)
GSV_DI fp12 ws_load(const uint32_t* __restrict__ ws, uint32_t n, uint32_t c, int slot) {
    fp12 e;
    uint32_t* w = (uint32_t*)&e;
#pragma unroll
    for (int k = 0; k < 108; k++) w[k] = ws[((size_t)slot * 108 + k) * n + c];
    return e;
}
GSV_DI void ws_store(uint32_t* __restrict__ ws, uint32_t n, uint32_t c, int slot, const fp12& e) {
    const uint32_t* w = (const uint32_t*)&e;
#pragma unroll
    for (int k = 0; k < 108; k++) ws[((size_t)slot * 108 + k) * n + c] = w[k];
}
// A in LDS: word q of the lane's F_p^12 at lds[q * 64] (the lane's column of a [108][64] array: every
// access is one conflict-free ds_read/write_b32 across the wave)
GSV_DI fp6 lds_fp6(const uint32_t* lds, int half) {
    fp6 e;
    uint32_t* w = (uint32_t*)&e;
#pragma unroll
    for (int q = 0; q < 54; q++) w[q] = lds[(half * 54 + q) * 64];
    return e;
}
GSV_DI fp12 lds_fp12(const uint32_t* lds) { return fp12{lds_fp6(lds, 0), lds_fp6(lds, 1)}; }
// A = ws[slot] straight from HBM into LDS (global_load_lds_dword: word q of every lane lands at
// lds_base[q * 64 + lane], the [word][lane] layout A has), no VGPRs on the way; the data is there after
// fe_lds_wait()
GSV_DI void lds_fetch(uint32_t* lds_base, const uint32_t* __restrict__ ws, uint32_t n, uint32_t c0, uint32_t t,
                      int slot) {
    // saddr form: the row's base for the wave's first check c0 in an SGPR pair (64-bit: the workspace
    // is BN_FINAL_SLOTS x 432 bytes per check, beyond 4 GiB above ~1.24 M checks), the lane's byte
    // offset t * 4 (< 256) in a VGPR; M0 = the word's LDS row.  c0, n and slot are wave-uniform.
    const uint32_t* wb = ws + (size_t)slot * 108u * n + c0;
    const uint32_t row = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)lds_base;
#pragma unroll
    for (int q = 0; q < 108; q++)
        asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dword %0, %1" ::"v"(t * 4u), "s"(wb + (size_t)q * n),
                     "s"(row + (uint32_t)q * 256u)
                     : "memory", "m0");
}
GSV_DI void fe_lds_wait() {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (gfx9 encoding: expcnt 7, lgkmcnt 15 left open)
    asm volatile("" ::: "memory");
}
GSV_DI void lds_put(uint32_t* lds, const fp12& e) {
    const uint32_t* w = (const uint32_t*)&e;
#pragma unroll
    for (int q = 0; q < 108; q++) lds[q * 64] = w[q];
}
// the operand's halves from LDS; x conjugated (negated) for FE_MULC
struct FeOperand {
    const uint32_t* lds;
    bool conj;
    GSV_DI fp6 x() const {
        fp6 v = lds_fp6(lds, 0);
        if (conj) v = fp6_store(fp6_neg(v));
        return v;
    }
    GSV_DI fp6 y() const { return lds_fp6(lds, 1); }
};
// an F_p element below 2^256 (limbs normalised, value < 3p) packed into eight words and back: the
// 29-bit limbs are the value's base-2^29 digits, so the round trip is exact
GSV_DI void fq_pack_lds(uint32_t* lds, const fqm<1, 3>& a) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
        uint32_t w = 0;
#pragma unroll
        for (int i = 0; i < 9; i++) {
            int lo = 29 * i - 32 * j;  // bit of word j where limb i starts
            if (lo >= 32 || lo + 29 <= 0) continue;
            w |= lo >= 0 ? a.v[i] << lo : a.v[i] >> -lo;
        }
        lds[j * 64] = w;
    }
}
GSV_DI fqm<1, 3> fq_unpack_lds(const uint32_t* lds) {
    uint32_t w[9];
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = lds[j * 64];
    w[8] = 0;
    fqm<1, 3> r;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        int k = 29 * i / 32, sh = 29 * i % 32;
        uint32_t v = sh ? (w[k] >> sh) | (w[k + 1] << (32 - sh)) : w[k];
        r.v[i] = v & FQ_M29;
    }
    return r;
}
// X = X A (fp12_mul_i; A = lds, conjugated when conj).  The three F_p^6 products run one after the
// other (scheduling barriers keep the scheduler from interleaving them), A's halves are read from LDS
// where each product needs them, v0 waits in LDS (reduced below 3p and packed into 48 words, next to
// A's 108: 156 words per lane, 39 KB per workgroup) and v1 and X.x + X.y take X's registers — so each
// product runs with only one other F_p^6 value live beside it, and nothing spills.
constexpr int FE_LDS_V0 = 108;  // word offset of the packed v0 in the lane's LDS column
GSV_DI void fp12_mul_lds(fp12& X, uint32_t* lds, const FeOperand& B) {
    {
        auto v0 = fp6_mul(X.x, B.x());
        fq_pack_lds(lds + (FE_LDS_V0 + 0) * 64, fq_reduce(v0.x.x));
        fq_pack_lds(lds + (FE_LDS_V0 + 8) * 64, fq_reduce(v0.x.y));
        fq_pack_lds(lds + (FE_LDS_V0 + 16) * 64, fq_reduce(v0.y.x));
        fq_pack_lds(lds + (FE_LDS_V0 + 24) * 64, fq_reduce(v0.y.y));
        fq_pack_lds(lds + (FE_LDS_V0 + 32) * 64, fq_reduce(v0.z.x));
        fq_pack_lds(lds + (FE_LDS_V0 + 40) * 64, fq_reduce(v0.z.y));
    }
    __builtin_amdgcn_sched_barrier(0);
    X.x = fp6_store(fp6_add(X.x, X.y));
    X.y = fp6_store(fp6_mul(X.y, B.y()));  // v1
    __builtin_amdgcn_sched_barrier(0);
    fp6 v2 = fp6_store(fp6_mul(X.x, fp6_add(B.x(), B.y())));
    __builtin_amdgcn_sched_barrier(0);
    using e3 = fp2m<1, 3>;
    fp6t<e3> v0{e3{fq_unpack_lds(lds + (FE_LDS_V0 + 0) * 64), fq_unpack_lds(lds + (FE_LDS_V0 + 8) * 64)},
                e3{fq_unpack_lds(lds + (FE_LDS_V0 + 16) * 64), fq_unpack_lds(lds + (FE_LDS_V0 + 24) * 64)},
                e3{fq_unpack_lds(lds + (FE_LDS_V0 + 32) * 64), fq_unpack_lds(lds + (FE_LDS_V0 + 40) * 64)}};
    X.x = fp6_store(fp6_sub(fp6_sub(v2, v0), X.y));
    X.y = fp6_store(fp6_add(X.y, fp6_mul_tau(v0)));
}
// the three-lane form of fp12_mul_i: role 0 X.x A.x, role 1 X.y A.y, role 2 (X.x + X.y)(A.x + A.y)
GSV_DI void fp12_mul3_lds(fp12& X, const FeOperand& B, int role, int base) {
    fp6 l = role == 0 ? X.x : role == 1 ? X.y : fp6_store(fp6_add(X.x, X.y));
    fp6 ax = B.x(), ay = B.y();
    fp6 r = role == 0 ? ax : role == 1 ? ay : fp6_store(fp6_add(ax, ay));
    fp6 prod = fp6_store(fp6_mul(l, r)), v[3];
    gather3(v, prod, base);
    X.x = fp6_store(fp6_sub(fp6_sub(v[2], v[0]), v[1]));
    X.y = fp6_store(fp6_add(v[1], fp6_mul_tau(v[0])));
}

// FinalArgs: maxl = the most Miller lanes any check of the batch has (the prologue's length, uniform
// across the wave); ws = the final exponentiation's workspace, BN_FINAL_SLOTS F_p^12 values per check
struct FinalArgs {
    const uint32_t* check_lane;
    uint32_t nchecks;
    const uint8_t* cbad;
    const uint8_t* lstat;
    const uint32_t* fv;
    uint32_t nlanes;
    uint8_t* verdict;
    uint32_t* ws;
    uint32_t maxl;
};
// Per-lane quantities the machine needs at every operation (the check index, the lane's LDS column,
// the triple's role and base) are recomputed from the lane id when used instead of being carried
// across the loop: at the product's register peak every loop-carried VGPR beyond X is one the
// allocator would otherwise spill to scratch and reload around each product.  The lane id comes from
// a volatile v_mbcnt pair so the compiler cannot hoist it out of the loop.
GSV_DI uint32_t lane_id_v() {
    uint32_t l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
// three lanes per check (21 triples per wave, lane 63 idle); a triple's lanes take the same path
constexpr uint32_t FINAL3_PER_WAVE = 21;
template <bool COOP>
struct FeLane {
    uint32_t lane;
    GSV_DI FeLane() : lane(lane_id_v()) {}
    GSV_DI uint32_t t() const { return COOP ? lane / 3 : lane; }
    GSV_DI uint32_t check0() const { return blockIdx.x * (COOP ? FINAL3_PER_WAVE : 64u); }  // wave-uniform
    GSV_DI uint32_t check() const { return check0() + t(); }
    GSV_DI int role() const { return COOP ? (int)(lane - 3 * t()) : 0; }
    GSV_DI int base() const { return COOP ? (int)(3 * t()) : -1; }
};
// the check's Miller-lane value l0 + 1 + k (one for a lane the check does not have or whose pairs were
// all at infinity)
GSV_DI fp12 fv_extra(const FinalArgs& fa, uint32_t c, uint32_t k) {
    uint32_t l = fa.check_lane[c] + 1 + k;
    return (l < fa.check_lane[c + 1] && fa.lstat[l] == CS_OK) ? fp12_load(fa.fv, fa.nlanes, l) : fp12_one();
}
// The machine.  COOP: the lane is one of three (base, base+1, base+2) sharing the check (role = its
// index); each F_p^12 product and cyclotomic squaring is split three ways and exchanged (the other
// operations are cheap and run on all three lanes).  The prologue multiplies in the check's
// Miller-lane values after the first (nextra of them, uniform across the wave; the product is exact).
template <bool COOP>
GSV_DI fp12 final_exp_run(fp12 X, const FinalArgs& fa, uint32_t* lds_base, uint32_t nextra) {
    const uint32_t npro = 2 * nextra;
#pragma unroll 1
    for (uint32_t pc = 0;; pc++) {
        uint32_t op = pc < npro ? ((pc & 1) ? (uint32_t)FE_MUL : (uint32_t)FE_LDFV) : (uint32_t)FE_PROG.op[pc - npro];
        uint32_t k = op & 31, slot = op >> 5;
        if (k == FE_END) break;
        const FeLane<COOP> ln;
        uint32_t* lds = lds_base + ln.lane;
        if (k != FE_CSQR && k != FE_CSQR_LDA) fe_lds_wait();  // an A fetched by an earlier op has landed
        switch (k) {
        case FE_MUL:
        case FE_MULC: {
            const FeOperand B{lds, k == FE_MULC};
            if constexpr (COOP) fp12_mul3_lds(X, B, ln.role(), ln.base());
            else fp12_mul_lds(X, lds, B);
            break;
        }
        case FE_CSQR:
        case FE_CSQR_LDA: {
            if (k == FE_CSQR_LDA) lds_fetch(lds_base, fa.ws, fa.nchecks, ln.check0(), ln.t(), (int)slot);
            if constexpr (COOP) {
                fp12 m;
                fp12_cyclo_sqr3_i(&m, X, ln.role(), ln.base());
                X = m;
            } else {
                X = fp12_cyclo_sqr_i(X);
            }
            break;
        }
        case FE_FROB: X = fp12_frob_i(X); break;
        case FE_FROB2: X = fp12_frob_p2_i(X); break;
        case FE_CONJ: X = fp12_conj(X); break;
        case FE_INV: X = fp12_inv_i(X); break;
        case FE_XA: lds_put(lds, X); break;
        case FE_AX: X = lds_fp12(lds); break;
        case FE_SWAP: {
            fp12 t = lds_fp12(lds);
            lds_put(lds, X);
            X = t;
            break;
        }
        case FE_LDX: X = ws_load(fa.ws, fa.nchecks, ln.check(), (int)slot); break;
        case FE_LDA: lds_fetch(lds_base, fa.ws, fa.nchecks, ln.check0(), ln.t(), (int)slot); break;
        case FE_STX: ws_store(fa.ws, fa.nchecks, ln.check(), (int)slot, X); break;
        case FE_LDFV: lds_put(lds, fv_extra(fa, ln.check(), pc >> 1)); break;
        default: break;
        }
    }
    return X;
}

// cbad[c] != 0: the check's input length is not a multiple of 192 (errBadPairingInput,
// core/vm/contracts.go:336-338); it has no pairs
// the verdict is written by the lane of role 0
template <bool COOP>
GSV_DI void final_check(const FinalArgs& fa, uint32_t* lds_base) {
    const FeLane<COOP> ln;
    if (COOP && ln.t() >= FINAL3_PER_WAVE) return;
    uint32_t c = ln.check();
    if (c >= fa.nchecks) return;
    uint32_t l0 = fa.check_lane[c], l1 = fa.check_lane[c + 1];
    bool bad = fa.cbad[c] != 0;
    for (uint32_t l = l0; l < l1; l++) bad = bad || fa.lstat[l] == CS_BAD;
    if (bad) {
        if (ln.role() == 0) fa.verdict[c] = GSV_PAIRING_BAD_INPUT;
        return;
    }
    // the product of the check's finite lane values (finalExponentiation(1) == 1 when there are none):
    // X = the first lane's value, the prologue multiplies in the rest
    fp12 X = (l0 < l1 && fa.lstat[l0] == CS_OK) ? fp12_load(fa.fv, fa.nlanes, l0) : fp12_one();
    fp12 r = final_exp_run<COOP>(X, fa, lds_base, fa.maxl > 1 ? fa.maxl - 1 : 0);
    if (ln.role() == 0) fa.verdict[c] = fp12_is_one(r) ? GSV_PAIRING_TRUE : GSV_PAIRING_FALSE;
}

__global__ __launch_bounds__(64) void k_bn_final(FinalArgs fa) {
    __shared__ uint32_t lds[(FE_LDS_V0 + 48) * 64];  // per lane: the machine's operand A, a product's v0
    final_check<false>(fa, lds);
}
__global__ __launch_bounds__(64) void k_bn_final3(FinalArgs fa) {
    __shared__ uint32_t lds[108 * 64];
    final_check<true>(fa, lds);
}


// ---------------------------------------------------------------- synthetic workload (bench data)
// Not on the validation path.  Check i = e(aP, bQ) e(-bP, aQ) e(cP, dQ) e(-dP, cQ) == 1 with
// a, b, c, d = Keccak-256(le64(seed) || le64(i) || tag) truncated to 253 bits (nonzero), P, Q the
// G1 / G2 generators (curve.go:16-21, twist.go:20-32).  Every 8th check (i % 8 == 7) uses
// -(d+1)P (false); every 1024th (i % 1024 == 1023) also corrupts a coordinate to p (bad input).
struct g1j { fq x, y, z; };
// curve.go:143-172 dbl-2009-l
static BN_NI void g1_double_p(g1j* pc, const g1j* pa) {
    const g1j a = *pa;
    fq A = fq_store(fq_mul(a.x, a.x));
    fq B = fq_store(fq_mul(a.y, a.y));
    fq C = fq_store(fq_mul(B, B));
    auto t = fq_add(a.x, B);
    fq d = fq_store(fq_mul_small<2>(fq_sub(fq_sub(fq_mul(t, t), A), C)));
    fq e = fq_store(fq_mul_small<3>(A));
    g1j r;
    r.x = fq_store(fq_sub(fq_mul(e, e), fq_mul_small<2>(d)));
    r.y = fq_store(fq_sub(fq_mul(e, fq_sub(d, r.x)), fq_mul_small<8>(C)));
    r.z = fq_store(fq_mul_small<2>(fq_mul(a.y, a.z)));
    *pc = r;
}
// curve.go:63-141 add-2007-bl
static BN_NI void g1_add_p(g1j* pc, const g1j* pa, const g1j* pb) {
    const g1j a = *pa, b = *pb;
    if (fq_is_zero(a.z)) { *pc = b; return; }
    if (fq_is_zero(b.z)) { *pc = a; return; }
    fq z12 = fq_store(fq_mul(a.z, a.z));
    fq z22 = fq_store(fq_mul(b.z, b.z));
    fq u1 = fq_store(fq_mul(a.x, z22));
    fq u2 = fq_store(fq_mul(b.x, z12));
    fq s1 = fq_store(fq_mul(a.y, fq_mul(b.z, z22)));
    fq s2_ = fq_store(fq_mul(b.y, fq_mul(a.z, z12)));
    fq h = fq_store(fq_sub(u2, u1));
    bool xeq = fq_is_zero(h);
    auto h2 = fq_mul_small<2>(h);
    fq i = fq_store(fq_mul(h2, h2));
    fq j = fq_store(fq_mul(h, i));
    fq t = fq_store(fq_sub(s2_, s1));
    bool yeq = fq_is_zero(t);
    if (xeq && yeq) { g1_double_p(pc, pa); return; }
    fq r = fq_store(fq_mul_small<2>(t));
    fq v = fq_store(fq_mul(u1, i));
    g1j o;
    o.x = fq_store(fq_sub(fq_sub(fq_mul(r, r), j), fq_mul_small<2>(v)));
    o.y = fq_store(fq_sub(fq_mul(r, fq_sub(v, o.x)), fq_mul_small<2>(fq_mul(s1, j))));
    auto zs = fq_add(a.z, b.z);
    o.z = fq_store(fq_mul(fq_sub(fq_sub(fq_mul(zs, zs), z12), z22), h));
    *pc = o;
}
// k * P (k < 2^253 as 8 limbs, nonzero) -> affine Montgomery coordinates
GSV_DI void g1_mul_gen(fq& ox, fq& oy, const uint32_t k[8]) {
    g1j base{fq_c(FQ_ONE), fq_c(FQ_TWO), fq_c(FQ_ONE)};
    g1j sum{fq_zero(), fq_c(FQ_ONE), fq_zero()};
#pragma unroll 1
    for (int b = 252; b >= 0; b--) {
        g1j t;
        g1_double_p(&t, &sum);
        if ((k[b >> 5] >> (b & 31)) & 1u) g1_add_p(&sum, &t, &base);
        else sum = t;
    }
    fq zi = fq_inv(sum.z);
    fq zi2 = fq_store(fq_mul(zi, zi));
    ox = fq_store(fq_mul(sum.x, zi2));
    oy = fq_store(fq_mul(sum.y, fq_mul(zi2, zi)));
}
// a fixed point on the twist outside G2 (x = 12345 + 86416 i, tests/bn254_py.py
// twist_point_outside_g2(12345)), in the precompile encoding (imaginary part first)
__device__ constexpr uint8_t SYNTH_T[128] = {
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x01, 0x51, 0x90,
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x30, 0x39,
    0x2f, 0x7a, 0xba, 0x3d, 0x52, 0xda, 0x8d, 0x8d, 0x95, 0x21, 0x32, 0xa9, 0x9c, 0xd9, 0xdc, 0x90,
    0x4e, 0x51, 0x0a, 0x61, 0x17, 0x56, 0x54, 0xbe, 0x75, 0xa9, 0x5d, 0x0d, 0x2a, 0x12, 0xfc, 0x1d,
    0x13, 0x76, 0x85, 0x1a, 0x42, 0x91, 0x39, 0x13, 0xf7, 0xaf, 0xd2, 0x6c, 0x8b, 0x1c, 0x1a, 0x33,
    0x6d, 0xb5, 0xce, 0xd0, 0x33, 0x1c, 0x5c, 0x20, 0xbc, 0x3e, 0x7c, 0xdc, 0x57, 0xde, 0xdc, 0x27};
// k Q (Q the G2 generator), plus T (outside G2) when add_t: the sum is then on the twist and outside G2
GSV_DI void g2_mul_gen(g2a& o, const uint32_t k[8], bool add_t) {
    g2j base{fp2_const(FQ_TWIST_GEN_XX, FQ_TWIST_GEN_XY), fp2_const(FQ_TWIST_GEN_YX, FQ_TWIST_GEN_YY), fp2_one(),
             fp2_one()};
    g2j sum{fp2_zero(), fp2_one(), fp2_zero(), fp2_zero()};
#pragma unroll 1
    for (int b = 252; b >= 0; b--) {
        g2j t;
        g2_double_p(&t, &sum);
        if ((k[b >> 5] >> (b & 31)) & 1u) g2_add_p(&sum, &t, &base);
        else sum = t;
    }
    if (add_t) {
        g2j tj{fp2_zero(), fp2_zero(), fp2_one(), fp2_one()}, r;
        fp_unmarshal(tj.x.x, SYNTH_T);
        fp_unmarshal(tj.x.y, SYNTH_T + 32);
        fp_unmarshal(tj.y.x, SYNTH_T + 64);
        fp_unmarshal(tj.y.y, SYNTH_T + 96);
        g2_add_p(&r, &sum, &tj);
        sum = r;
    }
    fp2 zi = fp2_inv(sum.z);
    fp2 zi2 = s2(fp2_sqr(zi));
    o.x = s2(fp2_mul(sum.x, zi2));
    o.y = s2(fp2_mul(sum.y, fp2_mul(zi2, zi)));
}
GSV_DI void synth_scalar(uint32_t k[8], uint64_t seed, uint64_t i, uint32_t tag) {
    uint64_t a[25];
#pragma unroll
    for (int j = 0; j < 25; j++) a[j] = 0;
    a[0] = seed;
    a[1] = i;
    a[2] = (uint64_t)(tag & 0xFFFFFFu) | (0x01ull << 24);
    a[16] = 0x8000000000000000ULL;
    keccakf(a);
#pragma unroll
    for (int j = 0; j < 4; j++) {
        k[2 * j] = (uint32_t)a[j];
        k[2 * j + 1] = (uint32_t)(a[j] >> 32);
    }
    k[7] &= 0x1FFFFFFFu;  // < 2^253 < r
    if ((k[0] | k[1] | k[2] | k[3] | k[4] | k[5] | k[6] | k[7]) == 0) k[0] = 1;
}
// one (G1, G2) pair of the check: lane (check, j) for j = 0..3.  Classes by c mod 1024 (besides the
// false checks, c mod 8 == 7, whose fourth pair uses -(d+1)P):
//   100: pairs 0 and 1 have G1 = infinity (skipped by PairingCheck, bn256.go:318) -> true
//   200: pairs 0 and 1 have G2 = infinity -> true
//   300: pair 1 is (infinity, bQ + T) with T outside G2: G2.Unmarshal rejects it before the infinity
//        pair is skipped (core/vm/contracts.go:341-352, twist.go:60-62) -> bad input
//   400: pair 1 is (infinity, bQ with y.re's low bit flipped): off the twist -> bad input
//   500: pair 3's G2 point is cQ + T (outside G2) -> bad input
//   1023: pair 2's G1 x coordinate == p -> bad input
__global__ __launch_bounds__(64) void k_bn_synth(uint64_t seed, uint32_t nchecks, uint8_t* __restrict__ out,
                                                 uint8_t* __restrict__ expect) {
    uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= nchecks * 4u) return;
    uint32_t c = id >> 2, j = id & 3u;
    uint32_t s1[8], s2w[8];
    // pair j: (x P, y Q) with (x, y) = (a, b), (-b, a), (c, d), (-d', c)
    const uint32_t tags[4] = {0x61u, 0x62u, 0x63u, 0x64u};  // "a" "b" "c" "d"
    uint32_t tx = (j == 0) ? tags[0] : (j == 1) ? tags[1] : (j == 2) ? tags[2] : tags[3];
    uint32_t ty = (j == 0) ? tags[1] : (j == 1) ? tags[0] : (j == 2) ? tags[3] : tags[2];
    synth_scalar(s1, seed, c, tx);
    synth_scalar(s2w, seed, c, ty);
    const uint32_t cls = c % 1024u;
    bool is_false = (c % 8u) == 7u, is_bad = cls == 1023u || cls == 300u || cls == 400u || cls == 500u;
    bool inf_g1 = (cls == 100u && j <= 1u) || ((cls == 300u || cls == 400u) && j == 1u);
    bool inf_g2 = cls == 200u && j <= 1u;
    bool add_t = (cls == 300u && j == 1u) || (cls == 500u && j == 3u);
    bool off_twist = cls == 400u && j == 1u;
    if (j == 3 && is_false) {  // d + 1 (no overflow: d < 2^253)
        uint64_t cy = 1;
#pragma unroll
        for (int w = 0; w < 8; w++) {
            cy += s1[w];
            s1[w] = (uint32_t)cy;
            cy >>= 32;
        }
    }
    fq px, py;
    g1_mul_gen(px, py, s1);
    if (j & 1u) py = fq_store(fq_neg(py));  // -xP
    g2a q;
    g2_mul_gen(q, s2w, add_t);
    uint8_t* o = out + (size_t)c * 768 + j * 192;
    fp_marshal(o, px);
    fp_marshal(o + 32, py);
    fp_marshal(o + 64, q.x.x);
    fp_marshal(o + 96, q.x.y);
    fp_marshal(o + 128, q.y.x);
    fp_marshal(o + 160, q.y.y);
    if (inf_g1)
        for (int i = 0; i < 64; i++) o[i] = 0;
    if (inf_g2)
        for (int i = 64; i < 192; i++) o[i] = 0;
    if (off_twist) o[191] ^= 1u;  // stays < p unless y.re == p - 1 (then coordinate == p: also bad)
    if (j == 2 && cls == 1023u) {  // coordinate == p: bn256 "coordinate equals modulus"
#pragma unroll
        for (int i = 0; i < 8; i++) {
            uint32_t w = BN_P_W[7 - i];
            o[4 * i] = (uint8_t)(w >> 24);
            o[4 * i + 1] = (uint8_t)(w >> 16);
            o[4 * i + 2] = (uint8_t)(w >> 8);
            o[4 * i + 3] = (uint8_t)w;
        }
    }
    if (j == 0 && expect)
        expect[c] = is_bad ? GSV_PAIRING_BAD_INPUT : is_false ? GSV_PAIRING_FALSE : GSV_PAIRING_TRUE;
}

}  // namespace bn


hipError_t launch_bn256_synth(uint64_t seed, uint32_t nchecks, uint8_t* d_out, uint8_t* d_expect, hipStream_t st) {
    if (nchecks == 0) return hipSuccess;
    uint32_t lanes = nchecks * 4u;
    hipLaunchKernelGGL(bn::k_bn_synth, dim3((lanes + 63) / 64), dim3(64), 0, st, seed, nchecks, d_out, d_expect);
    return hipGetLastError();
}

hipError_t launch_bn256_pairing(const uint8_t* d_in, const uint64_t* d_pair_src, uint32_t npairs,
                                const uint32_t* d_lane_first, const uint32_t* d_pidx, uint32_t nlanes,
                                const uint32_t* d_check_lane, const uint8_t* d_cbad, uint32_t nchecks,
                                uint8_t* d_pstat, uint32_t* d_lines, uint8_t* d_lstat, uint32_t* d_fv,
                                uint32_t* d_fws, uint32_t maxl, uint8_t* d_verdict, int layout, hipStream_t st, void (*timer_begin)(void*, int),
                                void (*timer_end)(void*, int), void* tctx) {
    // the pairs: decode, curve checks, lines, G2 membership (k_bn_lines, or its two-wave form LINESW2)
    const uint8_t* d_use = d_pstat;
    if (npairs) {
        if (timer_begin) timer_begin(tctx, GSV_K_BN_PREPARE);
        if (layout & GSV_BN_LAYOUT_LINESW2)
            hipLaunchKernelGGL(bn::k_bn_lines_w2, dim3((npairs + 63) / 64), dim3(64), 0, st, d_in, d_pair_src, npairs,
                               d_lines, d_pstat);
        else
            hipLaunchKernelGGL(bn::k_bn_lines, dim3((npairs + 63) / 64), dim3(64), 0, st, d_in, d_pair_src, npairs,
                               d_lines, d_pstat);
        if (timer_end) timer_end(tctx, GSV_K_BN_PREPARE);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (nchecks) {
        // the tail: Miller loop + final exponentiation at ~one wave per SIMD (marking after the Miller
        // loop instead, or not at all, measured the same or lower: profiles/r02/ab_pipeline.txt)
        if (timer_begin) timer_begin(tctx, GSV_HOOK_TAIL);
        if (timer_begin) timer_begin(tctx, GSV_K_PAIRING);
        if (layout & GSV_BN_LAYOUT_MILLER2)
            hipLaunchKernelGGL(bn::k_bn_miller2, dim3((2 * nlanes + 63) / 64), dim3(64), 0, st, d_lane_first, nlanes,
                               d_pidx, d_use, d_lines, npairs, d_lstat, d_fv);
        else if (layout & GSV_BN_LAYOUT_MILLERL)
            hipLaunchKernelGGL(bn::k_bn_miller_l, dim3((nlanes + 63) / 64), dim3(64), 0, st, d_lane_first, nlanes,
                               d_pidx, d_use, d_lines, npairs, d_lstat, d_fv);
        else if (layout & GSV_BN_LAYOUT_MILLERW2)
            hipLaunchKernelGGL(bn::k_bn_miller_w2, dim3((nlanes + 63) / 64), dim3(64), 0, st, d_lane_first, nlanes,
                               d_pidx, d_use, d_lines, npairs, d_lstat, d_fv);
        else
            hipLaunchKernelGGL(bn::k_bn_miller, dim3((nlanes + 63) / 64), dim3(64), 0, st, d_lane_first, nlanes,
                               d_pidx, d_use, d_lines, npairs, d_lstat, d_fv);
        if (timer_end) timer_end(tctx, GSV_K_PAIRING);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        if (timer_begin) timer_begin(tctx, GSV_K_BN_FINAL);
        bn::FinalArgs fa{d_check_lane, nchecks, d_cbad, d_lstat, d_fv, nlanes, d_verdict, d_fws, maxl};
        if (layout & GSV_BN_LAYOUT_FINAL3)
            hipLaunchKernelGGL(bn::k_bn_final3, dim3((nchecks + bn::FINAL3_PER_WAVE - 1) / bn::FINAL3_PER_WAVE),
                               dim3(64), 0, st, fa);
        else
            hipLaunchKernelGGL(bn::k_bn_final, dim3((nchecks + 63) / 64), dim3(64), 0, st, fa);
        if (timer_end) timer_end(tctx, GSV_K_BN_FINAL);
    }
    return hipGetLastError();
}

}  // namespace gsv

GSV_OPCOUNT_READER(bn256)

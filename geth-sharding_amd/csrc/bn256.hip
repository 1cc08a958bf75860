// Batched BN254 PairingCheck on gfx950 (bn256.PairingCheck as driven by the bn256Pairing
// precompile, core/vm/contracts.go:333-360; crypto/bn256/cloudflare/bn256.go:313-327).
//
// One lane per pair for decode + G2 subgroup check, one lane per check for the multi-Miller loop
// and the final exponentiation.  Three launches:
//   k_bn_prepare  decode the 192-byte pair (bn256.go:120-164 G1.Unmarshal, :256-306 G2.Unmarshal):
//                 coordinates < p, Montgomery encode, infinity detection, y^2 = x^3 + 3 on G1,
//                 on-twist + subgroup membership on G2 (twist.go:47-63)  -> pair status + points
//   k_bn_miller   optimal-ate Miller loop (optate.go:122-210) over all of a check's pairs with one
//                 shared accumulator (the product of the per-pair values) -> F_p^12 per check
//   k_bn_final    finalExponentiation (optate.go:212-261), IsOne          -> verdict per check
// HBM layout is structure-of-arrays, word-major ([word][pair]), so each lane's word loads and
// stores coalesce across the wave.
#include "opcount.cuh"
#include "bn254_dev.cuh"
#include "gsv_internal.h"
#include "keccak_dev.cuh"

namespace gsv {
namespace bn {

// ---------------------------------------------------------------- F_p^12 (gfp12.go)
GSV_DI void fp12_one(fp12& e) { fp6_zero(e.x); fp6_one(e.y); }
GSV_DI bool fp12_is_one(const fp12& e) {
    fp one;
    fp_const(one, BN_ONE);
    return fp2_is_zero(e.x.x) && fp2_is_zero(e.x.y) && fp2_is_zero(e.x.z) && fp2_is_zero(e.y.x) &&
           fp2_is_zero(e.y.y) && fp_is_zero(e.y.z.x) && fp_eq(e.y.z.y, one);
}
GSV_DI void fp12_conj(fp12& e, const fp12& a) { fp6_neg(e.x, a.x); e.y = a.y; }
// gfp12.go:60-66
static BN_NI void fp12_frob_p(fp12* pe, const fp12* pa) {
    const fp12 a = *pa;
    fp12& e = *pe;
    fp6 t;
    fp6_frob(t, a.x);
    fp6_frob(e.y, a.y);
    fp2 k;
    fp2_const(k, XI_P1_6_X, XI_P1_6_Y);
    fp6_mul_fp2(e.x, t, k);
}
GSV_DI void fp12_frob(fp12& e, const fp12& a) { fp12_frob_p(&e, &a); }
// gfp12.go:68-74
static BN_NI void fp12_frob_p2_p(fp12* pe, const fp12* pa) {
    const fp12 a = *pa;
    fp12& e = *pe;
    fp6 t;
    fp6_frob_p2(t, a.x);
    fp k;
    fp_const(k, XI_PSQ1_6);
    fp6_mul_fp(e.x, t, k);
    fp6_frob_p2(e.y, a.y);
}
GSV_DI void fp12_frob_p2(fp12& e, const fp12& a) { fp12_frob_p2_p(&e, &a); }
// gfp12.go:94-106
// Karatsuba over F_p^6: x = (a.x + a.y)(b.x + b.y) - a.x b.x - a.y b.y equals the reference's
// a.x b.y + b.x a.y, so 3 F_p^6 products instead of 4 give the same canonical words.
static BN_NI void fp12_mul_p(fp12* pe, const fp12* pa, const fp12* pb) {
    const fp12& a = *pa;
    const fp12& b = *pb;
    fp12& e = *pe;
    fp6 v0, v1, sa, sb, tx;
    // F_p^6 products inlined (one out-of-line call level fewer: 11.5 -> 10.7 ms per 65,536 final exps)
    fp6_mul_i(v0, a.x, b.x);
    fp6_mul_i(v1, a.y, b.y);
    fp6_add(sa, a.x, a.y);
    fp6_add(sb, b.x, b.y);
    fp6_mul_i(tx, sa, sb);
    fp6_sub(tx, tx, v0);
    fp6_sub(tx, tx, v1);
    fp6_mul_tau(v0, v0);
    e.x = tx;
    fp6_add(e.y, v1, v0);
}
GSV_DI void fp12_mul(fp12& e, const fp12& a, const fp12& b) { fp12_mul_p(&e, &a, &b); }
// gfp12.go:129-143
// (the _i form is always inlined: the Miller loop's accumulator never leaves VGPRs)
GSV_DI void fp12_sqr_i(fp12& e, const fp12& a_) {
    const fp12 a = a_;
    fp6 v0, t, ty;
    fp6_mul_i(v0, a.x, a.y);
    fp6_mul_tau(t, a.x);
    fp6_add(t, a.y, t);
    fp6_add(ty, a.x, a.y);
    fp6_mul_i(ty, ty, t);
    fp6_sub(ty, ty, v0);
    fp6_mul_tau(t, v0);
    fp6_sub(ty, ty, t);
    fp6_add(e.x, v0, v0);
    e.y = ty;
}
static BN_NI void fp12_sqr_p(fp12* pe, const fp12* pa) { fp12_sqr_i(*pe, *pa); }
GSV_DI void fp12_sqr(fp12& e, const fp12& a) { fp12_sqr_p(&e, &a); }
// Squaring in the cyclotomic subgroup (Granger-Scott, "Faster squaring in the cyclotomic subgroup of
// sixth degree extensions", PKC 2010): 9 F_p^2 squarings instead of two F_p^6 products.  Valid for
// every element of norm 1 over F_p^6 — everything finalExponentiation squares after its easy part
// (optate.go:218-222) — and it yields the same field element (hence the same canonical words) as
// fp12_sqr there.  Coefficients of a = sum c_k w^k over F_p^2 (w^2 = tau, tau^3 = xi):
// c0 = y.z, c1 = x.z, c2 = y.y, c3 = x.y, c4 = y.x, c5 = x.x.
GSV_DI void fp12_cyclo_sqr_i(fp12& e, const fp12& pa_) {
    const fp12 a = pa_;
    const fp2 &x0 = a.y.z, &x1 = a.y.y, &x2 = a.y.x, &x3 = a.x.z, &x4 = a.x.y, &x5 = a.x.x;
    fp2 t0, t1, t2, t3, t4, t5, t6, t7, t8, u;
    fp2_sqr(t0, x4);
    fp2_sqr(t1, x0);
    fp2_add(u, x4, x0);
    fp2_sqr(t6, u);
    fp2_sub(t6, t6, t0);
    fp2_sub(t6, t6, t1);  // 2 x4 x0
    fp2_sqr(t2, x2);
    fp2_sqr(t3, x3);
    fp2_add(u, x2, x3);
    fp2_sqr(t7, u);
    fp2_sub(t7, t7, t2);
    fp2_sub(t7, t7, t3);  // 2 x2 x3
    fp2_sqr(t4, x5);
    fp2_sqr(t5, x1);
    fp2_add(u, x5, x1);
    fp2_sqr(t8, u);
    fp2_sub(t8, t8, t4);
    fp2_sub(t8, t8, t5);
    fp2_mul_xi(t8, t8);  // 2 x5 x1 xi
    fp2_mul_xi(t0, t0);
    fp2_add(t0, t0, t1);  // x4^2 xi + x0^2
    fp2_mul_xi(t2, t2);
    fp2_add(t2, t2, t3);  // x2^2 xi + x3^2
    fp2_mul_xi(t4, t4);
    fp2_add(t4, t4, t5);  // x5^2 xi + x1^2
    // c0' = 3 t0 - 2 x0, c2' = 3 t2 - 2 x1, c4' = 3 t4 - 2 x2
    fp2_sub(u, t0, x0);
    fp2_add(u, u, u);
    fp2_add(e.y.z, u, t0);
    fp2_sub(u, t2, x1);
    fp2_add(u, u, u);
    fp2_add(e.y.y, u, t2);
    fp2_sub(u, t4, x2);
    fp2_add(u, u, u);
    fp2_add(e.y.x, u, t4);
    // c1' = 3 t8 + 2 x3, c3' = 3 t6 + 2 x4, c5' = 3 t7 + 2 x5
    fp2_add(u, t8, x3);
    fp2_add(u, u, u);
    fp2_add(e.x.z, u, t8);
    fp2_add(u, t6, x4);
    fp2_add(u, u, u);
    fp2_add(e.x.y, u, t6);
    fp2_add(u, t7, x5);
    fp2_add(u, u, u);
    fp2_add(e.x.x, u, t7);
}
static BN_NI void fp12_cyclo_sqr_p(fp12* pe, const fp12* pa) { fp12_cyclo_sqr_i(*pe, *pa); }
GSV_DI void fp12_cyclo_sqr(fp12& e, const fp12& a) { fp12_cyclo_sqr_p(&e, &a); }
// gfp12.go:145-160
GSV_DI void fp12_inv(fp12& e, const fp12& a) {
    fp6 t1, t2;
    fp6_sqr(t1, a.x);
    fp6_sqr(t2, a.y);
    fp6_mul_tau(t1, t1);
    fp6_sub(t1, t2, t1);
    fp6_inv(t2, t1);
    fp6 nx;
    fp6_neg(nx, a.x);
    fp6_mul(e.x, nx, t2);
    fp6_mul(e.y, a.y, t2);
}
// NAF of u: u = U_NAF_POS - U_NAF_NEG, digit 62 = +1 (also used by the G2 subgroup predicate)
constexpr uint64_t U_NAF_POS = 0x450a14044a890a01ULL;
constexpr uint64_t U_NAF_NEG = 0x0020815000200010ULL;
// gfp12.go:113-127 with power = u; only called on cyclotomic-subgroup elements (the final
// exponentiation's hard part), where a^-1 = conj(a): the NAF of u needs 23 products instead of the
// 27 of its binary expansion, and the result is the same field element a^u (same canonical words).
// (Inlining the products too, down to the F_p product, was measured slower: 14.6 -> 17.9 ms per
// 65,536 final exponentiations, heavy spills of the 96-word operands.)
static BN_NI void fp12_exp_u(fp12* c, const fp12* a) {
    fp12 sum = *a;  // the leading digit: 1^2 * a
#pragma unroll 1
    for (int i = 61; i >= 0; i--) {
        fp12_cyclo_sqr_i(sum, sum);  // inlined (12.5 -> 11.7 ms per 65,536 final exps); products stay out of line
        bool pos = (U_NAF_POS >> i) & 1, neg = (U_NAF_NEG >> i) & 1;
        if (pos || neg) {
            fp12 t = *a;
            if (neg) fp6_neg(t.x, t.x);
            fp12_mul(sum, sum, t);
        }
    }
    *c = sum;
}

// ---- three-lane cooperative exponentiation by u, for batches too small to give every SIMD a wave.
// The three lanes of a triple (wave lanes base, base+1, base+2) all hold the whole F_p^12 value;
// each operation is split into three equal parts selected by the lane's role (same instruction
// stream, different operands: no divergence), and the parts are exchanged with ds_bpermute.  The
// dependent chain per exp_u step becomes a third as long; every part computes the same formula as
// the one-lane routine, so results are the same canonical words.
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
static BN_NI void fp12_cyclo_sqr3(fp12* pe, const fp12* pa, int role, int base) {
    const fp12 a = *pa;
    const fp2 &x0 = a.y.z, &x1 = a.y.y, &x2 = a.y.x, &x3 = a.x.z, &x4 = a.x.y, &x5 = a.x.x;
    fp2 p = role == 0 ? x4 : role == 1 ? x2 : x5;
    fp2 q = role == 0 ? x0 : role == 1 ? x3 : x1;
    fp2 m1 = role == 0 ? x0 : role == 1 ? x1 : x2;
    fp2 m2 = role == 0 ? x4 : role == 1 ? x5 : x3;
    fp2 tp, tq, tc, u, sq, tcx;
    fp2_sqr(tp, p);
    fp2_sqr(tq, q);
    fp2_add(u, p, q);
    fp2_sqr(tc, u);
    fp2_sub(tc, tc, tp);
    fp2_sub(tc, tc, tq);  // 2 p q
    fp2_mul_xi(sq, tp);
    fp2_add(sq, sq, tq);  // p^2 xi + q^2
    fp2_mul_xi(tcx, tc);
    if (role == 2) tc = tcx;  // 2 x5 x1 xi
    struct { fp2 lo, hi; } mine, all[3];
    fp2_sub(u, sq, m1);
    fp2_add(u, u, u);
    fp2_add(mine.lo, u, sq);  // 3 sq - 2 m1
    fp2_add(u, tc, m2);
    fp2_add(u, u, u);
    fp2_add(mine.hi, u, tc);  // 3 tc + 2 m2
    gather3(all, mine, base);
    pe->y.z = all[0].lo;
    pe->x.y = all[0].hi;
    pe->y.y = all[1].lo;
    pe->x.x = all[1].hi;
    pe->y.x = all[2].lo;
    pe->x.z = all[2].hi;
}
// fp12_mul_p's three F_p^6 products, one per role
static BN_NI void fp12_mul3(fp12* pe, const fp12* pa, const fp12* pb, int role, int base) {
    const fp12 a = *pa, b = *pb;
    fp6 sa, sb, l, r, prod, v[3], tx;
    fp6_add(sa, a.x, a.y);
    fp6_add(sb, b.x, b.y);
    l = role == 0 ? a.x : role == 1 ? a.y : sa;
    r = role == 0 ? b.x : role == 1 ? b.y : sb;
    fp6_mul_i(prod, l, r);
    gather3(v, prod, base);
    fp6_sub(tx, v[2], v[0]);
    fp6_sub(tx, tx, v[1]);
    fp6_mul_tau(v[0], v[0]);
    pe->x = tx;
    fp6_add(pe->y, v[1], v[0]);
}
static BN_NI void fp12_exp_u3(fp12* c, const fp12* a, int role, int base) {
    fp12 sum = *a;
#pragma unroll 1
    for (int i = 61; i >= 0; i--) {
        fp12_cyclo_sqr3(&sum, &sum, role, base);
        bool pos = (U_NAF_POS >> i) & 1, neg = (U_NAF_NEG >> i) & 1;
        if (pos || neg) {
            fp12 t = *a;
            if (neg) fp6_neg(t.x, t.x);
            fp12_mul3(&sum, &sum, &t, role, base);
        }
    }
    *c = sum;
}

// ---------------------------------------------------------------- twist points (twist.go)
// twist.go:136-162 dbl-2009-l (t is not updated, as in the reference)
GSV_DI void g2_double_i(g2j& c, const g2j& pa_) {
    const g2j a = pa_;
    fp2 A, B, C, t, t2, d, e, f;
    fp2_sqr(A, a.x);
    fp2_sqr(B, a.y);
    fp2_sqr(C, B);
    fp2_add(t, a.x, B);
    fp2_sqr(t2, t);
    fp2_sub(t, t2, A);
    fp2_sub(t2, t, C);
    fp2_add(d, t2, t2);
    fp2_add(t, A, A);
    fp2_add(e, t, A);
    fp2_sqr(f, e);
    g2j r;
    fp2_add(t, d, d);
    fp2_sub(r.x, f, t);
    fp2_add(t, C, C);
    fp2_add(t2, t, t);
    fp2_add(t, t2, t2);
    fp2_sub(r.y, d, r.x);
    fp2_mul(t2, e, r.y);
    fp2_sub(r.y, t2, t);
    fp2_mul(t, a.y, a.z);
    fp2_add(r.z, t, t);
    r.t = a.t;
    c = r;
}
static BN_NI void g2_double_p(g2j* pc, const g2j* pa) { g2_double_i(*pc, *pa); }
GSV_DI void g2_double(g2j& c, const g2j& a) { g2_double_p(&c, &a); }
// twist.go:73-134 add-2007-bl with its infinity / doubling cases
GSV_DI void g2_add_i(g2j& c, const g2j& pa_, const g2j& pb_) {
    const g2j a = pa_, b = pb_;
    if (fp2_is_zero(a.z)) { c = b; return; }
    if (fp2_is_zero(b.z)) { c = a; return; }
    fp2 z12, z22, u1, u2, t, s1, s2, h, i, j, r, v, t4, t6;
    fp2_sqr(z12, a.z);
    fp2_sqr(z22, b.z);
    fp2_mul(u1, a.x, z22);
    fp2_mul(u2, b.x, z12);
    fp2_mul(t, b.z, z22);
    fp2_mul(s1, a.y, t);
    fp2_mul(t, a.z, z12);
    fp2_mul(s2, b.y, t);
    fp2_sub(h, u2, u1);
    bool xeq = fp2_is_zero(h);
    fp2_add(t, h, h);
    fp2_sqr(i, t);
    fp2_mul(j, h, i);
    fp2_sub(t, s2, s1);
    bool yeq = fp2_is_zero(t);
    if (xeq && yeq) { g2_double(c, a); return; }
    fp2_add(r, t, t);
    fp2_mul(v, u1, i);
    g2j o;
    fp2_sqr(t4, r);
    fp2_add(t, v, v);
    fp2_sub(t6, t4, j);
    fp2_sub(o.x, t6, t);
    fp2_sub(t, v, o.x);
    fp2_mul(t4, s1, j);
    fp2_add(t6, t4, t4);
    fp2_mul(t4, r, t);
    fp2_sub(o.y, t4, t6);
    fp2_add(t, a.z, b.z);
    fp2_sqr(t4, t);
    fp2_sub(t, t4, z12);
    fp2_sub(t4, t, z22);
    fp2_mul(o.z, t4, h);
    o.t = a.t;
    c = o;
}
static BN_NI void g2_add_p(g2j* pc, const g2j* pa, const g2j* pb) { g2_add_i(*pc, *pa, *pb); }
GSV_DI void g2_add(g2j& c, const g2j& a, const g2j& b) { g2_add_p(&c, &a, &b); }
// c = a + q with q affine (z = 1): madd-2007-bl, 8M + 3S instead of the general 11M + 5S.  Used only
// inside the subgroup predicate, whose boolean outcome does not depend on the formulas chosen.
GSV_DI void g2_add_mixed_i(g2j& c, const g2j& pa_, const g2a& pq_) {
    const g2j a = pa_;
    const g2a q = pq_;
    if (fp2_is_zero(a.z)) {
        c.x = q.x;
        c.y = q.y;
        fp2_one(c.z);
        fp2_one(c.t);
        return;
    }
    fp2 z12, u2, s2, h, t, i, j, r, v, t4, t6;
    fp2_sqr(z12, a.z);
    fp2_mul(u2, q.x, z12);
    fp2_mul(t, a.z, z12);
    fp2_mul(s2, q.y, t);
    fp2_sub(h, u2, a.x);
    fp2_sub(t, s2, a.y);
    if (fp2_is_zero(h) && fp2_is_zero(t)) {  // out of line: never taken on the hot path
        g2_double(c, a);
        return;
    }
    fp2_add(r, h, h);
    fp2_sqr(i, r);
    fp2_mul(j, h, i);
    fp2_add(r, t, t);
    fp2_mul(v, a.x, i);
    g2j o;
    fp2_sqr(t4, r);
    fp2_add(t, v, v);
    fp2_sub(t6, t4, j);
    fp2_sub(o.x, t6, t);
    fp2_sub(t, v, o.x);
    fp2_mul(t4, a.y, j);
    fp2_add(t6, t4, t4);
    fp2_mul(t4, r, t);
    fp2_sub(o.y, t4, t6);
    fp2_mul(o.z, a.z, h);
    fp2_add(o.z, o.z, o.z);  // (Z1 + 1)^2 - Z1^2 - 1 = 2 Z1
    o.t = a.t;
    c = o;
}
static BN_NI void g2_add_mixed_p(g2j* pc, const g2j* pa, const g2a* pq) { g2_add_mixed_i(*pc, *pa, *pq); }
// psi(X : Y : Z) = (conj(X) xi^((p-1)/3) : conj(Y) xi^((p-1)/2) : conj(Z)) — the p-power
// Frobenius carried through the twist isomorphism (optate.go:173-176 applies it to affine Q)
GSV_DI void g2_psi(g2j& o, const g2j& a) {
    fp2 k, c;
    fp2_conj(c, a.x);
    fp2_const(k, XI_P1_3_X, XI_P1_3_Y);
    fp2_mul(o.x, c, k);
    fp2_conj(c, a.y);
    fp2_const(k, XI_P1_2_X, XI_P1_2_Y);
    fp2_mul(o.y, c, k);
    fp2_conj(o.z, a.z);
    o.t = a.t;
}
// twist.go:47-63: y^2 == x^3 + 3/xi and Q in the order-r subgroup
GSV_DI bool g2_in_subgroup(const g2a* q) {
    fp2 y2, x3, b;
    fp2_sqr(y2, q->y);
    fp2_sqr(x3, q->x);
    fp2_mul(x3, x3, q->x);
    fp2_const(b, TWIST_B_X, TWIST_B_Y);
    fp2_add(x3, x3, b);
    if (!fp2_eq(y2, x3)) return false;
    // The reference decides membership with Order*Q == infinity (twist.go:60-62, 254-bit
    // double-and-add).  We decide the same predicate with the endomorphism psi (the
    // untwist-Frobenius-twist map the Miller loop already uses for Q1, optate.go:173-176):
    //   [r]Q == O  <=>  [u+1]Q + psi([u]Q) + psi^2([u]Q) == psi^3([2u]Q)
    // for every Q on E'(F_p^2) of BN254 (Dai-Lin-Zhao-Zhou, eprint 2022/348, sec. 3 and 5.1):
    // a 63-bit multiplication instead of a 254-bit one.  Checked against the oracle's
    // Order*Q on random points inside and outside G2 (tests/test_gpu_bn256.py).
    g2j a;
    a.x = q->x;
    a.y = q->y;
    fp2_one(a.z);
    fp2_one(a.t);
    // [u]Q, u = 4965661367192848881 (63 bits), NAF digits (24 nonzero instead of 28 set bits), mixed
    // additions of the affine +-Q
    g2a mq;
    mq.x = q->x;
    fp2_neg(mq.y, q->y);
    g2j uq = a;  // leading digit +1 at bit 62
    // inlined down to the F_p product: the running point stays in VGPRs
#pragma unroll 1
    for (int i = 61; i >= 0; i--) {
        g2_double_i(uq, uq);
        bool pos = (U_NAF_POS >> i) & 1, neg = (U_NAF_NEG >> i) & 1;
        if (pos || neg) g2_add_mixed_i(uq, uq, neg ? mq : *q);
    }
    g2j lhs, p1, p2, rhs, tmp;
    g2_add_i(lhs, uq, a);          // [u+1]Q
    g2_psi(p1, uq);              // psi([u]Q)
    g2_psi(p2, p1);              // psi^2([u]Q)
    g2_add_i(lhs, lhs, p1);
    g2_add_i(lhs, lhs, p2);
    g2_double_i(tmp, uq);          // [2u]Q
    g2_psi(rhs, tmp);
    g2_psi(rhs, rhs);
    g2_psi(rhs, rhs);            // psi^3([2u]Q)
    fp2_neg(rhs.y, rhs.y);
    g2_add_i(tmp, lhs, rhs);       // lhs - rhs
    return fp2_is_zero(tmp.z);
}

// ---------------------------------------------------------------- Miller loop (optate.go)
// optate.go:3-50 (mixed addition r + p, p affine with t = 1; r2 = p.y^2)
GSV_DI void line_add_i(fp2& a, fp2& b, fp2& c, g2j& r, const g2a& pp, const g1a& pq, const fp2& pr2) {
    const g2a p = pp;
    const g1a q = pq;
    const fp2 r2 = pr2;
    fp2 B, D, H, I, E, J, L1, V, t, t2;
    fp2_mul(B, p.x, r.t);
    fp2_add(D, p.y, r.z);
    fp2_sqr(D, D);
    fp2_sub(D, D, r2);
    fp2_sub(D, D, r.t);
    fp2_mul(D, D, r.t);
    fp2_sub(H, B, r.x);
    fp2_sqr(I, H);
    fp2_add(E, I, I);
    fp2_add(E, E, E);
    fp2_mul(J, H, E);
    fp2_sub(L1, D, r.y);
    fp2_sub(L1, L1, r.y);
    fp2_mul(V, r.x, E);
    g2j o;
    fp2_sqr(o.x, L1);
    fp2_sub(o.x, o.x, J);
    fp2_sub(o.x, o.x, V);
    fp2_sub(o.x, o.x, V);
    fp2_add(o.z, r.z, H);
    fp2_sqr(o.z, o.z);
    fp2_sub(o.z, o.z, r.t);
    fp2_sub(o.z, o.z, I);
    fp2_sub(t, V, o.x);
    fp2_mul(t, t, L1);
    fp2_mul(t2, r.y, J);
    fp2_add(t2, t2, t2);
    fp2_sub(o.y, t, t2);
    fp2_sqr(o.t, o.z);
    fp2_add(t, p.y, o.z);
    fp2_sqr(t, t);
    fp2_sub(t, t, r2);
    fp2_sub(t, t, o.t);
    fp2_mul(t2, L1, p.x);
    fp2_add(t2, t2, t2);
    fp2_sub(a, t2, t);
    fp2_mul_fp(c, o.z, q.y);
    fp2_add(c, c, c);
    fp2_neg(b, L1);
    fp2_mul_fp(b, b, q.x);
    fp2_add(b, b, b);
    r = o;
}
static BN_NI void line_add_p(fp2* pa, fp2* pb, fp2* pc, g2j* pr, const g2a* pp, const g1a* pq, const fp2* pr2) {
    line_add_i(*pa, *pb, *pc, *pr, *pp, *pq, *pr2);
}
GSV_DI void line_add(fp2& a, fp2& b, fp2& c, g2j& r, const g2a& p, const g1a& q, const fp2& r2) {
    line_add_p(&a, &b, &c, &r, &p, &q, &r2);
}
// optate.go:52-92
GSV_DI void line_double_i(fp2& a, fp2& b, fp2& c, g2j& r, const g1a& pq) {
    const g1a q = pq;
    fp2 A, B, C, D, E, G, t;
    fp2_sqr(A, r.x);
    fp2_sqr(B, r.y);
    fp2_sqr(C, B);
    fp2_add(D, r.x, B);
    fp2_sqr(D, D);
    fp2_sub(D, D, A);
    fp2_sub(D, D, C);
    fp2_add(D, D, D);
    fp2_add(E, A, A);
    fp2_add(E, E, A);
    fp2_sqr(G, E);
    g2j o;
    fp2_sub(o.x, G, D);
    fp2_sub(o.x, o.x, D);
    fp2_add(o.z, r.y, r.z);
    fp2_sqr(o.z, o.z);
    fp2_sub(o.z, o.z, B);
    fp2_sub(o.z, o.z, r.t);
    fp2_sub(o.y, D, o.x);
    fp2_mul(o.y, o.y, E);
    fp2_add(t, C, C);
    fp2_add(t, t, t);
    fp2_add(t, t, t);
    fp2_sub(o.y, o.y, t);
    fp2_sqr(o.t, o.z);
    fp2_mul(t, E, r.t);
    fp2_add(t, t, t);
    fp2_neg(b, t);
    fp2_mul_fp(b, b, q.x);
    fp2_add(a, r.x, E);
    fp2_sqr(a, a);
    fp2_sub(a, a, A);
    fp2_sub(a, a, G);
    fp2_add(t, B, B);
    fp2_add(t, t, t);
    fp2_sub(a, a, t);
    fp2_mul(c, o.z, r.t);
    fp2_add(c, c, c);
    fp2_mul_fp(c, c, q.y);
    r = o;
}
static BN_NI void line_double_p(fp2* pa, fp2* pb, fp2* pc, g2j* pr, const g1a* pq) {
    line_double_i(*pa, *pb, *pc, *pr, *pq);
}
GSV_DI void line_double(fp2& a, fp2& b, fp2& c, g2j& r, const g1a& q) { line_double_p(&a, &b, &c, &r, &q); }
// optate.go:94-112
GSV_DI void mul_line_i(fp12& ret, const fp2& a, const fp2& b, const fp2& c) {
    // ordered (in place) so that at most ret + one F_p^6 temporary + the line are live at a time
    fp6 a2;
    fp2 bc;
    fp6_mul_sparse_i(a2, ret.x, a, b);   // (0, a, b) * ret.x
    fp6_add(ret.x, ret.x, ret.y);        // s = ret.x + ret.y
    fp6_mul_fp2_i(ret.y, ret.y, c);      // t3
    fp2_add(bc, b, c);
    fp6_mul_sparse_i(ret.x, ret.x, a, bc);  // s * (0, a, b + c)
    fp6_sub(ret.x, ret.x, a2);
    fp6_sub(ret.x, ret.x, ret.y);
    fp6_mul_tau(a2, a2);
    fp6_add(ret.y, ret.y, a2);
}
static BN_NI void mul_line(fp12* ret, const fp2* a, const fp2* b, const fp2* c) { mul_line_i(*ret, *a, *b, *c); }

// optate.go:122-210 for affine q (twist) and p (G1), neither at infinity
GSV_DI void miller(fp12& ret, const g2a& A, const g1a& B) {
    fp12_one(ret);
    g2j r;
    r.x = A.x;
    r.y = A.y;
    fp2_one(r.z);
    fp2_one(r.t);
    fp2 r2, a, b, c;
    fp2_sqr(r2, A.y);
    g2a mA;
    mA.x = A.x;
    fp2_neg(mA.y, A.y);
#pragma unroll 1
    for (int i = 64; i > 0; i--) {
        line_double(a, b, c, r, B);
        if (i != 64) fp12_sqr(ret, ret);
        mul_line(&ret, &a, &b, &c);
        uint64_t bit = 1ull << (i - 1);
        if ((NAF_POS | NAF_NEG) & bit) {
            line_add(a, b, c, r, (NAF_POS & bit) ? A : mA, B, r2);
            mul_line(&ret, &a, &b, &c);
        }
    }
    // Q1 = pi(Q), -Q2 = -pi^2(Q) (optate.go:168-209)
    g2a q1, mq2;
    fp2 k;
    fp2_conj(q1.x, A.x);
    fp2_const(k, XI_P1_3_X, XI_P1_3_Y);
    fp2_mul(q1.x, q1.x, k);
    fp2_conj(q1.y, A.y);
    fp2_const(k, XI_P1_2_X, XI_P1_2_Y);
    fp2_mul(q1.y, q1.y, k);
    fp kk;
    fp_const(kk, XI_PSQ1_3);
    fp2_mul_fp(mq2.x, A.x, kk);
    mq2.y = A.y;
    fp2_sqr(r2, q1.y);
    line_add(a, b, c, r, q1, B, r2);
    mul_line(&ret, &a, &b, &c);
    fp2_sqr(r2, mq2.y);
    line_add(a, b, c, r, mq2, B, r2);
    mul_line(&ret, &a, &b, &c);
}

// optate.go:212-261
// base >= 0: the lane is one of the three lanes (base, base+1, base+2) sharing this check (role =
// its index), which run the three exponentiations by u cooperatively
static BN_NI void final_exp(fp12* out, const fp12* in, int role, int base) {
    // every F_p^12 product and cyclotomic squaring goes to the cooperative form on a triple
#define MUL(e, a, b) (base >= 0 ? fp12_mul3(&(e), &(a), &(b), role, base) : fp12_mul(e, a, b))
#define CSQR(e, a) (base >= 0 ? fp12_cyclo_sqr3(&(e), &(a), role, base) : fp12_cyclo_sqr(e, a))
    fp12 t1, t2, fp1, fp2_, fp3, fu, fu2, fu3, y0, y1, y2, y3, y4, y5, y6, t0;
    fp6_neg(t1.x, in->x);
    t1.y = in->y;
    fp12_inv(t2, *in);
    MUL(t1, t1, t2);
    fp12_frob_p2(t2, t1);
    MUL(t1, t1, t2);
    if (base >= 0) {
        fp12_exp_u3(&fu, &t1, role, base);
        fp12_exp_u3(&fu2, &fu, role, base);
        fp12_exp_u3(&fu3, &fu2, role, base);
    } else {
        fp12_exp_u(&fu, &t1);
        fp12_exp_u(&fu2, &fu);
        fp12_exp_u(&fu3, &fu2);
    }
    fp12_frob(fp1, t1);
    fp12_frob_p2(fp2_, t1);
    fp12_frob(fp3, fp2_);
    fp12_frob(y3, fu);
    fp12 fu2p, fu3p;
    fp12_frob(fu2p, fu2);
    fp12_frob(fu3p, fu3);
    fp12_frob_p2(y2, fu2);
    MUL(y0, fp1, fp2_);
    MUL(y0, y0, fp3);
    fp12_conj(y1, t1);
    fp12_conj(y5, fu2);
    fp12_conj(y3, y3);
    MUL(y4, fu, fu2p);
    fp12_conj(y4, y4);
    MUL(y6, fu3, fu3p);
    fp12_conj(y6, y6);
    CSQR(t0, y6);
    MUL(t0, t0, y4);
    MUL(t0, t0, y5);
    MUL(t1, y3, y5);
    MUL(t1, t1, t0);
    MUL(t0, t0, y2);
    CSQR(t1, t1);
    MUL(t1, t1, t0);
    CSQR(t1, t1);
    MUL(t0, t1, y1);
    MUL(t1, t1, y0);
    CSQR(t0, t0);
    MUL(*out, t0, t1);
#undef MUL
#undef CSQR
}

// ---------------------------------------------------------------- SoA helpers
// field element k (of K per item) of item i in a [K*8 words][n] word-major array
GSV_DI void soa_load(fp& r, const uint32_t* __restrict__ base, uint32_t n, uint32_t i, int k) {
#pragma unroll
    for (int w = 0; w < 8; w++) r.v[w] = base[(size_t)(k * 8 + w) * n + i];
}
GSV_DI void soa_store(uint32_t* __restrict__ base, uint32_t n, uint32_t i, int k, const fp& r) {
#pragma unroll
    for (int w = 0; w < 8; w++) base[(size_t)(k * 8 + w) * n + i] = r.v[w];
}
GSV_DI void fp12_load(fp12& e, const uint32_t* base, uint32_t n, uint32_t i) {
    fp* f = (fp*)&e;
#pragma unroll
    for (int k = 0; k < 12; k++) soa_load(f[k], base, n, i, k);
}
GSV_DI void fp12_store(uint32_t* base, uint32_t n, uint32_t i, const fp12& e) {
    const fp* f = (const fp*)&e;
#pragma unroll
    for (int k = 0; k < 12; k++) soa_store(base, n, i, k, f[k]);
}

// gfP.Unmarshal (gfp.go:61-78) + montEncode: big-endian bytes -> limbs; false if >= p
GSV_DI bool fp_unmarshal(fp& r, const uint8_t* p) {
    uint32_t x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint8_t* q = p + 28 - 4 * i;
        x[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
    }
    bool ok = !fp_geq_p(x);
    fp t, r2;
#pragma unroll
    for (int i = 0; i < 8; i++) t.v[i] = ok ? x[i] : 0u;
    fp_const(r2, BN_R2);
    fp_mul_c(r, t, r2);
    return ok;
}

// ---------------------------------------------------------------- kernels
enum : uint8_t { PS_OK = 0, PS_SKIP = 1, PS_BAD = 2 };

// Two waves per SIMD (a 256-register budget: the subgroup loop spills ~160 VGPRs to scratch) beat
// one wave with everything in registers: simple VALU ops issue at twice the rate with a second
// wave (profiles/r01_microbench_lat.txt), and a full batch has 4 waves of pairs per SIMD.
// Measured 7.8 -> 6.4 ms per 262,144 pairs.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_bn_prepare(const uint8_t* __restrict__ in,
                                                   const uint64_t* __restrict__ pair_src,
                                                   uint32_t npairs, uint8_t* __restrict__ pstat,
                                                   uint32_t* __restrict__ pts /* [48 words][npairs] */) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npairs) return;
    const uint8_t* s = in + pair_src[i];
    g1a P;
    g2a Q;
    bool ok = fp_unmarshal(P.x, s);
    ok = fp_unmarshal(P.y, s + 32) && ok;
    ok = fp_unmarshal(Q.x.x, s + 64) && ok;  // imaginary part first (bn256.go:267-278)
    ok = fp_unmarshal(Q.x.y, s + 96) && ok;
    ok = fp_unmarshal(Q.y.x, s + 128) && ok;
    ok = fp_unmarshal(Q.y.y, s + 160) && ok;
    bool inf1 = fp_is_zero(P.x) && fp_is_zero(P.y);
    bool inf2 = fp2_is_zero(Q.x) && fp2_is_zero(Q.y);
    if (ok && !inf1) {  // curve.go:39-52: y^2 == x^3 + 3
        fp y2, x3, b;
        fp_mul_c(y2, P.y, P.y);
        fp_mul_c(x3, P.x, P.x);
        fp_mul_c(x3, x3, P.x);
        fp_const(b, BN_THREE);
        fp_add(x3, x3, b);
        ok = fp_eq(y2, x3);
    }
    if (ok && !inf2) ok = g2_in_subgroup(&Q);
    pstat[i] = !ok ? PS_BAD : (inf1 || inf2) ? PS_SKIP : PS_OK;
    soa_store(pts, npairs, i, 0, P.x);
    soa_store(pts, npairs, i, 1, P.y);
    soa_store(pts, npairs, i, 2, Q.x.x);
    soa_store(pts, npairs, i, 3, Q.x.y);
    soa_store(pts, npairs, i, 4, Q.y.x);
    soa_store(pts, npairs, i, 5, Q.y.y);
}

// ---- per-check multi-Miller loop.  The product of a check's Miller values equals one loop that
// squares the shared accumulator once per step and multiplies in every pair's lines
// (prod f_i^2 l_i = (prod f_i)^2 prod l_i, exact in F_p^12), so a check of k pairs spends one
// F_p^12 squaring per step instead of k; the verdict is the reference's bit for bit.  One lane per
// check; pair j of a check lives at slot-major index pidx[first + j] (the j-th pairs of all checks
// contiguous), so the per-pair twist point R and the decoded points load/store coalesced.
enum : uint8_t { CS_OK = 0, CS_BAD = 1, CS_ONE = 2 };  // CS_ONE: no finite pair -> product is 1

GSV_DI void g2j_load(g2j& r, const uint32_t* __restrict__ base, uint32_t n, uint32_t i) {
    soa_load(r.x.x, base, n, i, 0);
    soa_load(r.x.y, base, n, i, 1);
    soa_load(r.y.x, base, n, i, 2);
    soa_load(r.y.y, base, n, i, 3);
    soa_load(r.z.x, base, n, i, 4);
    soa_load(r.z.y, base, n, i, 5);
    soa_load(r.t.x, base, n, i, 6);
    soa_load(r.t.y, base, n, i, 7);
}
GSV_DI void g2j_store(uint32_t* __restrict__ base, uint32_t n, uint32_t i, const g2j& r) {
    soa_store(base, n, i, 0, r.x.x);
    soa_store(base, n, i, 1, r.x.y);
    soa_store(base, n, i, 2, r.y.x);
    soa_store(base, n, i, 3, r.y.y);
    soa_store(base, n, i, 4, r.z.x);
    soa_store(base, n, i, 5, r.z.y);
    soa_store(base, n, i, 6, r.t.x);
    soa_store(base, n, i, 7, r.t.y);
}
GSV_DI void pts_load(g1a& P, g2a& Q, const uint32_t* __restrict__ pts, uint32_t n, uint32_t j) {
    soa_load(P.x, pts, n, j, 0);
    soa_load(P.y, pts, n, j, 1);
    soa_load(Q.x.x, pts, n, j, 2);
    soa_load(Q.x.y, pts, n, j, 3);
    soa_load(Q.y.x, pts, n, j, 4);
    soa_load(Q.y.y, pts, n, j, 5);
}

// A lane runs the loop over a group of <= k of its check's pairs (k = 4 covers a whole 4-pair check;
// smaller k when the batch is too small to give every SIMD work — the host's choice), and k_bn_final
// multiplies a check's lane values: the same exact product, so the same verdict.
__global__ __launch_bounds__(64) void k_bn_miller(const uint32_t* __restrict__ lane_first, uint32_t nlanes,
                                                  const uint32_t* __restrict__ pidx, const uint8_t* __restrict__ pstat,
                                                  const uint32_t* __restrict__ pts, uint32_t npairs,
                                                  uint32_t* __restrict__ rs /* [64 words][npairs] */,
                                                  uint8_t* __restrict__ cstat,
                                                  uint32_t* __restrict__ fv /* [96 words][nlanes] */) {
    uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nlanes) return;
    uint32_t b = lane_first[c], e = lane_first[c + 1];
    bool bad = false, any = false;
    for (uint32_t q = b; q < e; q++) {
        uint32_t j = pidx[q];
        uint8_t st = pstat[j];
        bad = bad || st == PS_BAD;
        if (st != PS_OK) continue;
        any = true;
        g1a P;
        g2a Q;
        pts_load(P, Q, pts, npairs, j);
        g2j r;
        r.x = Q.x;
        r.y = Q.y;
        fp2_one(r.z);
        fp2_one(r.t);
        g2j_store(rs, npairs, j, r);
    }
    cstat[c] = bad ? CS_BAD : any ? CS_OK : CS_ONE;
    if (bad || !any) return;
    fp12 f;
    fp12_one(f);
    fp2 la, lb, lc;
    // The loop body is inlined down to the out-of-line F_p product (whose 28 VGPRs are all it
    // clobbers), so f, R and the line stay in registers: no per-lane scratch on the hot path.  A
    // pair's doubling step and (on NAF digits) its addition step share one inlined mul_line.
#pragma unroll 1
    for (int i = 64; i > 0; i--) {
        if (i != 64) fp12_sqr_i(f, f);
        uint64_t bit = 1ull << (i - 1);
        bool add = ((NAF_POS | NAF_NEG) & bit) != 0;
#pragma unroll 1
        for (uint32_t q = b; q < e; q++) {
            uint32_t j = pidx[q];
            if (pstat[j] != PS_OK) continue;
#pragma unroll 1
            for (int k = 0; k < (add ? 2 : 1); k++) {
                // R and P are (re)loaded per line and R stored before the line product, so only
                // f and the line are live across mul_line (the R reload hits L2)
                g1a P;
                soa_load(P.x, pts, npairs, j, 0);
                soa_load(P.y, pts, npairs, j, 1);
                g2j r;
                g2j_load(r, rs, npairs, j);
                if (k == 0) {
                    line_double_i(la, lb, lc, r, P);
                } else {  // Q is only needed on the NAF's nonzero digits
                    g2a Q;
                    soa_load(Q.x.x, pts, npairs, j, 2);
                    soa_load(Q.x.y, pts, npairs, j, 3);
                    soa_load(Q.y.x, pts, npairs, j, 4);
                    soa_load(Q.y.y, pts, npairs, j, 5);
                    fp2 r2;
                    fp2_sqr(r2, Q.y);
                    if (NAF_NEG & bit) fp2_neg(Q.y, Q.y);
                    line_add_i(la, lb, lc, r, Q, P, r2);
                }
                g2j_store(rs, npairs, j, r);
                mul_line_i(f, la, lb, lc);
            }
        }
    }
    // Q1 = pi(Q), -Q2 = -pi^2(Q) (optate.go:168-209), per pair
    for (uint32_t q = b; q < e; q++) {
        uint32_t j = pidx[q];
        if (pstat[j] != PS_OK) continue;
        g1a P;
        g2a A;
        pts_load(P, A, pts, npairs, j);
        g2j r;
        g2j_load(r, rs, npairs, j);
        g2a q1, mq2;
        fp2 k, r2;
        fp2_conj(q1.x, A.x);
        fp2_const(k, XI_P1_3_X, XI_P1_3_Y);
        fp2_mul(q1.x, q1.x, k);
        fp2_conj(q1.y, A.y);
        fp2_const(k, XI_P1_2_X, XI_P1_2_Y);
        fp2_mul(q1.y, q1.y, k);
        fp kk;
        fp_const(kk, XI_PSQ1_3);
        fp2_mul_fp(mq2.x, A.x, kk);
        mq2.y = A.y;
        fp2_sqr(r2, q1.y);
        line_add(la, lb, lc, r, q1, P, r2);
        mul_line(&f, &la, &lb, &lc);
        fp2_sqr(r2, mq2.y);
        line_add(la, lb, lc, r, mq2, P, r2);
        mul_line(&f, &la, &lb, &lc);
    }
    fp12_store(fv, nlanes, c, f);
}

// role/base as final_exp: the verdict is written by role 0
// cbad[c] != 0: the check's input length is not a multiple of 192 (errBadPairingInput,
// core/vm/contracts.go:336-338); it has no pairs
GSV_DI void final_check(uint32_t c, const uint32_t* __restrict__ check_lane, const uint8_t* __restrict__ cbad,
                        const uint8_t* __restrict__ lstat, const uint32_t* __restrict__ fv, uint32_t nlanes,
                        uint8_t* __restrict__ verdict, int role, int base) {
    uint32_t l0 = check_lane[c], l1 = check_lane[c + 1];
    bool bad = cbad[c] != 0;
    for (uint32_t l = l0; l < l1; l++) bad = bad || lstat[l] == CS_BAD;
    if (bad) {
        if (role == 0) verdict[c] = GSV_PAIRING_BAD_INPUT;
        return;
    }
    // product of the check's lane values; finalExponentiation(1) == 1 when no pair is finite
    fp12 acc;
    bool any = false;
    for (uint32_t l = l0; l < l1; l++) {
        if (lstat[l] != CS_OK) continue;
        if (!any) {
            fp12_load(acc, fv, nlanes, l);
            any = true;
        } else {
            fp12 t;
            fp12_load(t, fv, nlanes, l);
            fp12_mul(acc, acc, t);
        }
    }
    if (!any) fp12_one(acc);
    fp12 r;
    final_exp(&r, &acc, role, base);
    if (role == 0) verdict[c] = fp12_is_one(r) ? GSV_PAIRING_TRUE : GSV_PAIRING_FALSE;
}

__global__ __launch_bounds__(64) void k_bn_final(const uint32_t* __restrict__ check_lane, uint32_t nchecks,
                                                 const uint8_t* __restrict__ cbad, const uint8_t* __restrict__ lstat,
                                                 const uint32_t* __restrict__ fv, uint32_t nlanes,
                                                 uint8_t* __restrict__ verdict) {
    uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchecks) return;
    final_check(c, check_lane, cbad, lstat, fv, nlanes, verdict, 0, -1);
}
// three lanes per check (21 triples per wave, lane 63 idle); a triple's lanes take the same path
constexpr uint32_t FINAL3_PER_WAVE = 21;
__global__ __launch_bounds__(64) void k_bn_final3(const uint32_t* __restrict__ check_lane, uint32_t nchecks,
                                                  const uint8_t* __restrict__ cbad, const uint8_t* __restrict__ lstat,
                                                  const uint32_t* __restrict__ fv, uint32_t nlanes,
                                                  uint8_t* __restrict__ verdict) {
    int t = threadIdx.x / 3, role = threadIdx.x - 3 * t;
    uint32_t c = blockIdx.x * FINAL3_PER_WAVE + t;
    if (t >= (int)FINAL3_PER_WAVE || c >= nchecks) return;
    final_check(c, check_lane, cbad, lstat, fv, nlanes, verdict, role, 3 * t);
}


// ---------------------------------------------------------------- synthetic workload (bench data)
// Not on the validation path.  Check i = e(aP, bQ) e(-bP, aQ) e(cP, dQ) e(-dP, cQ) == 1 with
// a, b, c, d = Keccak-256(le64(seed) || le64(i) || tag) truncated to 253 bits (nonzero), P, Q the
// G1 / G2 generators (curve.go:16-21, twist.go:20-32).  Every 8th check (i % 8 == 7) uses
// -(d+1)P (false); every 1024th (i % 1024 == 1023) also corrupts a coordinate to p (bad input).
__device__ constexpr uint32_t TWIST_GEN_XX[8] = {0xa84c6140u, 0xafb4737du, 0x5802d8c4u, 0x6043dd5au,
                                                 0x52a02f86u, 0x09e950fcu, 0x3aea7b6bu, 0x14fef083u};
__device__ constexpr uint32_t TWIST_GEN_XY[8] = {0x02bc2026u, 0x8e83b5d1u, 0x497b0172u, 0xdceb1935u,
                                                 0x97811adfu, 0xfbb82647u, 0xaf96503bu, 0x19573841u};
__device__ constexpr uint32_t TWIST_GEN_YX[8] = {0xc71856eeu, 0x64095b56u, 0x327d3cbbu, 0xdc57f922u,
                                                 0x33351076u, 0x55f935beu, 0x93fd6482u, 0x0da4a0e6u};
__device__ constexpr uint32_t TWIST_GEN_YY[8] = {0x886be9f6u, 0x619dfa9du, 0xf59e9b78u, 0xfe7fd297u,
                                                 0x231b7dfeu, 0xff9e1a62u, 0xae9e4206u, 0x28fd7eebu};
__device__ constexpr uint32_t BN_TWO[8] = {0x8b1e1b3au, 0xa6ba871bu, 0xeb8e167bu, 0x14f1d651u,
                                           0xf0f28c58u, 0xccdd46deu, 0x340fbe5eu, 0x1c14ef83u};

struct g1j { fp x, y, z; };
// curve.go:143-172 dbl-2009-l
static BN_NI void g1_double_p(g1j* pc, const g1j* pa) {
    const g1j a = *pa;
    fp A, B, C, t, t2, d, e, f;
    fp_mul_c(A, a.x, a.x);
    fp_mul_c(B, a.y, a.y);
    fp_mul_c(C, B, B);
    fp_add(t, a.x, B);
    fp_mul_c(t2, t, t);
    fp_sub(t, t2, A);
    fp_sub(t2, t, C);
    fp_add(d, t2, t2);
    fp_add(t, A, A);
    fp_add(e, t, A);
    fp_mul_c(f, e, e);
    g1j r;
    fp_add(t, d, d);
    fp_sub(r.x, f, t);
    fp_add(t, C, C);
    fp_add(t2, t, t);
    fp_add(t, t2, t2);
    fp_sub(r.y, d, r.x);
    fp_mul_c(t2, e, r.y);
    fp_sub(r.y, t2, t);
    fp_mul_c(t, a.y, a.z);
    fp_add(r.z, t, t);
    *pc = r;
}
// curve.go:63-141 add-2007-bl
static BN_NI void g1_add_p(g1j* pc, const g1j* pa, const g1j* pb) {
    const g1j a = *pa, b = *pb;
    if (fp_is_zero(a.z)) { *pc = b; return; }
    if (fp_is_zero(b.z)) { *pc = a; return; }
    fp z12, z22, u1, u2, t, s1, s2, h, i, j, r, v, t4, t6;
    fp_mul_c(z12, a.z, a.z);
    fp_mul_c(z22, b.z, b.z);
    fp_mul_c(u1, a.x, z22);
    fp_mul_c(u2, b.x, z12);
    fp_mul_c(t, b.z, z22);
    fp_mul_c(s1, a.y, t);
    fp_mul_c(t, a.z, z12);
    fp_mul_c(s2, b.y, t);
    fp_sub(h, u2, u1);
    bool xeq = fp_is_zero(h);
    fp_add(t, h, h);
    fp_mul_c(i, t, t);
    fp_mul_c(j, h, i);
    fp_sub(t, s2, s1);
    bool yeq = fp_is_zero(t);
    if (xeq && yeq) { g1_double_p(pc, pa); return; }
    fp_add(r, t, t);
    fp_mul_c(v, u1, i);
    g1j o;
    fp_mul_c(t4, r, r);
    fp_add(t, v, v);
    fp_sub(t6, t4, j);
    fp_sub(o.x, t6, t);
    fp_sub(t, v, o.x);
    fp_mul_c(t4, s1, j);
    fp_add(t6, t4, t4);
    fp_mul_c(t4, r, t);
    fp_sub(o.y, t4, t6);
    fp_add(t, a.z, b.z);
    fp_mul_c(t4, t, t);
    fp_sub(t, t4, z12);
    fp_sub(t4, t, z22);
    fp_mul_c(o.z, t4, h);
    *pc = o;
}
// k * P (k < 2^253 as 8 limbs, nonzero) -> affine Montgomery coordinates
GSV_DI void g1_mul_gen(fp& ox, fp& oy, const uint32_t k[8]) {
    g1j base, sum;
    fp_const(base.x, BN_ONE);
    fp_const(base.y, BN_TWO);
    fp_const(base.z, BN_ONE);
    fp_zero(sum.x);
    fp_const(sum.y, BN_ONE);
    fp_zero(sum.z);
#pragma unroll 1
    for (int b = 252; b >= 0; b--) {
        g1j t;
        g1_double_p(&t, &sum);
        if ((k[b >> 5] >> (b & 31)) & 1u) g1_add_p(&sum, &t, &base);
        else sum = t;
    }
    fp zi, zi2, zi3;
    fp_inv(zi, sum.z);
    fp_mul_c(zi2, zi, zi);
    fp_mul_c(zi3, zi2, zi);
    fp_mul_c(ox, sum.x, zi2);
    fp_mul_c(oy, sum.y, zi3);
}
GSV_DI void g2_mul_gen(g2a& o, const uint32_t k[8]) {
    g2j base, sum;
    fp2_const(base.x, TWIST_GEN_XX, TWIST_GEN_XY);
    fp2_const(base.y, TWIST_GEN_YX, TWIST_GEN_YY);
    fp2_one(base.z);
    fp2_one(base.t);
    fp2_zero(sum.x);
    fp2_one(sum.y);
    fp2_zero(sum.z);
    fp2_zero(sum.t);
#pragma unroll 1
    for (int b = 252; b >= 0; b--) {
        g2j t;
        g2_double(t, sum);
        if ((k[b >> 5] >> (b & 31)) & 1u) g2_add(sum, t, base);
        else sum = t;
    }
    fp2 zi, zi2, zi3;
    fp2_inv(zi, sum.z);
    fp2_sqr(zi2, zi);
    fp2_mul(zi3, zi2, zi);
    fp2_mul(o.x, sum.x, zi2);
    fp2_mul(o.y, sum.y, zi3);
}
// montDecode + big-endian marshal (gfp.go:51-59)
GSV_DI void fp_marshal(uint8_t* out, const fp& a) {
    fp one, t;
    fp_zero(one);
    one.v[0] = 1;
    fp_mul_c(t, a, one);
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint32_t w = t.v[7 - i];
        out[4 * i] = (uint8_t)(w >> 24);
        out[4 * i + 1] = (uint8_t)(w >> 16);
        out[4 * i + 2] = (uint8_t)(w >> 8);
        out[4 * i + 3] = (uint8_t)w;
    }
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
// one (G1, G2) pair of the check: lane (check, j) for j = 0..3
__global__ __launch_bounds__(64) void k_bn_synth(uint64_t seed, uint32_t nchecks, uint8_t* __restrict__ out,
                                                 uint8_t* __restrict__ expect) {
    uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= nchecks * 4u) return;
    uint32_t c = id >> 2, j = id & 3u;
    uint32_t s1[8], s2[8];
    // pair j: (x P, y Q) with (x, y) = (a, b), (-b, a), (c, d), (-d', c)
    const uint32_t tags[4] = {0x61u, 0x62u, 0x63u, 0x64u};  // "a" "b" "c" "d"
    uint32_t tx = (j == 0) ? tags[0] : (j == 1) ? tags[1] : (j == 2) ? tags[2] : tags[3];
    uint32_t ty = (j == 0) ? tags[1] : (j == 1) ? tags[0] : (j == 2) ? tags[3] : tags[2];
    synth_scalar(s1, seed, c, tx);
    synth_scalar(s2, seed, c, ty);
    bool is_false = (c % 8u) == 7u, is_bad = (c % 1024u) == 1023u;
    if (j == 3 && is_false) {  // d + 1 (no overflow: d < 2^253)
        uint32_t cy = 1;
#pragma unroll
        for (int w = 0; w < 8; w++) s1[w] = add_c(s1[w], 0u, cy);
    }
    fp px, py;
    g1_mul_gen(px, py, s1);
    if (j & 1u) fp_neg(py, py);  // -xP
    g2a q;
    g2_mul_gen(q, s2);
    uint8_t* o = out + (size_t)c * 768 + j * 192;
    fp_marshal(o, px);
    fp_marshal(o + 32, py);
    fp_marshal(o + 64, q.x.x);
    fp_marshal(o + 96, q.x.y);
    fp_marshal(o + 128, q.y.x);
    fp_marshal(o + 160, q.y.y);
    if (j == 2 && is_bad) {  // coordinate == p: bn256 "coordinate equals modulus"
#pragma unroll
        for (int i = 0; i < 8; i++) {
            uint32_t w = BN_P[7 - i];
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
                                uint8_t* d_pstat, uint32_t* d_pts, uint32_t* d_rs, uint8_t* d_lstat, uint32_t* d_fv,
                                uint8_t* d_verdict, bool final3, hipStream_t st, void (*timer_begin)(void*, int),
                                void (*timer_end)(void*, int), void* tctx) {
    if (npairs) {
        if (timer_begin) timer_begin(tctx, GSV_K_BN_PREPARE);
        hipLaunchKernelGGL(bn::k_bn_prepare, dim3((npairs + 63) / 64), dim3(64), 0, st, d_in, d_pair_src, npairs,
                           d_pstat, d_pts);
        if (timer_end) timer_end(tctx, GSV_K_BN_PREPARE);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (nchecks) {
        if (timer_begin) timer_begin(tctx, GSV_K_PAIRING);
        hipLaunchKernelGGL(bn::k_bn_miller, dim3((nlanes + 63) / 64), dim3(64), 0, st, d_lane_first, nlanes,
                           d_pidx, d_pstat, d_pts, npairs, d_rs, d_lstat, d_fv);
        if (timer_end) timer_end(tctx, GSV_K_PAIRING);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        if (timer_begin) timer_begin(tctx, GSV_K_BN_FINAL);
        if (final3)
            hipLaunchKernelGGL(bn::k_bn_final3, dim3((nchecks + bn::FINAL3_PER_WAVE - 1) / bn::FINAL3_PER_WAVE),
                               dim3(64), 0, st, d_check_lane, nchecks, d_cbad, d_lstat, d_fv, nlanes, d_verdict);
        else
            hipLaunchKernelGGL(bn::k_bn_final, dim3((nchecks + 63) / 64), dim3(64), 0, st, d_check_lane, nchecks,
                               d_cbad, d_lstat, d_fv, nlanes, d_verdict);
        if (timer_end) timer_end(tctx, GSV_K_BN_FINAL);
    }
    return hipGetLastError();
}

}  // namespace gsv

GSV_OPCOUNT_READER(bn256)
